"""One process per GPU over RCCL/xGMI: sharding, health aggregation, DP."""
