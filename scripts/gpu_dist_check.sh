#!/bin/bash
# 2 ranks sharing the box's single GPU (gloo over GPU tensors): exercises the
# multi-rank bench paths (sharding, health collectives, DP trainer, JSON
# contract) on real device memory.  The 8-GPU RCCL run is the driver's.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export FOREMAST_DIST_BACKEND=gloo
for cfg in canary lstm multicluster; do
  extra=""; c=$cfg
  if [ $cfg = multicluster ]; then extra="--multi-cluster"; c=canary; fi
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
    --master-port=29531 bench.py --gpus 2 --steps 5 --warmup 2 --series 20000 --config $c $extra \
    > gpurun_out/dist_$cfg.log 2>&1
  rc=$?
  echo "== dist $cfg rc=$rc"
  grep '^{' gpurun_out/dist_$cfg.log || tail -20 gpurun_out/dist_$cfg.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
