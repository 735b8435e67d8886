"""The RCCL path on one GPU.

The driver's scaling run launches ``bench.py --gpus N`` on an 8-GPU node, one
rank per GPU over RCCL (``nccl``).  One GPU cannot host two RCCL ranks, so
these tests run the SAME code in a 1-rank ``nccl`` group with
``FOREMAST_FORCE_COLLECTIVES=1``: every per-tick collective is issued exactly
as with N ranks — the canary tick's fused health all-gather (int32 records
the scoring kernel wrote in place), the multi-cluster baseline all-to-all
(int64 counts, ids, float32 windows with split sizes), the LSTM trainer's
gradient all-reduce and parameter broadcast, and the per-app all-reduce +
int8 verdict all-gather of the non-fused aggregator — and the results must
equal the collective-free run.  The same on CPU with gloo keeps the forced
mode itself covered in the CPU suite.
"""

import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench(args, force: bool, launcher: bool, cpu: bool):
    env = dict(os.environ, OMP_NUM_THREADS="4", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    if force:
        env["FOREMAST_FORCE_COLLECTIVES"] = "1"
    else:
        env.pop("FOREMAST_FORCE_COLLECTIVES", None)
    pre = ([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
            "--master-addr=127.0.0.1", f"--master-port={_port()}"] if launcher else [sys.executable])
    cmd = pre + [os.path.join(ROOT, "bench.py"), "--gpus", "1"] + args + (["--cpu"] if cpu else [])
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 0, (out.stdout[-1000:] + out.stderr[-3000:])
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


CANARY = ["--steps", "3", "--warmup", "2", "--series", "5000", "--ring", "2880", "--anomaly-frac", "0.02"]
CASES = {
    "canary": (CANARY, "1 fused all_gather"),
    "multicluster": (CANARY + ["--multi-cluster"], "1 fused all_gather"),
    "lstm": (["--config", "lstm", "--steps", "3", "--warmup", "2", "--series", "4096", "--ring", "2880",
              "--lstm-train-batch", "256", "--lstm-pretrain", "5", "--lstm-train-every", "1"],
             "all_reduce + all_gather"),
}


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(CASES))
def test_rccl_one_rank_collectives_match_local_tick(case):
    args, coll = CASES[case]
    ref = _bench(args, force=False, launcher=False, cpu=False)
    got = _bench(args, force=True, launcher=True, cpu=False)
    assert got["n_gpus"] == 1 and got["config"]["parallelism"] == "dp1"
    if case != "lstm":
        assert ref["config"]["health_collectives"] == "none"
        assert got["config"]["health_collectives"].startswith(coll)
        assert got["config"]["multi_cluster"] == (case == "multicluster")
        assert got["health"] == ref["health"] and got["detection"] == ref["detection"]
        # the RCCL all-gather and the health table's copy back are nodes of the tick's HIP
        # graph: one replay per tick, no host-launched collective (no host-side timing either)
        assert got["config"]["health_tail_in_graph"] is True
        assert got["config"]["health_collectives"].endswith("(captured in the tick graph)")
        return
    else:
        # training is stochastic across processes only through the all-reduce's
        # arithmetic (a 1-rank sum is exact), so the verdict counts agree too
        assert got["health"]["series_scored_last_tick"] == ref["health"]["series_scored_last_tick"]
        assert got["detection"]["recall"] == ref["detection"]["recall"]
    assert got["collective_ms_p50"] is not None and got["collective_ms_p50"] > 0


def test_forced_collectives_gloo_one_rank_cpu():
    """The forced mode on CPU (gloo, 1 rank): same health table as the plain run."""
    args = ["--steps", "2", "--warmup", "1", "--series", "200", "--ring", "480", "--season", "48",
            "--anomaly-frac", "0.05"]
    ref = _bench(args, force=False, launcher=False, cpu=True)
    got = _bench(args, force=True, launcher=True, cpu=True)
    assert got["config"]["health_collectives"] == "1 fused all_gather"
    assert got["health"] == ref["health"] and got["detection"] == ref["detection"]


def _reform(cpu: bool) -> dict:
    env = dict(os.environ, OMP_NUM_THREADS="4", HSA_ENABLE_IPC_MODE_LEGACY="0", FOREMAST_HEARTBEAT_S="0.5")
    for k in ("WORLD_SIZE", "RANK", "MASTER_PORT", "FOREMAST_NODE_STORE"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "tests", "helpers", "reform_rank.py")] + (["--cpu"] if cpu else [])
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=180, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-1000:] + out.stderr[-3000:]
    lines = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[-1])


def _check_reform(got: dict, backend: str) -> None:
    assert got["backend"] == backend and got["backend_after"] == backend
    assert got["injected"] == 1 and got["reforms"] == 1 and got["generation"] == 1 and got["new_group"]
    gens = [t["generation"] for t in got["ticks"]]
    assert gens == [0, 0, 1, 1, 1], gens          # the failed tick completed on the new communicator
    assert all(t["apps"] == t["want_apps"] and t["collectives"] for t in got["ticks"])
    assert got["grads_ok"] and got["allreduce_ok"] and got["flags"] == [1.0, 5.0]


@pytest.mark.gpu
def test_rccl_abort_and_reform_in_process():
    """ElasticWorld on RCCL: a collective deadline inside run_tick aborts the
    communicator, the group is re-formed (generation 1) in the same process, and
    the node exchange and a DP gradient all-reduce run on the new communicator."""
    _check_reform(_reform(cpu=False), "nccl")


def test_gloo_abort_and_reform_in_process():
    _check_reform(_reform(cpu=True), "gloo")


def _node_bench(gpus: int, cpu: bool, force: bool = False, extra=()) -> dict:
    env = dict(os.environ, OMP_NUM_THREADS="2", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "MASTER_PORT"):
        env.pop(k, None)
    if force:
        env["FOREMAST_FORCE_COLLECTIVES"] = "1"
    else:
        env.pop("FOREMAST_FORCE_COLLECTIVES", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--config", "node",
           "--arrival-per-tick", "8", "--steps", "4", "--warmup", "11"] + list(extra) + (["--cpu"] if cpu else [])
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-1000:] + out.stderr[-3000:]
    lines = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.slow
def test_node_bench_two_ranks_runs_the_deployed_exchange_cpu():
    """``bench.py --gpus 2 --config node`` (arrivals) under torch.distributed.run: the
    ranks join an ElasticWorld on the launcher's store and exchange roster deltas, as a
    deployed node does; the record says so and counts every rank's jobs."""
    got = _node_bench(2, cpu=True)
    ex = got["node"]["exchange"]
    assert got["n_gpus"] == 2 and ex["ranks"] == 2 and ex["path"].startswith("ElasticWorld")
    assert ex["generation"] == 0 and ex["samples"] == 4 and ex["exchange_ms_p50_p99_max"][0] is not None
    det = got["detection"]
    assert det["ranks"] == 2 and det["fn"] == 0 and det["jobs"] > 0


@pytest.mark.gpu
def test_node_bench_forced_rccl_exchange_one_gpu():
    """The node bench's deployed exchange on RCCL (a 1-member ElasticWorld with forced
    collectives): roster deltas through the store, health all-gather on the GPU."""
    got = _node_bench(1, cpu=False, force=True)
    ex = got["node"]["exchange"]
    assert ex["path"].startswith("ElasticWorld") and ex["generation"] == 0
    assert got["detection"]["fn"] == 0


def _mc_bench(gpus: int, cpu: bool, multi: bool, force: bool = False) -> dict:
    """The burst node bench (every job admitted at the first tick) with or without the
    config-4 layout (every other app's baseline pods in another cluster)."""
    env = dict(os.environ, OMP_NUM_THREADS="2", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "MASTER_PORT"):
        env.pop(k, None)
    if force:
        env["FOREMAST_FORCE_COLLECTIVES"] = "1"
    else:
        env.pop("FOREMAST_FORCE_COLLECTIVES", None)
    size = ["--series", "500", "--ring", "2880"] if cpu else ["--series", "20000"]
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--config", "node",
           "--steps", "3", "--warmup", "1"] + size + (["--multi-cluster"] if multi else []) + (["--cpu"] if cpu else [])
    if gpus == 1 and force:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
               "--master-addr=127.0.0.1", f"--master-port={_port()}"] + cmd[1:]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-1000:] + out.stderr[-3000:]
    lines = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


def _check_mc(single: dict, multi: dict) -> dict:
    mc = multi["config"]["multi_cluster"]
    assert mc and mc["clusters"] >= 2 and mc["exchanges_with_requests"] >= 1
    assert mc["values_moved"] > 0 and mc["admission"]["affine_requests"] > 0
    # the baseline windows crossed ranks bit for bit: the same verdicts as the one-cluster run
    assert multi["detection"] == single["detection"] and multi["health"] == single["health"]
    # after admission the exchange carries nothing but the request-count gather
    assert all(b.get("affine_bytes", 0) == 0 for b in multi["node"]["tick_breakdown_ms"])
    return mc


@pytest.mark.slow
def test_node_multi_cluster_two_gloo_ranks_cpu():
    """Config 4 through the product at 2 ranks (gloo): each rank's odd apps have their
    baseline pods in the other rank's cluster; those windows are decoded by that rank and
    delivered by the rollout engine's all_to_all at admission."""
    _check_mc(_mc_bench(2, cpu=True, multi=False), _mc_bench(2, cpu=True, multi=True))


@pytest.mark.gpu
def test_node_multi_cluster_forced_rccl_one_gpu():
    """The same exchange over RCCL on one GPU (forced collectives, 1-member world; the rank
    serves the other cluster itself through the collective path): identical verdicts to
    the one-cluster run, values delivered device to device."""
    mc = _check_mc(_mc_bench(1, cpu=False, multi=False, force=True), _mc_bench(1, cpu=False, multi=True, force=True))
    assert mc["admission"]["affine_bytes"] > 0


@pytest.mark.gpu
def test_double_buffered_graph_input_matches_single_buffer():
    """The canary's graph ticks with the next tick's input copied during the current one
    (two input buffers, one captured graph each) and a spin-wait give the same health
    table and detection as one buffer copied at the start of each tick."""
    args = CANARY + ["--steps", "6"]
    ref = _bench(args + ["--no-graph-prefetch"], force=False, launcher=False, cpu=False)
    got = _bench(args + ["--spin-wait"], force=False, launcher=False, cpu=False)
    assert got["config"]["input_prefetch"] and not ref["config"]["input_prefetch"]
    assert got["config"]["hip_graph"] and ref["config"]["hip_graph"]
    assert got["health"] == ref["health"] and got["detection"] == ref["detection"]


@pytest.mark.gpu
def test_doorbell_graph_ticks_match_plain_graph_ticks():
    """--doorbell: tick k+1's graph is enqueued while tick k runs and waits on the device for
    the host's pinned counter; every wait is rung (no timeout) and the health table and
    detection equal the plain graph ticks'."""
    args = CANARY + ["--steps", "6"]
    ref = _bench(args + ["--no-doorbell"], force=False, launcher=False, cpu=False)
    got = _bench(args + ["--doorbell"], force=False, launcher=False, cpu=False)
    assert got["config"]["doorbell"] and not ref["config"]["doorbell"]
    assert got["config"]["hip_graph"] and got["config"]["doorbell_timeouts"] == 0
    assert got["health"] == ref["health"] and got["detection"] == ref["detection"]
