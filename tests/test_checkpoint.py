"""Checkpoint / resume: a restored shard continues exactly like
the uninterrupted one."""

import pytest
import torch

from foremast_amd.brain import checkpoint as ck
from foremast_amd.brain.engine import ShardSpec, StreamingShard, synthetic_history
from foremast_amd.utils.config import BrainConfig


def _cfg():
    c = BrainConfig()
    c.min_historical_points = 0
    return c


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_streaming_shard_snapshot_resumes_bit_exact(tmp_path, dev):
    n, R, m, P, W = 20, 480, 48, 3, 4
    if dev == "cuda":
        n, R, m = 40, 2880, 1440  # the HIP Holt-Winters path (two seasons)
    hist = synthetic_history(n, R + 20, m, dev, seed=5)
    a = StreamingShard(ShardSpec(n_series=n, ring_len=R, season=m, pods=P, window=W, n_apps=4), _cfg(), dev,
                       app_id=(torch.arange(n, device=dev) % 4).int(), threshold=torch.full((n,), 3.0, device=dev))
    a.load_history(hist[:, :R - 30])  # ring not full yet: head/length both restored
    a.set_baseline(hist[:, R - W:R].repeat(1, P))
    step = lambda s, k: s.ingest_tick(hist[:, R + k:R + k + 1].repeat(1, P) * (1 + 0.5 * (k == 8)))
    for k in range(6):
        step(a, k)
        a.score()
    path = str(tmp_path / "shard.safetensors")
    ck.save_streaming_shard(a, path, extra={"rank": 0})
    b = ck.load_streaming_shard(path, _cfg(), dev)
    assert b.checkpoint_extra == {"rank": 0}
    assert torch.equal(b.fitted["sigma"], a.out["sigma"]) and torch.equal(b.fitted["best"], a.out["best"])
    for k in range(6, 12):
        step(a, k)
        step(b, k)
        oa, ob = a.score(), b.score()
        for key in ("verdict", "sigma", "level", "forecast", "count"):
            assert torch.equal(oa[key], ob[key]), (k, key)
        assert torch.equal(a.app_stats, b.app_stats)
    assert a.hist.head == b.hist.head and a.hist.length == b.hist.length
    torch.testing.assert_close(a.hist.data, b.hist.data, rtol=0, atol=0, equal_nan=True)


def test_lstm_shard_snapshot_resumes_training(tmp_path):
    from foremast_amd.brain.lstm_engine import LstmShard
    n, R, F = 16, 200, 2
    a = LstmShard(n, R, F, window=8, hidden=8, device="cpu", train_batch=16, seed=3)
    h = torch.randn(n, R, F).cumsum(1) * 0.1
    a.load_history(h)
    for _ in range(3):
        a.train_step()
    a.calibrate(64)
    path = str(tmp_path / "lstm.safetensors")
    ck.save_lstm_shard(a, path)
    b = ck.load_lstm_shard(path, "cpu")
    assert b.trainer.steps == a.trainer.steps and (b.mu, b.sigma) == (a.mu, a.sigma)
    for _ in range(2):  # Adam moments and the sampler's generator resume: same losses
        la, lb = a.train_step(), b.train_step()
        assert torch.equal(la, lb)
    for pa, pb in zip(a.model.parameters(), b.model.parameters()):
        assert torch.equal(pa, pb)
    x = torch.randn(n, F)
    oa, ob = a.tick(x, train=False), b.tick(x, train=False)
    assert torch.equal(oa["verdict"], ob["verdict"]) and torch.equal(oa["err"], ob["err"])


def test_checkpoint_rejects_foreign_files(tmp_path):
    from safetensors.torch import save_file
    p = str(tmp_path / "x.safetensors")
    save_file({"a": torch.zeros(2)}, p)
    try:
        ck.load_streaming_shard(p)
    except ValueError as e:
        assert "not a foremast-amd checkpoint" in str(e)
    else:
        raise AssertionError("foreign file accepted")
