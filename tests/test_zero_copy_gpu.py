"""Zero-copy tick I/O (bench.py --zero-copy): the ingest kernel reading a tick's
points from pinned host memory, and the health table written to pinned host
memory by a kernel, must equal the memcpy path bit for bit."""

import pytest
import torch


@pytest.mark.gpu
def test_ingest_from_pinned_host_matches_device_input():
    from foremast_amd.ops import kernels as K
    dev = torch.device("cuda:0")
    N, R, P, W = 1000, 64, 5, 10
    g = torch.Generator().manual_seed(0)
    hist0 = torch.randn(N, R, generator=g).to(torch.bfloat16)
    cur0 = torch.randn(N, P * W, generator=g)
    base0 = torch.randn(N, P * W, generator=g)
    vals = torch.randn(N, 2 * P, generator=g)
    vals[::7, 3] = float("nan")
    host = vals.pin_memory()
    outs = []
    for src in (host, vals.to(dev)):
        hist, cur, base = hist0.to(dev), cur0.to(dev), base0.to(dev)
        zero = torch.full((33,), 5, dtype=torch.int32, device=dev)
        K.tick_ingest(hist, 17, cur, P, W, 3, src[:, :P], graduate=True, base=base, newb=src[:, P:], zero=zero)
        torch.cuda.synchronize()
        outs.append((hist.cpu(), cur.cpu(), base.cpu(), zero.cpu()))
    for a, b in zip(*outs):
        assert torch.equal(a.view(torch.int16) if a.dtype == torch.bfloat16 else a.nan_to_num(7.5),
                           b.view(torch.int16) if b.dtype == torch.bfloat16 else b.nan_to_num(7.5))


@pytest.mark.gpu
def test_copy_to_host_kernel():
    from foremast_amd.ops import kernels as K
    dev = torch.device("cuda:0")
    for n in (1, 255, 256, 40_001):
        src = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device=dev)
        dst = torch.full((n,), 7, dtype=torch.int32).pin_memory()
        K.copy_to_host(dst, src)
        torch.cuda.current_stream().synchronize()
        assert torch.equal(dst, src.cpu())
    with pytest.raises(Exception):
        K.copy_to_host(torch.zeros(4, dtype=torch.int32), torch.zeros(4, dtype=torch.int32, device=dev))  # not pinned


@pytest.mark.gpu
def test_bench_zero_copy_matches_memcpy_tick():
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = []
    for extra in ([], ["--zero-copy"]):
        out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "3", "--warmup", "2",
                              "--series", "5000", "--ring", "2880", "--anomaly-frac", "0.02"] + extra,
                             capture_output=True, text=True, timeout=300, cwd=root)
        assert out.returncode == 0, out.stderr[-3000:]
        res.append(json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0]))
    assert res[1]["config"]["zero_copy"] is True and res[0]["config"]["zero_copy"] is False
    assert res[0]["health"] == res[1]["health"] and res[0]["detection"] == res[1]["detection"]
