"""LSTM autoencoder: reference model, DP training loop, fused-kernel layout.

The CPU tests emulate the documented gfx950 ``v_mfma_f32_32x32x16`` lane maps
(A: lane l holds A[l&31][8(l>>5)+j]; B: B[8(l>>5)+j][l&31]; C: col l&31,
row (r&3)+8(r>>2)+4(l>>5)) to check the host packing and the kernel's
register plan (gates lane-local, new h = next B operand) before any GPU run.
"""

import numpy as np
import pytest
import torch

from foremast_amd.models import lstm_ae
from foremast_amd.ops import lstm as L


def _emulate_mfma(afrag, bfrag, c):
    """afrag/bfrag: [64, 8] per-lane operand elements; c: [64, 16] accumulators."""
    A = np.zeros((32, 16))
    B = np.zeros((16, 32))
    for l in range(64):
        for j in range(8):
            A[l & 31, 8 * (l >> 5) + j] = afrag[l, j]
            B[8 * (l >> 5) + j, l & 31] = bfrag[l, j]
    Cm = A @ B
    out = c.copy()
    for l in range(64):
        for r in range(16):
            out[l, r] += Cm[(r & 3) + 8 * (r >> 2) + 4 * (l >> 5), l & 31]
    return out


def _sig(x):
    return 1 / (1 + np.exp(-x))


def test_register_plan_matches_reference_step():
    torch.manual_seed(0)
    F = 3
    m = lstm_ae.LSTMAutoencoder(F, 64).double()
    frag = L.pack_fragments(L._augment(m.enc_w_hh, m.enc_b, m.enc_w_ih, F)).double().numpy()
    B = 32
    x = torch.randn(B, F, dtype=torch.float64)
    h0 = torch.randn(B, 64, dtype=torch.float64) * 0.5
    c0 = torch.randn(B, 64, dtype=torch.float64) * 0.5
    # reference one step
    gates = x @ m.enc_w_ih.t() + h0 @ m.enc_w_hh.t() + m.enc_b
    h_ref, c_ref = m._cell(gates, c0)
    # kernel register plan: lane l -> series l&31, half hh = l>>5 owns units 16s+8hh+4e+q
    hreg = np.zeros((64, 32))
    creg = np.zeros((64, 32))
    for l in range(64):
        hh = l >> 5
        for t in range(8):
            for q in range(4):
                u = 16 * (t >> 1) + 8 * hh + 4 * (t & 1) + q
                hreg[l, 4 * t + q] = h0[l & 31, u]
                creg[l, 4 * t + q] = c0[l & 31, u]
    hb = np.zeros((4, 64, 8))
    for s in range(4):
        for j in range(8):
            hb[s, :, j] = hreg[:, (2 * s + (j >> 2)) * 4 + (j & 3)]
    xb = np.zeros((64, 8))
    for l in range(32):
        xb[l, :F] = x[l].numpy()
        xb[l, 7] = 1.0
    hnew = np.zeros_like(hreg)
    for t in range(8):
        acc = np.zeros((64, 16))
        for s in range(5):
            acc = _emulate_mfma(frag[t, s], hb[s] if s < 4 else xb, acc)
        for q in range(4):
            gi, gf, gg, go = acc[:, q], acc[:, 4 + q], acc[:, 8 + q], acc[:, 12 + q]
            c = _sig(gf) * creg[:, 4 * t + q] + _sig(gi) * np.tanh(gg)
            hnew[:, 4 * t + q] = _sig(go) * np.tanh(c)
    for l in range(64):
        hh = l >> 5
        for t in range(8):
            for q in range(4):
                u = 16 * (t >> 1) + 8 * hh + 4 * (t & 1) + q
                assert abs(hnew[l, 4 * t + q] - h_ref[l & 31, u].item()) < 1e-9


def test_lstm_ae_trains_and_scores():
    torch.manual_seed(1)
    N, Lh, F, T = 16, 300, 2, 16
    t = torch.arange(Lh, dtype=torch.float32)
    base = torch.stack([torch.sin(2 * np.pi * t / 24 + i) for i in range(N)])
    series = torch.stack([base, 0.5 * base + 0.1 * torch.randn(N, Lh)], 2)
    z, mu, sd = lstm_ae.normalize(series)
    m = lstm_ae.LSTMAutoencoder(F, 32)
    opt = torch.optim.Adam(m.parameters(), lr=1e-2)
    g = torch.Generator().manual_seed(0)
    first = None
    for it in range(60):
        w = lstm_ae.make_windows(z, T, 64, g)
        loss = m.recon_error(w).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
        first = first if first is not None else float(loss)
    assert float(loss) < 0.6 * first
    with torch.no_grad():
        normal = lstm_ae.make_windows(z, T, 64, g)
        cal = lstm_ae.calibrate(m.recon_error(normal))
        spike = normal.clone()
        spike[:, T // 2:, 0] += 6.0
        e = m.recon_error(spike)
    zs = (e - cal.mu) / cal.sigma
    assert float(zs.min()) > 3.0


@pytest.mark.gpu
@pytest.mark.parametrize("fp8", [False, True])
def test_fused_lstm_kernel_matches_reference(fp8):
    torch.manual_seed(2)
    dev = torch.device("cuda:0")
    N, T, F = 300, 24, 3
    m = lstm_ae.LSTMAutoencoder(F, 64)
    x = torch.randn(N, T, F)
    x[:40, 10:14] += 4.0
    with torch.no_grad():
        ref_err = m.recon_error(x)
        ref_y = m(x)
    p = L.pack(m, fp8=fp8, device=dev)
    out = L.lstm_score(p, x.to(dev).contiguous(), mu=float(ref_err.mean()), sigma=float(ref_err.std()),
                       want_recon=True)
    torch.cuda.synchronize()
    err = out["err"].cpu()
    y = out["recon"].cpu()
    if not fp8:
        np.testing.assert_allclose(y.numpy(), ref_y.numpy(), atol=3e-2, rtol=3e-2)
        np.testing.assert_allclose(err.numpy(), ref_err.numpy(), rtol=5e-2, atol=1e-3)
    else:
        corr = np.corrcoef(err.numpy(), ref_err.numpy())[0, 1]
        assert corr > 0.98
        assert (y - ref_y).abs().mean() < 0.08
    # ranking: the perturbed windows are the highest errors in both
    top_ref = set(torch.topk(ref_err, 40).indices.tolist())
    top_k = set(torch.topk(err, 40).indices.tolist())
    assert len(top_ref & top_k) >= 36


@pytest.mark.gpu
@pytest.mark.parametrize("F", [2, 3])
def test_fp8_kernel_matches_emulated_fp8_reference(F):
    """The fp8 kernel against a PyTorch reference that applies the SAME e4m3 rounding
    (per-(row, 32-k) E8M0 weight scales, h entering as e4m3(h * 2^8) * 2^-8, saturated
    e4m3 inputs; ops/lstm.py fp8_emulated_forward): what is left is accumulation order and
    the hardware exp / rcp, so the reconstruction error agrees to rtol 1e-2 on every
    window -- a wrong scale map or a bias would not pass."""
    torch.manual_seed(11 + F)
    dev = torch.device("cuda:0")
    N, T = 512, 24
    m = lstm_ae.LSTMAutoencoder(F, 64)
    with torch.no_grad():  # a trained-like spread of weights: some blocks far from the others
        m.enc_w_hh[:, :32] *= 3.0
        m.dec_w_hh[64:128] *= 0.05
        m.enc_b[::5] *= 6.0
        m.out_w *= 8.0       # a read-out that carries the hidden state into y
    x = torch.randn(N, T, F)
    x[:40, 10:14] += 4.0
    ref_y, ref_err = L.fp8_emulated_forward(m, x)
    p = L.pack(m, fp8=True, device=dev)
    out = L.lstm_score(p, x.to(dev).contiguous(), mu=float(ref_err.mean()), sigma=float(ref_err.std()),
                       want_recon=True)
    torch.cuda.synchronize()
    err, y = out["err"].cpu(), out["recon"].cpu()
    np.testing.assert_allclose(err.numpy(), ref_err.numpy(), rtol=1e-2, atol=1e-5)
    # the reconstruction is the sensitive output (the error is dominated by x): kernel vs
    # emulated fp8 must be far closer than emulated fp8 vs the unquantised model
    d_kernel = (y - ref_y).abs()
    with torch.no_grad():
        d_quant = (m(x) - ref_y).abs()
    assert float(d_quant.mean()) > 1e-3                       # the test can tell fp8 from fp32
    assert float(d_kernel.mean()) < 0.1 * float(d_quant.mean()), (float(d_kernel.mean()), float(d_quant.mean()))
    assert float(np.percentile(d_kernel.numpy(), 99.9)) < 0.25 * float(np.percentile(d_quant.numpy(), 99.9))


@pytest.mark.gpu
def test_fp8_scoring_saturates_out_of_range_inputs():
    """A regressed window's z-scored inputs can exceed the fp8 e4m3 range
    (|x| > 448): the kernel saturates them, so the error stays
    finite and large instead of becoming NaN (which would read as healthy)."""
    torch.manual_seed(4)
    dev = torch.device("cuda:0")
    N, T, F = 64, 16, 2
    m = lstm_ae.LSTMAutoencoder(F, 64)
    x = torch.randn(N, T, F) * 0.5
    x[:8, 4:] += 60.0  # x3 regression of a calm series, in z units
    p = L.pack(m, fp8=True, device=dev)
    out = L.lstm_score(p, x.to(dev).contiguous(), mu=1.0, sigma=1.0, thr_default=4.0)
    torch.cuda.synchronize()
    err = out["err"].cpu()
    assert torch.isfinite(err).all()
    assert float(err[:8].min()) > 10 * float(err[8:].max())
    assert out["verdict"][:8].cpu().eq(1).all()


@pytest.mark.gpu
def test_device_fp8_matches_torch_ocp():
    dev = torch.device("cuda:0")
    v = torch.tensor([0.0, 1.0, -1.5, 0.3, 447.0, -240.0, 1e-3, 3.14159], device=dev)
    got = L.device_fp8(v).cpu()
    exp = v.cpu().to(torch.float8_e4m3fn).view(torch.uint8)
    assert torch.equal(got, exp)


def _toy_history(n, R, F, seed=0):
    g = torch.Generator().manual_seed(seed)
    t = torch.arange(R, dtype=torch.float32)
    ph = torch.rand(n, 1, generator=g) * 6.28
    return [10 + 3 * torch.sin(2 * np.pi * t / 48 + ph + f) + 0.1 * torch.randn(n, R, generator=g)
            for f in range(F)]


def test_lstm_shard_cpu_streaming():
    from foremast_amd.brain.lstm_engine import LstmShard
    n, R, F = 40, 200, 2
    sh = LstmShard(n, R, F, window=12, device="cpu", app_id=(torch.arange(n) // 4).int(), n_apps=10,
                   train_batch=32, lr=1e-2)
    sh.load_history(_toy_history(n, R, F))
    l0 = float(sh.train_step())
    for k in range(25):
        sh.ingest_tick(torch.randn(n, F) * 0.1 + 10)
        l1 = float(sh.train_step())
    assert l1 < l0
    sh.calibrate(64)
    out = sh.score()
    assert out["verdict"].shape == (n,) and int(sh.app_stats[:, 1].sum()) == n


def test_lstm_per_series_calibration_cpu():
    """One shared model, series of very different noise: the per-series
    calibration learns each series' own healthy error level, so a x3
    regression of a calm series is flagged while no healthy series — noisy
    ones included — crosses the threshold."""
    from foremast_amd.brain.lstm_engine import LstmShard
    n, R, T = 64, 240, 12
    g = torch.Generator().manual_seed(7)
    t = torch.arange(R, dtype=torch.float32)
    noise = torch.where(torch.arange(n) % 2 == 0, 0.05, 1.5)[:, None]  # calm / noisy alternate
    ph = torch.rand(n, 1, generator=g) * 6.28
    hist = 10 + 3 * torch.sin(2 * np.pi * t / 48 + ph) + noise * torch.randn(n, R, generator=g)
    torch.manual_seed(0)
    sh = LstmShard(n, R, 1, window=T, device="cpu", app_id=torch.arange(n).int(), n_apps=n,
                   train_batch=64, lr=1e-2, cal_windows=8)
    sh.load_history([hist])
    for _ in range(60):
        sh.train_step()
    sh.calibrate(256)
    mu = sh.cal[:, 0]
    assert float(mu[1::2].median()) > 3 * float(mu[0::2].median())  # noisy series reconstruct worse
    bad = torch.tensor([0, 2, 4])
    for k in range(8):
        tk = torch.tensor([float(R + k)])
        v = 10 + 3 * torch.sin(2 * np.pi * tk / 48 + ph) + noise * torch.randn(n, 1, generator=g)
        v[bad] *= 3.0
        sh.ingest_tick(v)
    out = sh.score()
    flagged = set(torch.nonzero(out["verdict"]).flatten().tolist())
    assert set(bad.tolist()) <= flagged
    assert len(flagged - set(bad.tolist())) <= 1


@pytest.mark.gpu
@pytest.mark.parametrize("fp8", [False, True])
def test_lstm_shard_gpu_matches_model(fp8):
    """Streaming shard on the GPU: rings + window_stats + device repack +
    fused kernel agree with the PyTorch model on the same windows."""
    from foremast_amd.brain.lstm_engine import LstmShard
    dev = torch.device("cuda:0")
    n, R, F = 512, 300, 2
    sh = LstmShard(n, R, F, window=16, device=dev, fp8=fp8, app_id=(torch.arange(n, device=dev) // 4).int(),
                   n_apps=128, train_batch=256, lr=1e-2)
    sh.load_history([h.to(dev) for h in _toy_history(n, R, F)])
    # stats from the native window_stats kernel equal torch's
    ref_mean = torch.stack([r.logical().float().mean(1) for r in sh.rings], 1)
    assert torch.allclose(sh.mean, ref_mean, rtol=1e-4, atol=1e-3)
    for k in range(5):
        sh.ingest_tick(torch.full((n, F), 10.0, device=dev))
        sh.train_step()
    sh.calibrate(1000)  # sampled window count != series count
    assert sh.cal is not None and sh.cal.shape == (n, 2) and bool((sh.cal[:, 0] > 0).all())
    cal0 = sh.cal.clone()
    out = sh.score()
    torch.cuda.synchronize()
    # per-series z-score from the calibration in force at scoring time; the
    # epilogue then moved mu_i of the non-flagged series toward their error
    z_ref = torch.minimum((out["err"] - sh.mu) / sh.sigma, (out["err"] - cal0[:, 0]) * cal0[:, 1])
    assert torch.allclose(out["zscore"], z_ref, rtol=1e-5, atol=1e-5)
    from foremast_amd.brain.lstm_engine import CAL_GATE
    upd = (out["verdict"] == 0) & ((out["err"] - cal0[:, 0]) * cal0[:, 1] <= CAL_GATE)
    mu_ref = torch.where(upd, cal0[:, 0] + sh.cal_ewma * (out["err"] - cal0[:, 0]), cal0[:, 0])
    assert torch.allclose(sh.cal[:, 0], mu_ref, rtol=1e-5, atol=1e-7)
    assert torch.allclose(sh.cal[:, 0] * sh.cal[:, 1], cal0[:, 0] * cal0[:, 1], rtol=1e-5)
    x = sh._gather(sh._all, sh._zero_off)
    with torch.no_grad():
        ref = sh.model.recon_error(x)
    err = out["err"]
    if fp8:
        assert np.corrcoef(err.cpu().numpy(), ref.cpu().numpy())[0, 1] > 0.95
    else:
        assert torch.allclose(err, ref, rtol=5e-2, atol=2e-3)
    assert int(sh.app_stats[:, 1].sum()) == n
    # overlapped tick (training on a side stream, scoring with the pre-step weights)
    before = [p.detach().clone() for p in sh.model.parameters()]
    out = sh.tick(torch.full((n, F), 10.0, device=dev))
    torch.cuda.synchronize()
    assert int(sh.app_stats[:, 1].sum()) == n and torch.isfinite(out["err"]).all()
    assert any(not torch.equal(b, p) for b, p in zip(before, sh.model.parameters()))


@pytest.mark.gpu
@pytest.mark.parametrize("fp8", [False, True])
def test_lstm_tick_graph_matches_eager(fp8, monkeypatch):
    """A steady-state training tick as ONE HIP-graph replay (ring appends at the device
    column, repack, level term, training kernel + tail + Adam on the side stream,
    scoring with the device head) gives the eager tick's outputs and weights, over
    ticks that cross a statistics refresh (an eager tick inside the graph run)."""
    from foremast_amd.brain.lstm_engine import LstmShard
    dev = torch.device("cuda:0")
    n, R, F = 512, 300, 2

    def make(graph):
        monkeypatch.setenv("FOREMAST_LSTM_GRAPH", "1" if graph else "0")
        sh = LstmShard(n, R, F, window=16, device=dev, fp8=fp8, app_id=(torch.arange(n, device=dev) // 4).int(),
                       n_apps=128, train_batch=256, lr=1e-2, restat_every=4, seed=3)
        sh.load_history([h.to(dev) for h in _toy_history(n, R, F)])
        for _ in range(3):
            sh.train_step()
        sh.calibrate(512)
        return sh
    a, b = make(False), make(True)
    xa = torch.empty((n, F), device=dev)
    xb = torch.empty((n, F), device=dev)
    g = torch.Generator().manual_seed(5)
    for k in range(9):
        x = torch.randn(n, F, generator=g) + 10.0
        xa.copy_(x)
        xb.copy_(x)
        oa, ob = a.tick(xa), b.tick(xb)
        torch.cuda.synchronize()
        assert torch.equal(oa["verdict"], ob["verdict"]), k
        torch.testing.assert_close(ob["err"], oa["err"], rtol=1e-6, atol=1e-7)
        for pa, pb in zip(a.model.parameters(), b.model.parameters()):
            torch.testing.assert_close(pb, pa, rtol=1e-6, atol=1e-7)
        assert torch.equal(a.app_stats, b.app_stats)
    assert b.graph_replays >= 4 and a.graph_replays == 0
    assert a.trainer.steps == b.trainer.steps


@pytest.mark.gpu
def test_lstm_tick_graph_enqueued_back_to_back(monkeypatch):
    """Graph ticks enqueued without a host wait between them (the replay steps the
    device ring record itself, the host writes nothing per tick) end in the eager
    shard's rings, weights and counters, across a statistics refresh."""
    from foremast_amd.brain.lstm_engine import LstmShard
    dev = torch.device("cuda:0")
    n, R, F = 512, 300, 2

    def make(graph):
        monkeypatch.setenv("FOREMAST_LSTM_GRAPH", "1" if graph else "0")
        sh = LstmShard(n, R, F, window=16, device=dev, fp8=False, app_id=(torch.arange(n, device=dev) // 4).int(),
                       n_apps=128, train_batch=256, lr=1e-2, restat_every=5, seed=3)
        sh.load_history([h.to(dev) for h in _toy_history(n, R, F)])
        sh.train_step()
        sh.calibrate(512)
        return sh
    a, b = make(False), make(True)
    g = torch.Generator().manual_seed(9)
    xs = [(torch.randn(n, F, generator=g) + 10.0).pin_memory() for _ in range(9)]
    for sh in (a, b):
        x = torch.empty((n, F), device=dev)
        for xk in xs:
            x.copy_(xk, non_blocking=True)  # stream-ordered: lands after the previous tick's replay
            sh.tick(x)
    torch.cuda.synchronize()
    assert b.graph_replays >= 4
    for ra, rb in zip(a.rings, b.rings):
        assert ra.head == rb.head
        assert torch.equal(ra.data, rb.data)
    for pa, pb in zip(a.model.parameters(), b.model.parameters()):
        torch.testing.assert_close(pb, pa, rtol=1e-6, atol=1e-7)
    assert torch.equal(a.app_stats, b.app_stats)


def test_backward_register_plan_matches_wT_dgates():
    """CPU emulation of the K7 backward recurrence step: dh_{t-1} = W_hh^T dgates
    from lane-local dgates (forward accumulator order) through the packed W^T
    fragments lands in the h register layout."""
    from foremast_amd.ops import lstm_train as LT
    rng = np.random.default_rng(0)
    W = rng.standard_normal((256, 64))
    d = rng.standard_normal((32, 256))  # [series, pytorch gate row]
    frag = W.flatten()[LT.transposed_frag_index().numpy()].reshape(2, 16, 64, 8)

    def unit(t, hh, q):
        return 16 * (t >> 1) + 8 * hh + 4 * (t & 1) + q

    acc = [np.zeros((64, 16)), np.zeros((64, 16))]
    for ks in range(16):
        tt, e = ks >> 1, ks & 1
        b = np.zeros((64, 8))
        for l in range(64):
            for j in range(8):
                r = 8 * e + j
                b[l, j] = d[l & 31, (r >> 2) * 64 + unit(tt, l >> 5, r & 3)]
        for mt in range(2):
            acc[mt] = _emulate_mfma(frag[mt, ks], b, acc[mt])
    ref = d @ W  # [series, unit] = (W^T d)^T
    for l in range(64):
        for mt in range(2):
            for r in range(16):
                u = unit(4 * mt + (r >> 2), l >> 5, r & 3)
                assert abs(acc[mt][l, r] - ref[l & 31, u]) < 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("F,variant", [(1, 0), (3, 0), (1, 1), (3, 1)])
def test_fused_lstm_training_grads_match_autograd(F, variant):
    from foremast_amd.ops.lstm_train import FusedLstmGrad
    torch.manual_seed(5)
    dev = torch.device("cuda:0")
    B, T = 64, 12
    m = lstm_ae.LSTMAutoencoder(F, 64).to(dev)
    x = torch.randn(B, T, F, device=dev)
    loss = m.recon_error(x).mean()
    ref = torch.autograd.grad(loss, list(m.parameters()))
    fg = FusedLstmGrad(B, T, F, dev, variant=variant)
    with torch.no_grad():
        err_ref = m.recon_error(x)
    got_loss = fg.grads(m, x)
    torch.cuda.synchronize()
    assert torch.allclose(fg.err, err_ref, rtol=3e-2, atol=1e-3)
    assert abs(float(got_loss) - float(loss)) < 3e-2 * abs(float(loss))
    for (name, p), g in zip(m.named_parameters(), ref):
        cos = torch.nn.functional.cosine_similarity(p.grad.flatten(), g.flatten(), dim=0)
        rel = (p.grad - g).norm() / g.norm().clamp(min=1e-12)
        assert cos > 0.99 and rel < 0.08, (name, float(cos), float(rel))



@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1])
def test_fused_training_reads_rings_directly(variant):
    """K7 with ring-direct input: sampled (series, start) windows read from the
    bf16 rings (wrapping past column R-1) and z-scored in the kernel give the
    same errors and gradients as the same windows gathered on the host."""
    from foremast_amd.ops.lstm import RingSource
    from foremast_amd.ops.lstm_train import FusedLstmGrad
    torch.manual_seed(7)
    dev = torch.device("cuda:0")
    n, R, F, B, T = 200, 90, 2, 64, 16
    m = lstm_ae.LSTMAutoencoder(F, 64).to(dev)
    # row-padded [n, 96] storage viewed as [n, R], like HistoryRing
    rings = [torch.randn(n, 96, device=dev).mul_(f + 1).add_(f).to(torch.bfloat16)[:, :R] for f in range(F)]
    mean = torch.randn(n, F, device=dev) * 0.1
    rstd = 1.0 / (0.5 + torch.rand(n, F, device=dev))
    si = torch.randint(0, n, (B,), device=dev, dtype=torch.int32)
    st = torch.randint(0, 3 * R, (B,), device=dev, dtype=torch.int32)  # kernel reduces mod R
    st[:8] = R - 5  # windows that wrap
    cols = (st.long()[:, None] + torch.arange(T, device=dev)[None]) % R
    x = torch.stack([r[si.long()[:, None], cols].float() for r in rings], 2)
    x = ((x - mean[si.long()][:, None]) * rstd[si.long()][:, None]).contiguous()
    fg = FusedLstmGrad(B, T, F, dev, variant=variant)
    loss_d = fg.grads(m, x)
    err_d = fg.err.clone()
    g_d = [p.grad.clone() for p in m.parameters()]
    loss_r = fg.grads(m, RingSource(rings=rings, mean=mean, rstd=rstd, win_series=si, win_start=st))
    torch.cuda.synchronize()
    assert torch.allclose(fg.err, err_d, rtol=1e-5, atol=1e-6)
    assert abs(float(loss_r) - float(loss_d)) <= 1e-5 * abs(float(loss_d))
    for p, g in zip(m.parameters(), g_d):
        assert torch.allclose(p.grad, g, rtol=1e-4, atol=1e-6)
    # scoring the newest window of every row straight from the rings
    p = L.pack(m, device=dev)
    start = (R - T + 40) % R  # wraps
    cols = (start + torch.arange(T, device=dev)) % R
    xs = torch.stack([r[:, cols].float() for r in rings], 2)
    xs = ((xs - mean[:, None]) * rstd[:, None]).contiguous()
    ref = L.lstm_score(p, xs)["err"].clone()
    got = L.lstm_score(p, None, ring=RingSource(rings=rings, start_col=start, mean=mean, rstd=rstd), T=T)["err"]
    torch.cuda.synchronize()
    assert torch.allclose(got, ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("F", [1, 3])
def test_pack_codes_reproduce_reference_layouts(F):
    """The table-driven packer's codes (evaluated with torch) equal the
    reference fragment layouts: augmented forward fragments of both phases and
    the transposed backward fragments."""
    from foremast_amd.ops import lstm_train as LT
    from foremast_amd.ops.pack import make_codes, reference_gather
    torch.manual_seed(3)
    m = lstm_ae.LSTMAutoencoder(F, 64)
    srcs = L.model_srcs(m)
    ref_e = L.pack_fragments(L._augment(m.enc_w_hh, m.enc_b, m.enc_w_ih, F)).flatten()
    ref_d = L.pack_fragments(L._augment(m.dec_w_hh, m.dec_b, None, F)).flatten()
    assert torch.equal(reference_gather(L.augmented_codes(F, True), srcs), ref_e)
    assert torch.equal(reference_gather(L.augmented_codes(F, False), srcs), ref_d)
    # block-scaled fp8 layout: codes = the fp8 index gather of the augmented weight
    for enc, A in ((True, L._augment(m.enc_w_hh, m.enc_b, m.enc_w_ih, F)), (False, L._augment(m.dec_w_hh, m.dec_b, None, F))):
        idx = L._fp8_index("cpu")
        want = torch.where(idx >= 0, A.flatten()[idx.clamp(min=0)], torch.zeros(()))
        assert torch.equal(reference_gather(L.augmented_codes(F, enc, fp8=True), srcs), want)
    tidx = LT.transposed_frag_index()
    got = reference_gather(make_codes(torch.full_like(tidx, L.LSTM_SRCS.index("dec_w_hh")), tidx), srcs)
    assert torch.equal(got, m.dec_w_hh.detach().flatten()[tidx])


@pytest.mark.parametrize("F", [1, 2, 5])
def test_block_scaled_fp8_pack_layout_and_precision(F):
    """The fp8 scoring buffer (ops/lstm.py pack_fp8): fragment bytes of tile t, k-step s,
    lane l hold gate row 32 t + (l & 31) (permuted) at the k order the kernel's B operand
    uses (k-step 0: the lane half's 32 h-register units; k-step 1: inputs, then the bias
    at byte 7); dequantised with their lane-major E8M0 scales they reproduce the weights
    within e4m3's half-ulp (2^-4 relative; subnormals: a 2^-10 share of the row's
    maximum), and every (row, 32-k block) scale is the smallest power of two that fits
    the block's maximum in 448."""
    torch.manual_seed(11)
    m = lstm_ae.LSTMAutoencoder(F, 64)
    A = L._augment(m.enc_w_hh, m.enc_b, m.enc_w_ih, F)
    A[5, :64] *= 1e-3                           # rows of very different magnitude: per-block scales
    A[9, :] *= 300.0
    buf = L.pack_fp8(A)
    assert buf.dtype == torch.uint8 and buf.numel() == L.FP8_FRAG_BYTES + L.FP8_SCALE_BYTES
    q = buf[:L.FP8_FRAG_BYTES].view(torch.float8_e4m3fn).float().view(L.TILES, 2, 2, 64, 16)  # half-major
    q = q.permute(0, 1, 3, 2, 4).reshape(L.TILES, 2, 64, 32)
    sc = buf[L.FP8_FRAG_BYTES:].view(64, L.TILES * 2).t().reshape(L.TILES, 2, 2, 32).float()  # [t, s, b, r]
    lanes = torch.arange(64)
    f = torch.exp2(sc - 127)[:, :, (torch.arange(32) // 16)[None, :], (lanes & 31)[:, None]]   # [t, s, lane, j]
    deq = q * f
    rows = L.gate_row_perm()
    units = L.h_units(torch.arange(64) >> 5)
    for t in (0, 3, 7):
        for lane in (0, 17, 40, 63):
            r = int(rows[32 * t + (lane & 31)])
            np.testing.assert_allclose(deq[t, 0, lane].numpy(), A[r, units[lane]].numpy(), rtol=2 ** -4,
                                       atol=float(A[r, units[lane]].abs().max()) * 2 ** -10 + 1e-30)
            want1 = A[r, 64:72] if lane < 32 else torch.zeros(8)
            np.testing.assert_allclose(deq[t, 1, lane, :8].numpy(), want1.numpy(), rtol=2 ** -4,
                                       atol=float(want1.abs().max()) * 2 ** -10 + 1e-30)
            assert float(deq[t, 1, lane, 8:].abs().max()) == 0.0
    # one scale per (tile, k-step, row r, block b) in lane r + 32 b: bytes 16 b .. 16 b + 15 of
    # lanes r and r + 32; the smallest power of two with the block's absmax <= 448 * scale
    vals = torch.where(L._fp8_index("cpu") >= 0, A.flatten()[L._fp8_index("cpu").clamp(min=0)],
                       torch.zeros(())).view(L.TILES * 2, 2, 32, 2, 16)        # [(t, s), h, r, b, j]
    blk = vals.abs().amax(dim=(1, 4)).permute(0, 2, 1).reshape(-1)             # [(t, s), b, r]
    s_flat = (buf[L.FP8_FRAG_BYTES:].view(64, L.TILES * 2).t().float() - 127).reshape(-1)  # [(t, s), lane]
    nz = blk > 0
    assert bool((blk[nz] <= 448 * torch.exp2(s_flat[nz])).all())
    assert bool((blk[nz] > 448 * torch.exp2(s_flat[nz] - 1)).all())


@pytest.mark.gpu
@pytest.mark.parametrize("fp8", [False, True])
def test_native_pack_matches_torch_repack(fp8):
    """One pack launch gives the same fragments as the torch gather path, fp8
    block scales included (exact: frexp exponents and round-to-nearest-even e4m3
    on both sides)."""
    torch.manual_seed(4)
    dev = torch.device("cuda:0")
    m = lstm_ae.LSTMAutoencoder(3, 64).to(dev)
    ref = L.pack(m.cpu(), fp8=fp8, device=dev)
    m = m.to(dev)
    p = L.pack(m, fp8=fp8, device=dev)
    with torch.no_grad():
        for q in m.parameters():
            q.mul_(1.5)
    ref = L.pack(m, fp8=fp8, device=dev)
    L.repack_into(p, m)
    torch.cuda.synchronize()
    assert torch.equal(p.w_enc, ref.w_enc) and torch.equal(p.w_dec, ref.w_dec)
    assert torch.equal(p.w_out, ref.w_out) and torch.equal(p.b_out, ref.b_out)


def _level_shard(device, dtype, n=64, m=480, days=4, F=2, seed=3):
    """Seasonal series with noise sigma 1 and, on half of them, a trend of ~5 sigma a day
    (a naive same-minutes-of-earlier-days baseline would flag every trending series)."""
    from foremast_amd.brain.lstm_engine import LstmShard
    R = m * days
    g = torch.Generator().manual_seed(seed)
    slope = torch.zeros(n, 1)
    slope[::2] = 5.0 / m

    def values(t, noise):
        t = torch.as_tensor(t, dtype=torch.float32)
        return 100.0 + 20.0 * torch.sin(2 * np.pi * t / m) + slope * t + noise

    t = torch.arange(R, dtype=torch.float32)[None, :]
    hist = [values(t, torch.randn(n, R, generator=g)) for _ in range(F)]
    shard = LstmShard(n, R, F, window=16, hidden=64 if device == "cuda" else 16, device=device, dtype=dtype,
                      fused_train=False, cal_windows=4, train_batch=64, season=m, level_points=8,
                      level_threshold=5.5)
    shard.load_history([h.to(device) for h in hist])
    shard._test_values = values
    return shard, g, m


def _level_ticks(shard, g, m, shifted, k=8, size=4.0):
    n, F = shard.n, shard.F
    for j in range(k):
        tt = float(shard.rings[0].length + shard.ticks)
        v = torch.stack([shard._test_values(tt, torch.randn(n, generator=g)[:, None])[:, 0] for _ in range(F)], 1)
        v[shifted] += size
        shard.ingest_tick(v.to(shard.device))


def test_lstm_level_term_flags_small_shift_cpu():
    """The level term (mean of the newest 8 points minus the same minutes of the earlier
    days, over its calibrated spread) flags a +4 sigma shift the shape-scoring AE cannot
    see, and stays quiet on the healthy series."""
    shard, g, m = _level_shard("cpu", torch.float32)
    shard.calibrate(256)
    assert shard.lvl_sig is not None and torch.isfinite(shard.lvl_sig).all()
    # the spread of an 8-point mean against the 3 earlier days' 16-point means (E = 4 at
    # m = 480) extrapolated over the days: sigma * sqrt(1/8 + (21/9)/16) ~ 0.52, trending
    # series included
    assert 0.35 < float(shard.lvl_sig.median()) < 0.7
    assert float(shard.lvl_sig[::2].median()) < 1.3 * float(shard.lvl_sig[1::2].median())
    shifted = torch.arange(8)
    _level_ticks(shard, g, m, shifted)
    zl = shard.level_z()
    z = zl.abs().amax(1)
    assert bool((z[shifted] > 5.5).all()), z[shifted]
    assert int((z[8:] > 5.5).sum()) == 0
    shard.threshold = 1e9  # AE term off: the verdict is the level term alone
    out = shard.score()
    assert out["verdict"][:8].all() and int(out["verdict"][8:].sum()) == 0


@pytest.mark.gpu
def test_lstm_level_kernel_matches_cpu():
    """lstm_level (GPU, bf16 rings) == the torch definition, calibration and scoring."""
    shard, g, m = _level_shard("cuda", torch.bfloat16, n=300, F=3)
    shifted = torch.arange(0, 300, 7)
    _level_ticks(shard, g, m, shifted, k=8)
    r0 = shard.rings[0]
    newest, avail = (r0.head + r0.length - 1) % r0.R, r0.length
    st = L.lstm_level([r.data for r in shard.rings], newest, avail, m, 8, K=20, back_step=9)
    torch.cuda.synchronize()
    shard.gpu = False
    ref = torch.stack([shard._level_stat_cpu((k + 1) * 9) for k in range(20)])
    shard.gpu = True
    torch.testing.assert_close(st.cpu(), ref.cpu(), rtol=1e-5, atol=1e-4, equal_nan=True)
    shard.calibrate(256)
    zl = shard.level_z()
    shard.gpu = False
    zref = shard.level_z()
    shard.gpu = True
    torch.testing.assert_close(zl.cpu(), zref.cpu(), rtol=1e-4, atol=1e-4)
    assert bool((zl.abs().amax(1)[shifted] > 5.5).all())


@pytest.mark.gpu
def test_fused_level_term_matches_level_kernel():
    """The scoring kernel's fused level term (its prologue) gives the standalone
    lstm_level kernel's z, with the head absolute or on the device, and flags the
    shifted series."""
    shard, g, m = _level_shard("cuda", torch.bfloat16, n=300, F=3)
    shifted = torch.arange(0, 300, 7)
    _level_ticks(shard, g, m, shifted, k=8)
    shard.calibrate(256)
    zl = shard.level_z()
    r0 = shard.rings[0]
    shard._pack_scoring()
    for dev_head in (False, True):
        if dev_head:
            shard._grec_dev[1] = r0.head
            ring = shard._ring_src_dev()
        else:
            ring = shard._ring_src()
        lv = shard._level_args(ring)
        assert lv is not None
        lv["out"] = torch.full_like(zl, float("nan"))
        out = L.lstm_score(shard.packed, None, shard.mu, shard.sigma, thr_default=shard.threshold, ring=ring,
                           T=shard.T, thr_level=float(shard.level_threshold), level=lv)
        torch.cuda.synchronize()
        torch.testing.assert_close(lv["out"], zl, rtol=1e-5, atol=1e-5)
        assert bool((out["verdict"][shifted] == 1).all())


@pytest.mark.gpu
@pytest.mark.parametrize("sel", [0, 1, 2, 3])
def test_block_scaled_fp8_mfma_lane_map(sel):
    """The CDNA4 block-scaled MFMA (v_mfma_scale_f32_32x32x64_f8f6f4, e4m3) under the maps
    the fp8 LSTM kernel relies on, on exact data (small integers, exact in e4m3; a
    different power of two per (row, k block) of A and (column, k block) of B; asymmetric,
    so a transposed map cannot pass): lane l holds row / column l & 31 (byte j at
    k = 32 (l >> 5) + j, the same for A and B), and bytes 16 b .. 16 b + 15 of lanes r and
    r + 32 form k block b, scaled by byte ``sel`` of lane r + 32 b's scale register
    (scripts/probe_mfma_scale.py decoded this map; the other bytes hold decoys)."""
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(7 + sel)
    A = torch.randint(-8, 9, (32, 64), generator=g).float()
    B = torch.randint(-8, 9, (64, 32), generator=g).float()
    A[3, :] += torch.arange(64) % 5           # asymmetric rows / columns
    B[:, 5] += torch.arange(64) % 3
    sa = torch.randint(120, 135, (32, 2), generator=g)   # [row, block]
    sb = torch.randint(120, 135, (32, 2), generator=g)   # [column, block]

    def regs(s, decoy):   # lane r + 32 b: the scale of (r, b) in byte sel
        out = []
        for lane in range(64):
            v = 0
            for j in range(4):
                v |= (int(s[lane & 31, lane >> 5]) if j == sel else decoy) << (8 * j)
            out.append(v - (1 << 32) if v >= 1 << 31 else v)
        return torch.tensor(out, dtype=torch.int32, device=dev)
    got = L.mfma_scale_probe(A.to(dev), B.to(dev), regs(sa, 0x55), regs(sb, 0x66), sel).cpu().double()
    blk = (torch.arange(64) % 32) // 16                    # k block of probe index k
    fa = torch.exp2(sa.double() - 127)[:, blk]             # [32, 64]
    fb = torch.exp2(sb.double() - 127)[:, blk].t()         # [64, 32]
    want = (A.double() * fa) @ (B.double() * fb)
    # products of different powers of two: the fp32 accumulation rounds (2^-23 relative)
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-6)
