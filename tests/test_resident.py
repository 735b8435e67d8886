"""Reference counting, readiness and expiry of the resident history
(``brain/resident.py``): the bulk (C-level) paths keep the per-key semantics."""

import asyncio

import numpy as np
import torch

from foremast_amd.brain.resident import ResidentHistory


def test_history_references_readiness_and_expiry():
    hist = ResidentHistory(prom=None, device="cpu", ring_len=16, step=60.0, clock=lambda: 0.0, retain_s=100.0,
                           min_capacity=4)
    keys = [("http://p/api/v1/", "m", "ns", "a"), ("http://p/api/v1/", "m", "ns", "b")]
    hs = [hist.key_hash(k) for k in keys]
    both = np.array(hs, dtype=np.uint64)
    # a twice (two jobs of app a), b once; neither has a row yet: pending, not ready
    hist.want_h(hs + hs[:1], 0.0, (keys + keys[:1]).__getitem__)
    assert hist.refs == {hs[0]: 2, hs[1]: 1}
    assert hist.pending == set(hs)
    assert not hist.ready_mask(both).any()
    asyncio.run(hist.assign_only(0.0))
    hist.load_rows(keys, torch.zeros(2, 16))
    assert hist.ready_mask(both).all() and not hist.pending
    assert sorted(hist.rows_of_h(hs).tolist()) == sorted(hist.rows[h] for h in hs)
    assert hist.rows_of_h([hs[1]]).tolist() == [hist.rows[hs[1]]]
    # a third key without a row: ready_mask flags exactly it
    k3 = ("http://p/api/v1/", "m", "ns", "c")
    h3 = hist.key_hash(k3)
    hist.want_h([h3], 5.0, lambda i: k3)
    assert hist.ready_mask(np.array(hs + [h3], dtype=np.uint64)).tolist() == [True, True, False]
    # releases: b's only reference and one of a's (a stays referenced), then c's, then a's last
    hist.unwant_h([hs[0], hs[1]], 10.0)
    assert hist.refs == {hs[0]: 1, h3: 1}
    hist.unwant_h([h3], 12.0)
    hist.unwant_h([hs[0]], 20.0)
    assert hist.refs == {}
    assert hist.last_used[hs[0]] == 20.0 and hist.last_used[hs[1]] == 10.0
    # unreferenced rows expire retain_s after their last use, not before
    hist._assign(70.0)
    assert set(hist.rows) == set(hs)
    hist._assign(115.0)  # b (idle since 10) expires; a (20) stays
    assert set(hist.rows) == {hs[0]}
    # a wanted again before it expires: it is not freed
    hist.want_h([hs[0]], 116.0, lambda i: keys[0])
    hist._assign(500.0)
    assert set(hist.rows) == {hs[0]} and hist.refs == {hs[0]: 1}
