"""Batched scorers (the brain's model families) — reference semantics in
PyTorch; the gfx950 kernels in :mod:`foremast_amd.ops` implement the same math."""
