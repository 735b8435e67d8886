"""Hand-written gfx950 (CDNA4) HIP kernels and their launchers.

Kernels (``csrc/``), each with a PyTorch reference in ``foremast_amd.models``:

==========  ============================  ==========================================
K#          kernel                        reference
==========  ============================  ==========================================
K1          ``window_stats``              models/moving_average.py
K2/K3       ``smooth_fit`` (ES/DES/HW)    models/smoothing.py
K5/K11      ``rank_tests``                models/pairwise.py
K6/K7       ``lstm_*``                    models/lstm_ae.py
K8          ``bivariate``                 models/bivariate.py
K9          fused detection epilogue      models/detect.py
K10         ``ring_append``               ingest/ringbuffer.py
==========  ============================  ==========================================
"""

from . import _native  # noqa: F401


def available() -> bool:
    return _native.available()
