"""Brain configuration, read from the reference's environment-variable names.

Names and defaults follow ``deploy/foremast/3_brain/foremast-brain.yaml:21-81``
and ``foremast-brain/README.md:22-38``:

``ES_ENDPOINT``, ``ML_ALGORITHM``, ``threshold``, ``bound``,
``min_lower_bound``, ``metric_type_threshold_count``, ``metric_type{i}`` /
``threshold{i}`` / ``bound{i}`` / ``min_lower_bound{i}``,
``MIN_MANN_WHITE_DATA_POINTS``, ``MIN_WILCOXON_DATA_POINTS``,
``MIN_KRUSKAL_DATA_POINTS``, ``MAX_STUCK_IN_SECONDS``,
``ML_PAIRWISE_ALGORITHM``, ``ML_PAIRWISE_THRESHOLD``,
``MIN_HISTORICAL_DATA_POINT_TO_MEASURE``, ``MAX_CACHE_SIZE``, ``ML_BOUND``,
``ML_THRESHOLD``.

GPU-specific knobs use a ``FOREMAST_`` prefix (dtype, ring length, season,
Holt-Winters grid, pairwise threshold scale, poll interval).

``bound`` semantics (design decision, docs/SCORING.md): 1 = upper bound only,
2 = lower bound only, 3 = both.
"""

from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, Mapping, Optional

BOUND_UPPER = 1
BOUND_LOWER = 2
BOUND_BOTH = 3

ALGORITHMS = (
    "moving_average", "moving_average_all", "exponential_smoothing",
    "double_exponential_smoothing", "holt_winters", "prophet", "seasonal_decompose",
    "bivariate_normal", "lstm",
)

PAIRWISE_ALGORITHMS = ("ALL", "ANY", "MANN_WHITE", "WILCOXON", "KRUSKAL", "FRIEDMAN", "NONE")


@dataclass
class MetricThreshold:
    threshold: float
    bound: int
    min_lower_bound: float


@dataclass
class BrainConfig:
    es_endpoint: str = ""
    algorithm: str = "moving_average_all"
    threshold: float = 2.0
    bound: int = BOUND_UPPER
    min_lower_bound: float = 0.0
    per_metric: Dict[str, MetricThreshold] = field(default_factory=dict)
    min_mann_white: int = 20
    min_wilcoxon: int = 20
    min_kruskal: int = 5
    min_friedman: int = 5  # complete time blocks (MIN_FRIEDMAN_DATA_POINTS; not in the reference env)
    max_stuck_seconds: float = 90.0
    pairwise_algorithm: str = "ALL"
    pairwise_threshold: float = 0.05
    min_historical_points: int = 60
    max_cache_size: int = 1000
    lstm_threshold: float = 4.0  # z-score of the joint reconstruction error (ML_LSTM_THRESHOLD)
    # resident LSTM engine: |z| of the level term (newest points vs their forecast from the
    # earlier days); <= 0 turns it off (FOREMAST_LSTM_LEVEL_THRESHOLD)
    lstm_level_threshold: float = 5.5
    # downstream impact: joint model over each caller's metrics (ML_DOWNSTREAM_ALGORITHM lstm | none)
    downstream_algorithm: str = "lstm"
    # --- MI355X engine knobs -------------------------------------------------------
    dtype: str = "bf16"
    device: str = "auto"
    ring_len: int = 10080
    season: int = 1440
    ma_window: int = 60
    pairwise_scale: float = 0.5
    # detection semantics (docs/SCORING.md "Band, bound and verdict"): the lowered
    # pairwise band needs this many points outside it (ML_PAIRWISE_MIN_ANOMALIES);
    # per-point thresholds are Sidak-corrected for the window size
    # (FOREMAST_WINDOW_CORRECTION = sidak | none); sigma is scaled to the forecast
    # horizon (FOREMAST_HORIZON_VARIANCE = 1 | 0)
    pairwise_min_points: int = 3
    # mean-shift rule (ML_PAIRWISE_SHIFT, 0 = off; ON by default): when the rank tests say
    # the pods differ, a canary window whose mean lies beyond this many sigmas of the
    # BASELINE pods' mean (not of the forecast) is anomalous even if few of its points
    # leave the window-corrected band.  A departure from the reference brain's per-point
    # band semantics (docs/SCORING.md); set ML_PAIRWISE_SHIFT=0 for the per-point rule only
    pairwise_shift: float = 1.25  # round 6: 1.5 -> 1.25 (docs/SCORING.md, profiles/bench/shift_thr_r6/)
    pairwise_shift_min_points: int = 20  # ML_PAIRWISE_SHIFT_MIN_POINTS (as MIN_MANN_WHITE_DATA_POINTS)
    # the mean-shift rule's spread (ML_PAIRWISE_SHIFT_ONE_STEP = 1 | 0): the model's one-step
    # sigma, not the horizon-scaled band sigma.  The rule compares the canary window with the
    # baseline pods' window over the same minutes, so the forecast's h-step error growth is not
    # part of the comparison (docs/SCORING.md)
    pairwise_shift_one_step: bool = True
    window_correction: str = "sidak"
    horizon_variance: bool = True
    poll_seconds: float = 5.0
    hw_alpha: tuple = (0.1, 0.3, 0.5, 0.8)
    hw_beta: tuple = (0.0, 0.01, 0.05, 0.1)
    hw_gamma: tuple = (0.05, 0.1, 0.3, 0.5)
    lstm_hidden: int = 64
    lstm_window: int = 32
    metrics_port: int = 8000

    def for_metric(self, alias: str, metric_name: str = "") -> MetricThreshold:
        """Threshold / bound / lower clamp for a metric alias
        (exact alias match, then substring match against alias or metric name)."""
        if alias in self.per_metric:
            return self.per_metric[alias]
        for mt, th in self.per_metric.items():
            if mt and (mt in alias or (metric_name and mt in metric_name)):
                return th
        return MetricThreshold(self.threshold, self.bound, self.min_lower_bound)

    @classmethod
    def from_env(cls, env: Optional[Mapping[str, str]] = None) -> "BrainConfig":
        e = dict(os.environ if env is None else env)
        c = cls()

        def f(name, default, conv=float):
            v = e.get(name)
            if v is None or v == "":
                return default
            try:
                return conv(v)
            except ValueError:
                return default

        c.es_endpoint = e.get("ES_ENDPOINT", "")
        c.algorithm = (e.get("ML_ALGORITHM") or c.algorithm).strip().lower()
        c.threshold = f("ML_THRESHOLD", f("threshold", c.threshold))
        c.bound = int(f("ML_BOUND", f("bound", c.bound, int), int))
        c.min_lower_bound = f("min_lower_bound", c.min_lower_bound)
        n = int(f("metric_type_threshold_count", 0, int))
        for i in range(max(n, 0)):
            mt = e.get(f"metric_type{i}")
            if not mt:
                continue
            c.per_metric[mt] = MetricThreshold(
                threshold=f(f"threshold{i}", c.threshold),
                bound=int(f(f"bound{i}", c.bound, int)),
                min_lower_bound=f(f"min_lower_bound{i}", c.min_lower_bound))
        c.min_mann_white = int(f("MIN_MANN_WHITE_DATA_POINTS", c.min_mann_white, int))
        c.min_wilcoxon = int(f("MIN_WILCOXON_DATA_POINTS", c.min_wilcoxon, int))
        c.min_kruskal = int(f("MIN_KRUSKAL_DATA_POINTS", c.min_kruskal, int))
        c.min_friedman = int(f("MIN_FRIEDMAN_DATA_POINTS", c.min_friedman, int))
        c.max_stuck_seconds = f("MAX_STUCK_IN_SECONDS", c.max_stuck_seconds)
        c.pairwise_algorithm = (e.get("ML_PAIRWISE_ALGORITHM") or c.pairwise_algorithm).upper()
        c.pairwise_threshold = f("ML_PAIRWISE_THRESHOLD", c.pairwise_threshold)
        c.min_historical_points = int(f("MIN_HISTORICAL_DATA_POINT_TO_MEASURE",
                                        c.min_historical_points, int))
        c.max_cache_size = int(f("MAX_CACHE_SIZE", c.max_cache_size, int))
        c.lstm_threshold = f("ML_LSTM_THRESHOLD", c.lstm_threshold)
        c.lstm_level_threshold = f("FOREMAST_LSTM_LEVEL_THRESHOLD", c.lstm_level_threshold)
        c.downstream_algorithm = (e.get("ML_DOWNSTREAM_ALGORITHM") or c.downstream_algorithm).strip().lower()
        c.dtype = e.get("FOREMAST_DTYPE", c.dtype)
        c.device = e.get("FOREMAST_DEVICE", c.device)
        c.ring_len = int(f("FOREMAST_RING_LEN", c.ring_len, int))
        c.season = int(f("FOREMAST_SEASON", c.season, int))
        c.ma_window = int(f("FOREMAST_MA_WINDOW", c.ma_window, int))
        c.pairwise_scale = f("FOREMAST_PAIRWISE_SCALE", c.pairwise_scale)
        c.poll_seconds = f("FOREMAST_POLL_SECONDS", c.poll_seconds)
        c.pairwise_min_points = int(f("ML_PAIRWISE_MIN_ANOMALIES", c.pairwise_min_points, int))
        c.pairwise_shift = f("ML_PAIRWISE_SHIFT", c.pairwise_shift)
        c.pairwise_shift_min_points = int(f("ML_PAIRWISE_SHIFT_MIN_POINTS", c.pairwise_shift_min_points, int))
        c.pairwise_shift_one_step = e.get("ML_PAIRWISE_SHIFT_ONE_STEP", "1").strip().lower() not in ("0", "false", "no")
        c.window_correction = (e.get("FOREMAST_WINDOW_CORRECTION") or c.window_correction).strip().lower()
        c.horizon_variance = e.get("FOREMAST_HORIZON_VARIANCE", "1").strip().lower() not in ("0", "false", "no")
        # FOREMAST_DETECTION_PRESET=reference: the reference brain's documented per-point
        # semantics (foremast-brain/README.md:22-38): threshold applied to each point as is (no
        # window correction), a single point outside the lowered band fires, one-step sigma at
        # every horizon.  Explicit variables still override the preset.
        if (e.get("FOREMAST_DETECTION_PRESET") or "").strip().lower() == "reference":
            c.window_correction = (e.get("FOREMAST_WINDOW_CORRECTION") or "none").strip().lower()
            c.pairwise_min_points = int(f("ML_PAIRWISE_MIN_ANOMALIES", 1, int))
            c.horizon_variance = e.get("FOREMAST_HORIZON_VARIANCE", "0").strip().lower() not in ("0", "false", "no")
            c.pairwise_shift = f("ML_PAIRWISE_SHIFT", 0.0)
        c.lstm_hidden = int(f("FOREMAST_LSTM_HIDDEN", c.lstm_hidden, int))
        c.lstm_window = int(f("FOREMAST_LSTM_WINDOW", c.lstm_window, int))
        c.metrics_port = int(f("FOREMAST_METRICS_PORT", c.metrics_port, int))
        for key, attr in (("FOREMAST_HW_ALPHA", "hw_alpha"), ("FOREMAST_HW_BETA", "hw_beta"),
                          ("FOREMAST_HW_GAMMA", "hw_gamma")):
            if e.get(key):
                setattr(c, attr, tuple(float(x) for x in e[key].split(",") if x.strip()))
        return c


def reference_default_env() -> Dict[str, str]:
    """The brain env block shipped in ``deploy/foremast/3_brain/foremast-brain.yaml``."""
    env = {
        "ML_ALGORITHM": "moving_average_all", "threshold": "2.0", "min_lower_bound": "0",
        "bound": "1", "metric_type_threshold_count": "5",
        "MIN_MANN_WHITE_DATA_POINTS": "20", "MIN_WILCOXON_DATA_POINTS": "20",
        "MIN_KRUSKAL_DATA_POINTS": "5", "MAX_STUCK_IN_SECONDS": "90",
    }
    rows = [("error5xx", "2", "1"), ("error4xx", "3", "1"), ("latency", "10", "3"),
            ("cpu", "5", "1"), ("memory", "5", "1")]
    for i, (mt, th, b) in enumerate(rows):
        env[f"metric_type{i}"] = mt
        env[f"threshold{i}"] = th
        env[f"bound{i}"] = b
        env[f"min_lower_bound{i}"] = "0"
    return env
