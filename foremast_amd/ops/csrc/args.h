// Kernel argument structs (C ABI shared with foremast_amd/ops/_native.py).
//
// Field order/types here and the ctypes Structures in _native.py must agree;
// tests/test_ops_abi.py checks sizeof/offsetof through fm_abi_* exports.
#pragma once
#include <stddef.h>

struct DetectArgs {
  const int* horizons;          // [C] (h_ld = 0) or [N, h_ld]
  long long h_ld;               // horizon row stride; 0 = shared across series
  int C;
  int min_valid;
  const float* cur;             // [N, ld_cur] (NaN = missing) or null
  long long ld_cur;
  const float* threshold;       // [N]
  const signed char* bound;     // [N]
  const float* min_lower;       // [N]
  const unsigned char* differs; // [N] or null
  float pw_scale;               // lowered threshold = threshold * pw_scale (when threshold_low is null)
  int pw_min_points;            // the lowered band applies only with >= this many points beyond it
  const float* threshold_low;   // [N] lowered (pairwise) threshold, or null
  // h-step forecast variance of the fitted smoothing model (null grid: sigma is used
  // unchanged for every horizon).  hv_mode 1 ES, 2 DES, 3 HW (season hv_m)
  const float* hv_grid;         // [G, 3] (alpha, beta, gamma)
  int hv_mode;
  int hv_m;
  float* forecast;              // [N, C] or null
  float* upper;                 // [N, C] or null
  float* lower;                 // [N, C] or null
  int* count;                   // [N]
  signed char* verdict;         // [N]
  float* score;                 // [N]
  const int* app_id;            // [N] or null
  int* app_stats;               // [A, 2] (anomalous, scored) or null
  // K9 compaction (optional): every anomalous (series, column, value) is
  // appended at slot atomicAdd(anom_count, 1) while slot < anom_cap
  int* anom_count;              // [1] (zeroed by the caller) or null
  int* anom_series;             // [anom_cap]
  int* anom_col;                // [anom_cap]
  float* anom_val;              // [anom_cap]
  int anom_cap;
  // > 0: mean-shift rule when differs -- the window's mean of (x - base_mean) / s (canary
  // points against the baseline pods' mean) beyond shift_thr; needs base_mean
  float shift_thr;
  const float* base_mean;       // [N] mean of the baseline pods' window (NaN: none) or null
  int shift_min_points;         // the mean-shift rule needs this many valid canary points
  int shift_one_step;           // 1: the mean-shift rule's spread is the one-step sigma (no horizon factor)
  // per-point thresholds by (class, valid points of the window): the Sidak window
  // correction of models/detect.py window_threshold, tabulated on the host in fp64 (no
  // per-tick fp64 on the device).  Null: threshold / threshold_low as given.
  const float* thr_lut;          // [classes, 2, lut_n] (full, lowered)
  const unsigned short* thr_cls; // [N] class of each series
  int lut_n;                     // valid-point counts covered: 0 .. lut_n - 1 (larger: clamped)
  int last_ncol;                 // columns per pod window (row_out's newest column is in 0 .. last_ncol - 1)
  // per-series record for the host's ONE copy back (or null): verdict, valid points,
  // upper and lower at the newest column clamp(tick_min[0] - start_min[n], 0, last_ncol - 1)
  float* row_out;                // [N, 4]
  const int* start_min;          // [N] minute of each series' first window column
  const int* tick_min;           // [1] newest minute (device scalar: HIP-graph replays read it)
};

struct SmoothArgs {
  const void* hist;     // [N, ld] ring buffer (float or bf16)
  long long ld;         // row stride (elements)
  int ring_len;         // R (physical columns)
  int head;             // physical column of logical t = 0
  int T;                // logical window length
  int Tp;               // padded length (multiple of seg)
  int pad;              // front padding (Tp - T)
  int m;                // season (HW) or 1
  int K;                // steps per lane per segment
  int seg;              // segment length (HW: m; ES/DES: 64*K)
  const float* grid;    // [G, 3] (alpha, beta, gamma)
  int G;
  int N;
  float* level;         // [N]
  float* trend;         // [N]
  float* sigma;         // [N]
  int* best;            // [N]
  float* season_out;    // [N, m] or null
  const float* pair_tab;  // per combo-pair precomputed table (hw_scan variant 3) or null
  DetectArgs det;
  const int* head_dev;  // HW variants 4/5: if set, `head` is read from device memory (HIP-graph replays)
  // HW variants 4/5, deferred detection (det.C = 0 at fit time): the fit writes the
  // seasonal terms of the first HALF_HB forecast phases and the valid-sample count, and
  // fm_hw_detect_params runs the band/verdict epilogue later (after the rank tests,
  // which then overlap the fit on another stream)
  float* season_hb;     // [N, 16] or null
  float* nvalid_out;    // [N] or null
};

struct RankArgs {
  const float* base;
  long long ld_base;
  const float* cur;
  long long ld_cur;
  int nb;
  int nc;
  int N;
  int mode;       // 0 none, 1 ALL, 2 ANY, 3 MW, 4 WILCOXON, 5 KRUSKAL, 6 FRIEDMAN
  float alpha;
  int min_mw;
  int min_wilcoxon;
  int min_kruskal;
  float* pvals;            // [N, 3] (mw, wilcoxon, kruskal) or null
  unsigned char* differs;  // [N]
  float* counts;           // [N, 3] (n_base, n_cur, n_pairs) or null
  // Friedman chi-square over time blocks x pods: the windows are pod-major
  // ([pods_b][nb / pods_b] and [pods_c][nc / pods_c], slot-aligned)
  int pods_b;
  int pods_c;
  int min_friedman;        // complete blocks needed
  float* p_friedman;       // [N, 2] (p, complete blocks) or null; computed when set or mode == 6
  float* base_mean;        // [N] mean of the valid baseline values (NaN if none) or null
  // > 0: two-sided normal quantile of alpha (isf(alpha / 2), fp64 on the host).  Without
  // pvals, MW / Wilcoxon / Kruskal decide by |z| > z_crit (H > z_crit^2) -- no erfc
  float z_crit;
  int _pad;
};

struct WindowArgs {
  const void* hist;
  long long ld;
  int ring_len;
  int head;      // physical column of the first sample of the window
  int len;       // window length (logical samples)
  int N;
  float* mean;   // [N]
  float* stdv;   // [N]
  float* count;  // [N]
  DetectArgs det;
};

struct BivArgs {
  const void* hx;       // [N, ld] metric 0 ring
  const void* hy;       // [N, ld] metric 1 ring
  long long ld;
  int ring_len;
  int head;
  int len;
  int N;
  const float* cur;     // [N, C, 2]
  int C;
  int min_valid;
  const float* threshold;       // [N]
  const unsigned char* differs; // [N] or null
  float pw_scale;
  float eps;
  float* mean;          // [N, 2]
  float* cov;           // [N, 3]
  float* d2;            // [N, C] or null
  int* count;           // [N]
  signed char* verdict; // [N]
  float* score;         // [N] max d
  const int* app_id;
  int* app_stats;
};
