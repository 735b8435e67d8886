// K6: fused LSTM-autoencoder inference on MFMA (bf16, or fp8 e4m3 OCP on the CDNA4
// block-scaled v_mfma_scale_f32_32x32x64_f8f6f4).
//
// Semantics: foremast_amd/models/lstm_ae.py (encoder LSTM(F→H), decoder with
// zero input starting from the encoder's final (h, c), linear read-out,
// reconstruction MSE → z-score vs calibration → verdict).  H = 64.
//
// Layout (one 64-lane wave = 32 series, a workgroup = 4 waves = 128 series):
//  * gates^T [256 x 32] = Waug^T [256 x 80] · [h; x_t; 1] [80 x 32] on
//    v_mfma_f32_32x32x16_bf16 (8 row tiles x 5 k-steps = 40 MFMAs per step), or in
//    fp8 on v_mfma_scale_f32_32x32x64_f8f6f4 (8 row tiles x 2 k-steps of K = 64 =
//    16 MFMAs per step, an E8M0 scale per (gate row, 32-k block) of the
//    weights).  The input projection and bias ride in the last k-step (x at
//    k=64..64+F-1, bias at k=71), so no VALU matmul is needed for them.
//  * The 256 gate rows are permuted host-side so that in tile t, accumulator
//    register 4*gate+q of lane half hh holds gate `gate` of hidden unit
//    u = 16(t>>1) + 8hh + 4(t&1) + q: each lane has i,f,g,o of its units
//    (cell update is lane-local) AND the new h lands exactly where the next
//    step's B operand needs unit 16s + 8hh + j (s = t>>1, j = 4(t&1)+q) —
//    h never leaves registers across time steps, no LDS transpose.
//  * Weights are pre-packed into A-fragment order [tile][kstep][lane][8] and
//    staged in LDS once per phase (encoder, then decoder): one 16-byte
//    ds_read per MFMA, lane-contiguous (conflict-free).
#include "common.h"
#include "args.h"
#include "lstm_common.h"

struct LstmArgs {
  const float* x;          // [N, T, F] normalised windows
  int N;
  int T;
  int F;                   // 1..7
  int fp8;                 // 0 bf16, 1 fp8 e4m3 (CDNA4 block-scaled MFMA)
  const void* w_enc;       // packed A fragments: bf16 [8][5][64][8]; fp8 [8][2][64][32] e4m3 + [64][16] E8M0
  const void* w_dec;
  const float* w_out;      // [F][64]
  const float* b_out;      // [F]
  float mu;                // calibration
  float sigma;
  const float* threshold;  // [N] or null (→ thr_default)
  float thr_default;
  float* err;              // [N]
  float* zscore;           // [N] or null
  signed char* verdict;    // [N] or null
  float* recon;            // [N, T, F] or null
  const int* app_id;       // [N] or null
  int* app_stats;          // [A, 2] or null
  LstmRingSrc src;         // ring-direct input (x == null)
  float* cal;              // [N, 2] per-series (mu, 1/sigma) of the reconstruction error, or null (global only)
  float cal_ewma;          // > 0: mu_i tracks healthy errors, mu_i += cal_ewma * (err - mu_i) when verdict 0
  const float* zlvl;       // [N, F] level z-scores (lstm_level_kernel) or null
  float thr_level;         // a window is also anomalous when any |zlvl| exceeds this
  int _pad2;
  // fused level term (ring input, one window per row): with lvl_sig the kernel computes the
  // level z of its series itself, in a prologue whose loads the other waves' MFMA work hides
  // (the separate lstm_level_kernel is ~100k tiny waves on the scoring kernel's critical path)
  const float* lvl_sig;    // [N, F] spread of the level statistic, or null
  int lvl_m;               // samples per day
  int lvl_E;               // extra points each side of the earlier days' windows
  int lvl_newest;          // newest column (an offset from src.head_dev when that is set)
  int lvl_avail;           // valid samples in the rings
  float* lvl_out;          // optional [N, F] level z written out, or null
};

// Level term of the LSTM-AE verdict (lstm_level_kernel): the autoencoder scores the SHAPE
// of a z-scored window, so a level shift of a few noise sigmas inside the daily swing is
// weak evidence for it.  The level statistic of (series, feature): the mean of the newest 8
// points minus its forecast from the earlier days — for each day d = 1..D (D <= 7 as the ring
// allows) the mean of the 32 points centred on the same minutes (b_d: 4x the points, and the
// daily profile's slope cancels in a centred window; E = 12 extra minutes each side for a
// 1440-minute day, fewer for short seasons where the profile's curvature would bias it), extrapolated to d = 0 by least squares
// over d (a linear trend across days cancels too; D = 1: b_1).  On a healthy series that is
// ~N(0, sigma^2 (1/8 + ~0.9/32)), so a +3 sigma shift of the newest 7 points is ~6.7 of its own
// spreads.  The spread per (series, feature) is calibrated on the series' own history: the
// RMS of the statistic at K earlier offsets (calibration mode writes the raw statistics).
constexpr int LVL_L = 8;      // newest points averaged
constexpr int LVL_EMAX = 12;  // extra minutes each side of the earlier days' windows (<= 32 points)
struct LevelArgs {
  LstmRingSrc src;   // rings, ld, ring_len, bf16 (start_col / windows unused)
  int N;
  int F;
  int newest;        // physical column of the newest sample
  int avail;         // valid samples in the rings
  int m;             // samples per day
  int L;             // points averaged: LVL_L (checked)
  int E;             // extra points each side of the earlier days' windows, 0..LVL_EMAX
  int K;             // calibration: number of offsets (grid.y); 0: scoring
  int back_step;     // calibration: offset k ends (k + 1) * back_step samples before the newest
  const float* sig;  // scoring: [N, F] spread of the statistic
  float* out;        // scoring: [N, F] z; calibration: [K, N, F] raw statistic (NaN: not enough data)
  const int* head_dev;  // optional device ring head: `newest` is then an offset from it
};

extern __shared__ __attribute__((aligned(16))) char fm_lstm_smem[];

constexpr float CAL_GATE = 2.f;  // per-series z above which an error does not refresh the calibration

namespace {

using namespace fm_lstm;

// Cell update of two gate tiles (lane-local): unit (tt, q) <-> acc[4*gate + q]; packed-FP32
// activation arithmetic, two units per step.
__device__ __forceinline__ void cell_update(const f32x16& acc0, const f32x16& acc1, int tp, float deq,
                                            float (&hreg)[32], float (&creg)[32]) {
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const f32x16& acc = e ? acc1 : acc0;
#pragma unroll
    for (int q = 0; q < 4; q += 2) {
      const f32x2_t gi = (f32x2_t){acc[q], acc[q + 1]} * deq, gf = (f32x2_t){acc[4 + q], acc[5 + q]} * deq;
      const f32x2_t gg = (f32x2_t){acc[8 + q], acc[9 + q]} * deq;
      const f32x2_t go = (f32x2_t){acc[12 + q], acc[13 + q]} * deq;
      const int u = (tp + e) * 4 + q;
      const f32x2_t c = sigm2(gf) * (f32x2_t){creg[u], creg[u + 1]} + sigm2(gi) * tanh2(gg);
      creg[u] = c.x;
      creg[u + 1] = c.y;
      const f32x2_t h = sigm2(go) * tanh2(c);
      hreg[u] = h.x;
      hreg[u + 1] = h.y;
    }
  }
}

// E8M0 scale register (4 scale bytes) and op_sel byte of fp8 fragment (tile, k-step)
template <int TS>
__device__ __forceinline__ f32x16 mfma_fp8(const f8x32& a, const f8x32& b, f32x16 c, const int4& sc, int scale_b) {
  const int sreg = (TS >> 2) == 0 ? sc.x : (TS >> 2) == 1 ? sc.y : (TS >> 2) == 2 ? sc.z : sc.w;
  return mfma_scaled<TS & 3>(a, b, c, sreg, scale_b);
}

// fp8 A fragment i: its two 16-byte halves are stored half-major ([i][half][64 lanes][16 B],
// ops/pack.py fp8_blocks_lane_major), so each ds_read_b128 covers 64 consecutive 16-byte
// slots; a 32-byte lane stride would conflict 2-way on every fragment read.
__device__ __forceinline__ f8x32 frag_fp8(const char* w, int i, int lo) {
  const int4 p = ((const int4*)(w + i * 2048))[lo];
  const int4 q = ((const int4*)(w + i * 2048 + 1024))[lo];
  return (f8x32){p.x, p.y, p.z, p.w, q.x, q.y, q.z, q.w};
}

template <int TP>
__device__ __forceinline__ void gates_fp8(const char* wl, int lo, const f8x32& hb, const f8x32& xb, const int4& sc,
                                          f32x16& acc0, f32x16& acc1) {
  acc0 = mfma_fp8<(TP * KSTEPS_FP8)>(frag_fp8(wl, TP * KSTEPS_FP8, lo), hb, (f32x16){}, sc, SCALE_H);
  acc1 = mfma_fp8<((TP + 1) * KSTEPS_FP8)>(frag_fp8(wl, (TP + 1) * KSTEPS_FP8, lo), hb, (f32x16){}, sc, SCALE_H);
  acc0 = mfma_fp8<(TP * KSTEPS_FP8 + 1)>(frag_fp8(wl, TP * KSTEPS_FP8 + 1, lo), xb, acc0, sc, SCALE_ONE);
  acc1 = mfma_fp8<((TP + 1) * KSTEPS_FP8 + 1)>(frag_fp8(wl, (TP + 1) * KSTEPS_FP8 + 1, lo), xb, acc1, sc, SCALE_ONE);
}

// One LSTM recurrence over T steps for this wave's 32 series.
// ENC: input x_t (and the bias) in the last k-step; DEC: zero input, read-out + error.
// bf16: v_mfma_f32_32x32x16_bf16, 5 k-steps (h: 4, input + bias: 1).  fp8: CDNA4
// v_mfma_scale_f32_32x32x64_f8f6f4 on e4m3 with per-(row, 32-k block) E8M0 weight scales
// (ops/lstm.py pack_fp8), 2 k-steps: the lane's 32 hidden units, then input + bias.
template <bool FP8, bool ENC>
__device__ __forceinline__ void run_phase(const LstmArgs& a, const void* wlds_v, const float* wout_lds,
                                          long long series, bool valid, int hh, float (&hreg)[32],
                                          float (&creg)[32], float& errsum) {
  const int lane = lane_id();
  const XPos xp = make_xpos(a.x, a.src, valid ? series : 0, a.T, a.F);  // tail lanes never index past N
  int4 sc = make_int4(0, 0, 0, 0);
  if constexpr (FP8) sc = ((const int4*)((const char*)wlds_v + FRAG_BYTES_FP8))[lane];
  for (int t = 0; t < a.T; ++t) {
    // the A fragments stay in LDS: an opaque lane offset per step stops the compiler hoisting
    // them (bf16: 40 fragments = 160 VGPRs; fp8: 16 x 8 = 128) out of the time loop
    int lo = lane;
    asm volatile("" : "+v"(lo));
    if constexpr (FP8) {
      const char* wl = (const char*)wlds_v;
      constexpr float HS = (float)(1 << ACT_SHIFT);
      f8x32 hb;
#pragma unroll
      for (int i = 0; i < 8; ++i)
        hb[i] = (int)pack_fp8x4(hreg[4 * i] * HS, hreg[4 * i + 1] * HS, hreg[4 * i + 2] * HS, hreg[4 * i + 3] * HS);
      // input + bias k-step: lane half 0, bytes 0..F-1 and 7; everything else zero
      f8x32 xb = (f8x32){0, 0, 0, 0, 0, 0, 0, 0};
      if (hh == 0) {
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 1.f};
        if (ENC && valid) {
#pragma unroll
          for (int f = 0; f < 7; ++f)
            if (f < a.F) v[f] = sat_fp8(load_x(a.src, xp, t, f, a.F));
        }
        xb[0] = (int)pack_fp8x4(v[0], v[1], v[2], v[3]);
        xb[1] = (int)pack_fp8x4(v[4], v[5], v[6], v[7]);
      }
      f32x16 acc0, acc1;
      gates_fp8<0>(wl, lo, hb, xb, sc, acc0, acc1);
      cell_update(acc0, acc1, 0, 1.f, hreg, creg);
      gates_fp8<2>(wl, lo, hb, xb, sc, acc0, acc1);
      cell_update(acc0, acc1, 2, 1.f, hreg, creg);
      gates_fp8<4>(wl, lo, hb, xb, sc, acc0, acc1);
      cell_update(acc0, acc1, 4, 1.f, hreg, creg);
      gates_fp8<6>(wl, lo, hb, xb, sc, acc0, acc1);
      cell_update(acc0, acc1, 6, 1.f, hreg, creg);
    } else {
      const FragBF16* wlds = (const FragBF16*)wlds_v;
      // B fragments: h (4 k-steps) and the input/bias k-step
      FragBF16 hb[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = hreg[(2 * s + (j >> 2)) * 4 + (j & 3)];
        hb[s] = make_b_bf16(v);
      }
      FragBF16 xb;
      {
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (hh == 0) {
          if (ENC && valid) {
#pragma unroll
            for (int f = 0; f < 7; ++f)
              if (f < a.F) v[f] = load_x(a.src, xp, t, f, a.F);
          }
          v[7] = 1.f;
        }
        xb = make_b_bf16(v);
      }
      // tiles in pairs: two independent accumulator chains, 32 accumulator regs live
#pragma unroll
      for (int tp = 0; tp < TILES; tp += 2) {
        f32x16 acc0 = (f32x16){}, acc1 = (f32x16){};
#pragma unroll
        for (int s = 0; s < KSTEPS; ++s) {
          const FragBF16 bfr = (s < 4) ? hb[s] : xb;
          acc0 = mfma_bf16(wlds[(tp * KSTEPS + s) * 64 + lo], bfr, acc0);
          acc1 = mfma_bf16(wlds[((tp + 1) * KSTEPS + s) * 64 + lo], bfr, acc1);
        }
        cell_update(acc0, acc1, tp, 1.f, hreg, creg);
      }
    }
    if (!ENC) {
      // read-out y_f = sum_u h_u W_out[f][u] + b_out[f]; halves hold 32 units each
#pragma unroll
      for (int f = 0; f < 7; ++f) {
        if (f >= a.F) break;
        float p = 0.f;
#pragma unroll
        for (int tt = 0; tt < TILES; ++tt)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int unit = 16 * (tt >> 1) + 8 * hh + 4 * (tt & 1) + q;
            p += hreg[tt * 4 + q] * wout_lds[f * H + unit];
          }
        p += __shfl_xor(p, 32, FM_WAVE);
        const float y = p + a.b_out[f];
        if (valid && hh == 0) {
          const float d = y - load_x(a.src, xp, t, f, a.F);
          errsum += d * d;
          if (a.recon) a.recon[(series * a.T + t) * a.F + f] = y;
        }
      }
    }
  }
}

// Level z of series n (same statistic as lstm_level_kernel): the two lanes of the series split
// the days (lane half hh: days hh, hh + 2, hh + 4, hh + 6), exchange their day means, and both
// fit the least squares over days 1..D.  Returns max_f |z_f|.  Every lane calls it (the
// exchange is a cross-half shuffle); rows past N compute on row 0 and write nothing.
__device__ __forceinline__ float fused_level_z(const LstmArgs& a, long long n, bool valid, int hh) {
  const LstmRingSrc& s = a.src;
  const int R = s.ring_len, m = a.lvl_m, E = a.lvl_E, W = LVL_L + 2 * E;
  const int newest = s.head_dev ? (s.head_dev[0] + a.lvl_newest) % R : a.lvl_newest;
  const int D = min(7, (a.lvl_avail - (LVL_L + E)) / m);
  const long long row = n * s.ld;
  float zmax = 0.f;
  for (int f = 0; f < a.F; ++f) {
    // a day's points are all loaded before any is summed (fixed trip count, predicated): one
    // memory latency per day window, not one per point
    float bm[4];
#pragma unroll 1
    for (int i = 0; i < 4; ++i) {
      const int d = hh + 2 * i;
      const bool day_ok = D >= 1 && d <= D;
      int col0 = newest - (LVL_L + E - 1) - d * m;
      col0 += col0 < 0 ? R : 0;
      const int p0 = d == 0 ? E : 0, p1 = d == 0 ? E + LVL_L : W;
      float v[2 * LVL_EMAX + LVL_L];
#pragma unroll
      for (int p = 0; p < 2 * LVL_EMAX + LVL_L; ++p) {
        float x = fm_nan();
        if (day_ok && p >= p0 && p < p1) {
          int col = col0 + p;
          col -= col >= R ? R : 0;
          x = s.bf16 ? bf16_to_f32(((const bf16_t*)s.ring[f])[row + col]) : ((const float*)s.ring[f])[row + col];
        }
        v[p] = x;
      }
      float sx = 0.f, cx = 0.f;
#pragma unroll
      for (int p = 0; p < 2 * LVL_EMAX + LVL_L; ++p)
        if (v[p] == v[p]) { sx += v[p]; cx += 1.f; }
      const float mean = cx > 0.f ? sx / cx : fm_nan();
      bm[0] = i == 0 ? mean : bm[0];
      bm[1] = i == 1 ? mean : bm[1];
      bm[2] = i == 2 ? mean : bm[2];
      bm[3] = i == 3 ? mean : bm[3];
    }
    float ob[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) ob[i] = __shfl_xor(bm[i], 32, FM_WAVE);
    // day d's mean: even days from lane half 0, odd days from half 1
    auto day = [&](int d) { const int i = d >> 1; return ((d & 1) == hh) ? bm[i] : ob[i]; };
    const float today = day(0);
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, sb = 0.f, sdb = 0.f;
#pragma unroll
    for (int d = 1; d <= 7; ++d) {
      const float b = day(d);
      if (d <= D && b == b) {
        const float fd = (float)d;
        s0 += 1.f; s1 += fd; s2 += fd * fd; sb += b; sdb += fd * b;
      }
    }
    float st = fm_nan();
    if (s0 > 0.f && today == today) {
      const float dbar = s1 / s0, bbar = sb / s0, sdd = s2 - s1 * dbar;
      const float slope = sdd > 1e-6f ? (sdb - s1 * bbar) / sdd : 0.f;
      st = today - (bbar - slope * dbar);
    }
    const float sg = a.lvl_sig[n * a.F + f];
    const float z = (st == st && sg > 0.f) ? st / sg : 0.f;
    if (valid && hh == 0 && a.lvl_out) a.lvl_out[n * a.F + f] = z;
    zmax = fmaxf(zmax, fabsf(z));
  }
  return zmax;
}

template <bool FP8>
__global__ __launch_bounds__(256, 2) void lstm_ae_kernel(const LstmArgs a) {
  const int w = wave_id(), lane = lane_id();
  const int hh = lane >> 5;
  const long long series = ((long long)blockIdx.x * 4 + w) * 32 + (lane & 31);
  const bool valid = series < a.N;
  const long long sidx = valid ? series : 0;
  constexpr int FB = FP8 ? FRAG_BYTES_FP8 + SCALE_BYTES_FP8 : FRAG_BYTES_BF16;
  float* wout = (float*)(fm_lstm_smem + FB);

  // stage encoder weights (+ fp8 scales) + read-out
  {
    const uint4* src = (const uint4*)a.w_enc;
    uint4* dst = (uint4*)fm_lstm_smem;
    for (int i = threadIdx.x; i < FB / 16; i += blockDim.x) dst[i] = src[i];
    for (int i = threadIdx.x; i < a.F * H; i += blockDim.x) wout[i] = a.w_out[i];
  }
  __syncthreads();
  const float zl_fused = a.lvl_sig ? fused_level_z(a, sidx, valid, hh) : 0.f;
  float hreg[32], creg[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) { hreg[i] = 0.f; creg[i] = 0.f; }
  float errsum = 0.f;
  run_phase<FP8, true>(a, fm_lstm_smem, wout, sidx, valid, hh, hreg, creg, errsum);
  __syncthreads();
  {
    const uint4* src = (const uint4*)a.w_dec;
    uint4* dst = (uint4*)fm_lstm_smem;
    for (int i = threadIdx.x; i < FB / 16; i += blockDim.x) dst[i] = src[i];
  }
  __syncthreads();
  run_phase<FP8, false>(a, fm_lstm_smem, wout, sidx, valid, hh, hreg, creg, errsum);
  if (valid && hh == 0) {
    const float err = errsum / (float)(a.T * a.F);
    a.err[series] = err;
    // global z (error in series-std units vs the pooled healthy level), and
    // with a calibration the smaller of it and the series' own z: a window is
    // anomalous only when it is unusual for its series AND in absolute terms
    float z = (err - a.mu) / fmaxf(a.sigma, 1e-12f);
    float zs = 0.f;  // the series' own z
    if (a.cal) {
      const float2 c = ((const float2*)a.cal)[series];
      zs = (err - c.x) * c.y;
      z = fminf(z, zs);
    }
    if (a.zscore) a.zscore[series] = z;
    const float thr = a.threshold ? a.threshold[series] : a.thr_default;
    float zl = zl_fused;  // level term: the largest |z| of the series' features
    if (a.zlvl)
      for (int f = 0; f < a.F; ++f) zl = fmaxf(zl, fabsf(a.zlvl[series * a.F + f]));
    const int v = (z > thr || zl > a.thr_level) ? 1 : 0;
    if (a.verdict) a.verdict[series] = (signed char)v;
    // healthy windows keep the per-series error level current as the shared
    // model keeps training.  Only windows within CAL_GATE of the series' own
    // level update it: a regression that builds up over several ticks (its
    // first windows still below the verdict threshold) must not be absorbed
    // into the baseline it is judged against.  NaN errors never update it.
    if (a.cal && a.cal_ewma > 0.f && !v && err == err && zs <= CAL_GATE) {
      const float mu = a.cal[2 * series];
      const float nmu = mu + a.cal_ewma * (err - mu);
      a.cal[2 * series] = nmu;
      a.cal[2 * series + 1] *= mu / nmu;  // the dispersion is relative to the level
    }
    if (a.app_id) {
      const int app = a.app_id[series];
      if (v) atomicAdd(&a.app_stats[2 * app], 1);
      atomicAdd(&a.app_stats[2 * app + 1], 1);
    }
  }
}

// one wave per (series, feature): lane = 8 d + q holds points 4q .. 4q+3 of day d's 32-point
// window (today: only the newest 8 of them).  Day sums: two DPP quad butterflies and one
// ds_swizzle (xor 4) inside each 8-lane day group; the eight day means are then read out with
// v_readlane (lanes 0, 8, .., 56) and the least squares over the days runs wave-uniform.  Every
// window of the D <= 7 usable days lies within the newest `avail` samples, so a column needs
// one conditional wrap, not a modulo.
__device__ __forceinline__ float day_sum8(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xf, 0xf, false));  // xor 1
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xf, 0xf, false));  // xor 2
  v += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (4 << 10) | 0x1F));     // xor 4
  return v;
}

__global__ __launch_bounds__(256) void lstm_level_kernel(const LevelArgs a) {
  const long long gw = (long long)blockIdx.x * (blockDim.x / FM_WAVE) + wave_id();
  if (gw >= (long long)a.N * a.F) return;  // wave-uniform
  const int n = (int)(gw / a.F), f = (int)(gw - (long long)n * a.F);
  const int lane = lane_id(), d = lane >> 3, q = lane & 7;
  const int back = a.K > 0 ? ((int)blockIdx.y + 1) * a.back_step : 0;
  const int E = a.E, W = LVL_L + 2 * E;
  const int D = min(7, (a.avail - back - (LVL_L + E)) / a.m);
  const int R = a.src.ring_len;
  // window of day d: points p = 0..W-1 at newest - back - (L + E - 1) + p - d m; today p in [E, E + 8)
  float s = 0.f, c = 0.f;
  if (D >= 1 && d <= D) {
    const long long row = (long long)n * a.src.ld;
    const int newest = a.head_dev ? (a.head_dev[0] + a.newest) % R : a.newest;
    int col0 = newest - back - (LVL_L + E - 1) - d * a.m;
    col0 += col0 < 0 ? R : 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = 4 * q + j;
      if (p >= W || (d == 0 && (p < E || p >= E + LVL_L))) continue;
      int col = col0 + p;
      col -= col >= R ? R : 0;
      const float x = a.src.bf16 ? bf16_to_f32(((const bf16_t*)a.src.ring[f])[row + col])
                                 : ((const float*)a.src.ring[f])[row + col];
      if (x == x) { s += x; c += 1.f; }
    }
  }
  s = day_sum8(s);
  c = day_sum8(c);
  const float mean = c > 0.f ? s / c : fm_nan();  // day d's mean in every lane of its group
  // least squares of the day means b_d over d = 1..D, extrapolated to d = 0 (wave-uniform)
  const float today = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mean), 0));
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, sb = 0.f, sdb = 0.f;
#pragma unroll
  for (int dd = 1; dd <= 7; ++dd) {
    const float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mean), 8 * dd));
    if (dd <= D && b == b) {
      const float fd = (float)dd;
      s0 += 1.f; s1 += fd; s2 += fd * fd; sb += b; sdb += fd * b;
    }
  }
  if (lane != 0) return;
  float st = fm_nan();
  if (s0 > 0.f && today == today) {
    const float dbar = s1 / s0, bbar = sb / s0, sdd = s2 - s1 * dbar;
    const float slope = sdd > 1e-6f ? (sdb - s1 * bbar) / sdd : 0.f;
    st = today - (bbar - slope * dbar);
  }
  if (a.K > 0) {
    a.out[((long long)blockIdx.y * a.N + n) * a.F + f] = st;
  } else {
    const float sg = a.sig[(long long)n * a.F + f];
    a.out[(long long)n * a.F + f] = (st == st && sg > 0.f) ? st / sg : 0.f;
  }
}

}  // namespace

extern "C" int fm_lstm_level(const LevelArgs* a, hipStream_t st) {
  if (a->N <= 0 || a->F <= 0) return 0;
  if (a->F > 7 || a->L != LVL_L || a->E < 0 || a->E > LVL_EMAX || a->m < LVL_L + 2 * a->E || a->K < 0 || a->K > 65535 || (a->K == 0 && !a->sig) ||
      (a->K > 0 && a->back_step < 1) || a->src.ring_len < 1 || a->newest < 0 || a->newest >= a->src.ring_len)
    return (int)hipErrorInvalidValue;
  const long long waves = (long long)a->N * a->F;
  dim3 grid((unsigned)((waves + 3) / 4), (unsigned)(a->K > 0 ? a->K : 1));
  hipLaunchKernelGGL(lstm_level_kernel, grid, dim3(256), 0, st, *a);
  return (int)hipGetLastError();
}

extern "C" long long fm_lstm_level_args_size() { return (long long)sizeof(LevelArgs); }

extern "C" size_t fm_lstm_lds_bytes(int F, int fp8) {
  return (size_t)(fp8 ? FRAG_BYTES_FP8 + SCALE_BYTES_FP8 : FRAG_BYTES_BF16) + (size_t)F * H * 4;
}

extern "C" int fm_lstm_ae(const LstmArgs* a, hipStream_t st) {
  if (a->N <= 0) return 0;
  if (a->F < 1 || a->F > 7 || a->T < 1) return (int)hipErrorInvalidValue;
  if (a->lvl_sig && (!a->src.ring[0] || a->src.win_series || a->lvl_m < LVL_L + 2 * a->lvl_E || a->lvl_E < 0 ||
                     a->lvl_E > LVL_EMAX || a->lvl_newest < 0 || a->lvl_newest >= a->src.ring_len ||
                     a->lvl_avail > a->src.ring_len))
    return (int)hipErrorInvalidValue;
  const size_t lds = fm_lstm_lds_bytes(a->F, a->fp8);
  dim3 grid((unsigned)((a->N + 127) / 128)), block(256);
  if (a->fp8)
    hipLaunchKernelGGL(lstm_ae_kernel<true>, grid, block, lds, st, *a);
  else
    hipLaunchKernelGGL(lstm_ae_kernel<false>, grid, block, lds, st, *a);
  return (int)hipGetLastError();
}

extern "C" long long fm_lstm_args_size() { return (long long)sizeof(LstmArgs); }

// debug helper: convert floats to fp8 e4m3 with the device instruction (for host-side agreement tests)
__global__ void fp8_cvt_kernel(const float* in, unsigned char* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int v = __builtin_amdgcn_cvt_pk_fp8_f32(in[i], 0.f, 0, false);
    out[i] = (unsigned char)(v & 0xff);
  }
}

extern "C" int fm_fp8_convert(const float* in, unsigned char* out, int n, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(fp8_cvt_kernel, dim3((n + 255) / 256), dim3(256), 0, st, in, out, n);
  return (int)hipGetLastError();
}

// Probe of the CDNA4 block-scaled MFMA (v_mfma_scale_f32_32x32x64_f8f6f4, e4m3 A / B): lane l
// loads row (A) / column (B) l & 31, k = 32 (l >> 5) + j into byte j of its 8-VGPR fragment
// (converted on the device), and passes the 32-bit scale registers it is given (sa_reg /
// sb_reg [64]) with op_sel SEL; D [32 x 32] is written with the standard 32x32 C map.
// scripts/probe_mfma_scale.py and tests/test_lstm.py decode which lane / byte scales what.
template <int SEL>
__global__ void mfma_scale_probe_kernel(const float* A, const float* B, const int* sa_reg, const int* sb_reg,
                                        float* D) {
  const int l = threadIdx.x, r = l & 31, hh = l >> 5;
  float av[32], bv[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    av[j] = A[r * 64 + 32 * hh + j];
    bv[j] = B[(32 * hh + j) * 32 + r];
  }
  const fm_lstm::f8x32 af = fm_lstm::pack_fp8x32(av), bf = fm_lstm::pack_fp8x32(bv);
  const f32x16 d = fm_lstm::mfma_scaled<SEL>(af, bf, (f32x16){}, sa_reg[l], sb_reg[l]);
#pragma unroll
  for (int i = 0; i < 16; ++i) D[((i & 3) + 8 * (i >> 2) + 4 * hh) * 32 + r] = d[i];
}

extern "C" int fm_mfma_scale_probe(const float* A, const float* B, const int* sa_reg, const int* sb_reg, float* D,
                                   int sel, hipStream_t st) {
  switch (sel) {
    case 0: hipLaunchKernelGGL(mfma_scale_probe_kernel<0>, dim3(1), dim3(64), 0, st, A, B, sa_reg, sb_reg, D); break;
    case 1: hipLaunchKernelGGL(mfma_scale_probe_kernel<1>, dim3(1), dim3(64), 0, st, A, B, sa_reg, sb_reg, D); break;
    case 2: hipLaunchKernelGGL(mfma_scale_probe_kernel<2>, dim3(1), dim3(64), 0, st, A, B, sa_reg, sb_reg, D); break;
    case 3: hipLaunchKernelGGL(mfma_scale_probe_kernel<3>, dim3(1), dim3(64), 0, st, A, B, sa_reg, sb_reg, D); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}
