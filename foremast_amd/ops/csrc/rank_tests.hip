// K5 + K11: batched Mann-Whitney U / Wilcoxon signed-rank / Kruskal-Wallis /
// Friedman chi-square and the pairwise "do baseline and current differ" decision
// (docs/guides/design.md:89-92 of the reference lists the four tests).
//
// Semantics: foremast_amd/models/pairwise.py (scipy asymptotic forms).
// One 64-lane wave per series; four series per 256-thread workgroup.  The
// pooled sample (n <= 1024) is staged in the wave's LDS slice and ranked by
// exact pairwise counting: rank_i = #(x_j < x_i) + (#(x_j == x_i) + 1) / 2,
// which gives average ranks under ties and the tie term sum(t^3 - t) =
// sum_i (eq_i^2 - 1) in the same sweep.  All lanes read the same x_j per
// iteration (an LDS broadcast), so the sweep is conflict-free.  For canary
// windows (n ~ 20-200) this beats a sort: no data-dependent control flow.
//
// Small windows (nb, nc <= 64: the product's 5 pods x 11 minutes = 55 per side) take a
// sort-and-scan path instead (rank_tests_kernel<true>): each lane holds ONE baseline,
// ONE canary and ONE |d| key; the three 64-key arrays are sorted together by a register
// bitonic network (21 steps of one exchange + one v_med3_u32 per array), and every
// statistic is summed per run of equal keys at the run's last lane (run starts by a
// DPP max-scan): R1 from n1 (n1 + 1) / 2 plus the baseline runs' canary counts (one
// lower / upper bound search in the sorted canary keys), the pooled tie term from the
// runs' lengths, Wilcoxon's rank sums from run positions and a prefix count of the
// positive differences.  Integer and exact; ~100 us per 100k rows where the sweep below
// takes 250 (scripts/bench_rank.py).
#include "common.h"
#include <stdlib.h>
#include "args.h"



extern __shared__ __attribute__((aligned(16))) char fm_rank_smem[];

// Rank the valid entries of x[0..n) (NaN = invalid); returns per-lane partial
// sums: sum of ranks for entries with group flag set, and the tie term.
template <typename GroupFn>
__device__ __forceinline__ void rank_sweep(const float* x, int n, GroupFn in_group,
                                           float& rsum_g, float& tie, float& rsum_o) {
  const int lane = lane_id();
  rsum_g = 0.f; rsum_o = 0.f; tie = 0.f;
  for (int i = lane; i < n; i += FM_WAVE) {
    const float xi = x[i];
    if (xi != xi) continue;
    // integer counters: each comparison is one v_cmp into VCC plus one add-with-carry
    int less = 0, eq = 0;
    int j = 0;
    for (; j + 4 <= n; j += 4) {
      const v4f q = *(const v4f*)(x + j);
      less += (q.x < xi); eq += (q.x == xi);
      less += (q.y < xi); eq += (q.y == xi);
      less += (q.z < xi); eq += (q.z == xi);
      less += (q.w < xi); eq += (q.w == xi);
    }
    for (; j < n; ++j) {
      const float q = x[j];
      less += (q < xi);
      eq += (q == xi);
    }
    const float r = (float)less + ((float)eq + 1.f) * 0.5f;
    if (in_group(i)) rsum_g += r; else rsum_o += r;
    tie += (float)(eq * eq - 1);
  }
  rsum_g = wave_sum(rsum_g);
  rsum_o = wave_sum(rsum_o);
  tie = wave_sum(tie);
}

// Upper tail of chi^2 with integer dof nu: Q(nu/2, x/2) by the finite series of the
// regularised incomplete gamma at integer / half-integer order.
__device__ __forceinline__ float chi2_sf(float x, int nu) {
  if (!(x > 0.f)) return 1.f;
  const float h = 0.5f * x;
  float sum = 0.f;
  if ((nu & 1) == 0) {
    float term = 1.f;
    for (int i = 0; i < nu / 2; ++i) {
      sum += term;
      term *= h / (float)(i + 1);
    }
    return fminf(expf(-h) * sum, 1.f);
  }
  float term = sqrtf(h) * 1.1283791670955126f;  // h^(1/2) / Gamma(3/2)
  for (int i = 1; i <= (nu - 1) / 2; ++i) {
    sum += term;
    term *= h / ((float)i + 0.5f);
  }
  return fminf(erfcf(sqrtf(h)) + expf(-h) * sum, 1.f);
}

// Friedman chi-square over time blocks (window slots present in every pod) x
// treatments (baseline pods, then canary pods): ranks within each complete
// block (ties averaged), rank sums per treatment accumulated in LDS, tie-
// corrected statistic, chi^2 with k - 1 dof.  One lane per block.
__device__ __forceinline__ void friedman_wave(const RankArgs& a, const float* x, float* R, float& p_out,
                                              float& nblk_out) {
  const int lane = lane_id();
  const int Pb = a.pods_b, Pc = a.pods_c, k = Pb + Pc;
  const int Wb = a.nb / Pb, Wc = a.nc / Pc;
  const int nbk = Wb < Wc ? Wb : Wc;
  auto val = [&](int t, int j) { return t < Pb ? x[t * Wb + j] : x[a.nb + (t - Pb) * Wc + j]; };
  if (lane < k) R[lane] = 0.f;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  float cnt = 0.f, tie = 0.f;
  for (int j = lane; j < nbk; j += FM_WAVE) {
    bool ok = true;
    for (int t = 0; t < k; ++t) {
      const float v = val(t, j);
      ok = ok && (v == v);
    }
    if (!ok) continue;
    cnt += 1.f;
    for (int t = 0; t < k; ++t) {
      const float vt = val(t, j);
      float less = 0.f, eq = 0.f;
      for (int u = 0; u < k; ++u) {
        const float vu = val(u, j);
        less += (vu < vt) ? 1.f : 0.f;
        eq += (vu == vt) ? 1.f : 0.f;
      }
      atomicAdd(&R[t], less + (eq + 1.f) * 0.5f);
      tie += eq * eq - 1.f;  // summed over a block's members = sum over tie groups of t^3 - t
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  const float r = lane < k ? R[lane] : 0.f;
  const float ssq = wave_sum(r * r);
  const float nb = wave_sum(cnt);
  tie = wave_sum(tie);
  nblk_out = nb;
  p_out = 1.f;
  if (nb > 0.f && k >= 2) {
    const float fk = (float)k;
    const float chi = 12.f / (nb * fk * (fk + 1.f)) * ssq - 3.f * nb * (fk + 1.f);
    const float c = 1.f - tie / (nb * fk * (fk * fk - 1.f));
    if (c > 0.f) p_out = chi2_sf(fmaxf(chi / c, 0.f), k - 1);
  }
}

// ---- small-window path: register bitonic sort, run scans, one cross search -------------
// All three arrays are sorted as monotone u32 keys: a float v maps to its bit pattern
// with the sign bit flipped (negatives: all bits), -0 folded onto +0; the |d| array is
// keyed (bits(|d|) << 1) | (d > 0) so equal magnitudes stay adjacent whatever their
// signs.  Padding is 0xffffffff, above every key.
__device__ __forceinline__ unsigned fkey(float v) {
  const unsigned u = __float_as_uint(v == 0.f ? 0.f : v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ unsigned med3u(unsigned a, unsigned b, unsigned c) {
  unsigned r;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// lane ^ J exchange: DPP quad permutes for 1 / 2, ds_swizzle (bit mode, 32-lane groups)
// for 4..16, a bpermute for 32.
template <int J>
__device__ __forceinline__ unsigned xor_lane(unsigned v) {
  const int x = (int)v;
  if constexpr (J == 1) return (unsigned)__builtin_amdgcn_mov_dpp(x, 0xB1, 0xf, 0xf, false);
  else if constexpr (J == 2) return (unsigned)__builtin_amdgcn_mov_dpp(x, 0x4E, 0xf, 0xf, false);
  else if constexpr (J < 32) return (unsigned)__builtin_amdgcn_ds_swizzle(x, (J << 10) | 0x1F);
  else return (unsigned)__shfl_xor(x, 32, FM_WAVE);
}

// One compare-exchange step of the bitonic network on three arrays: med3(a, partner, 0)
// is the min and med3(a, partner, ~0) the max, so a step is one VALU per array plus the
// exchange; the direction mask is shared.
template <int K, int J>
__device__ __forceinline__ void bitonic_step3(unsigned& a, unsigned& b, unsigned& c, int lane) {
  const bool take_min = ((lane & J) == 0) == ((lane & K) == 0);
  const unsigned sel = take_min ? 0u : ~0u;
  const unsigned pa = xor_lane<J>(a), pb = xor_lane<J>(b), pc = xor_lane<J>(c);
  a = med3u(a, pa, sel);
  b = med3u(b, pb, sel);
  c = med3u(c, pc, sel);
}

template <int K, int J>
__device__ __forceinline__ void bitonic_merge3(unsigned& a, unsigned& b, unsigned& c, int lane) {
  bitonic_step3<K, J>(a, b, c, lane);
  if constexpr (J > 1) bitonic_merge3<K, J / 2>(a, b, c, lane);
}

template <int K>
__device__ __forceinline__ void bitonic_sort3(unsigned& a, unsigned& b, unsigned& c, int lane) {
  if constexpr (K > 2) bitonic_sort3<K / 2>(a, b, c, lane);
  bitonic_merge3<K, K / 2>(a, b, c, lane);
}

// inclusive lane-order scan (sum or max; every value >= 0) by DPP row shifts + row broadcasts
template <bool MAX>
__device__ __forceinline__ int wave_scan_i(int v) {
#define FM_SCAN_STEP(C, RM)                                              \
  {                                                                      \
    const int t = __builtin_amdgcn_update_dpp(0, v, C, RM, 0xf, false); \
    v = MAX ? max(v, t) : v + t;                                         \
  }
  FM_SCAN_STEP(0x111, 0xf) FM_SCAN_STEP(0x112, 0xf) FM_SCAN_STEP(0x114, 0xf) FM_SCAN_STEP(0x118, 0xf)
  FM_SCAN_STEP(0x142, 0xa) FM_SCAN_STEP(0x143, 0xc)
#undef FM_SCAN_STEP
  return v;
}

// neighbour keys in lane order (wave_shr:1 / wave_shl:1); the edge lanes get ``edge``
__device__ __forceinline__ unsigned prev_lane(unsigned v, unsigned edge) {
  return (unsigned)__builtin_amdgcn_update_dpp((int)edge, (int)v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ unsigned next_lane(unsigned v, unsigned edge) {
  return (unsigned)__builtin_amdgcn_update_dpp((int)edge, (int)v, 0x130, 0xf, 0xf, false);
}

// Keys of the ascending 64-array s that are < v (LE: <= v).
template <bool LE>
__device__ __forceinline__ int bound64(const unsigned* s, unsigned v) {
  int pos = 0;
#pragma unroll
  for (int h = 32; h > 0; h >>= 1) {
    const unsigned q = s[pos + h - 1];
    pos += (LE ? q <= v : q < v) ? h : 0;
  }
  const unsigned q = s[pos];
  return pos + ((LE ? q <= v : q < v) ? 1 : 0);
}

// Pooled-rank statistics of the small path (returned wave-uniform): baseline rank sum
// R1, pooled tie term sum(t^3 - t), Wilcoxon positive / negative rank sums and its tie
// term.  bv / cv / dv: this lane's baseline, canary and signed difference (NaN: none).
//
// Everything is counted per RUN of equal keys in the sorted arrays, at the run's last
// lane: its first lane f comes from a max-scan of run starts, its length t = i - f + 1.
//  * R1 = n1 (n1 + 1) / 2 + U1 (ranks within the baseline sum to that whatever the ties),
//    U1 = sum over baseline runs of t_b (#(c < v) + #(c == v) / 2): one lower / upper
//    bound search of the run's key in the sorted canary keys (LDS).
//  * pooled ties: (t_b + t_c)^3 - (t_b + t_c) = (t_b^3 - t_b) + (t_c^3 - t_c)
//    + 3 t_b t_c (t_b + t_c): baseline runs add the first and last terms (t_c from the
//    same search), canary runs their own t_c^3 - t_c.
//  * Wilcoxon: a |d| run starting at f of length t holds average rank f + (t + 1) / 2;
//    its positive members are counted by a prefix sum carried through the run-start scan.
// All integer: exact, and independent of the summation order.
__device__ __forceinline__ void small_ranks(float bv, float cv, float dv, unsigned* s, int lane, int n1, int n2, int nd,
                                            float& R1, float& tie, float& Tp, float& Tm, float& wtie) {
  const unsigned PAD = ~0u;
  const float ad = fabsf(dv);
  unsigned kb = bv == bv ? fkey(bv) : PAD, kc = cv == cv ? fkey(cv) : PAD;
  unsigned kd = ad == ad ? ((__float_as_uint(ad) << 1) | (dv > 0.f ? 1u : 0u)) : PAD;
  bitonic_sort3<64>(kb, kc, kd, lane);
  s[lane] = kc;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  const unsigned vd = kd >> 1;
  // run starts / ends (the edge values differ from every key of their array)
  const bool sb_ = kb != prev_lane(kb, ~kb), eb = kb != next_lane(kb, ~kb);
  const bool sc_ = kc != prev_lane(kc, ~kc), ec = kc != next_lane(kc, ~kc);
  const bool sd_ = vd != prev_lane(vd, ~vd), ed = vd != next_lane(vd, ~vd);
  const int pos = (lane < nd && (kd & 1u)) ? 1 : 0;
  const int P = wave_scan_i<false>(pos);
  const int fb = wave_scan_i<true>(sb_ ? lane : 0);
  const int fc = wave_scan_i<true>(sc_ ? lane : 0);
  const int fd = wave_scan_i<true>(sd_ ? (lane << 8) | (P - pos) : 0);
  int u1x2 = 0, tpx2 = 0, t = 0, wt = 0;
  if (lane < n1 && eb) {
    const int tb = lane - fb + 1;
    const int lc = bound64<false>(s, kb), tc = bound64<true>(s, kb) - lc;
    u1x2 = tb * (2 * lc + tc);
    t = tb * tb * tb - tb + 3 * tb * tc * (tb + tc);
  }
  if (lane < n2 && ec) {
    const int tc = lane - fc + 1;
    t += tc * tc * tc - tc;
  }
  if (lane < nd && ed) {
    const int f = fd >> 8, td = lane - f + 1, npos = P - (fd & 0xff);
    tpx2 = npos * (2 * f + td + 1);
    wt = td * td * td - td;
  }
  // 2 U1 <= 8192 and 2 Tp <= 4160 share one exact reduction; Tm = np (np + 1) / 2 - Tp
  const int rr = wave_allsum_i(u1x2 | (tpx2 << 16));
  R1 = 0.5f * (float)(n1 * (n1 + 1) + (rr & 0xffff));
  Tp = 0.5f * (float)(rr >> 16);
  Tm = 0.5f * (float)(nd * (nd + 1)) - Tp;
  tie = (float)wave_allsum_i(t);
  wtie = (float)wave_allsum_i(wt);
}

// The three two-sample tests as z statistics, shared by the p-value and the decisions-only
// forms (so their verdicts agree by construction):
//  * Mann-Whitney: |U1 - n1 n2 / 2| with the tie-corrected sd; two-sided with continuity
//    correction, p = 2 sf((|U1 - mu| - 1/2) / sd).
//  * Kruskal-Wallis of two groups is the same statistic squared without the continuity
//    correction: H = 12 D^2 / ((n + 1) n1 n2) with D = R1 - n1 (n + 1) / 2 = U1 - n1 n2 / 2,
//    and its tie correction 1 - T / (n^3 - n) turns (n + 1) n1 n2 / 12 into the MW variance,
//    so H / corr = (U1 - mu)^2 / var and p = erfc(sqrt(H / corr / 2)) = 2 sf(|U1 - mu| / sd).
//    (The textbook form 12 / (n (n + 1)) sum R_i^2 / n_i - 3 (n + 1) subtracts two ~3 (n + 1)
//    terms; near H = 0 its fp32 rounding moved p by up to 3e-3.)
//  * Wilcoxon signed rank: |T - np (np + 1) / 4| with its tie-corrected sd.
struct RankZ {
  float dU, sd_u, dT, sd_t;
};
__device__ __forceinline__ RankZ rank_z(float R1, float tie, float Tp, float Tm, float wtie, float n1, float n2,
                                        float np) {
  RankZ z;
  const float nn = n1 + n2, nm = n1 * n2;
  z.dU = fabsf(R1 - n1 * (n1 + 1.f) * 0.5f - nm * 0.5f);
  const float var = nm * (1.f / 12.f) * ((nn + 1.f) - tie / fmaxf(nn * (nn - 1.f), 1.f));
  z.sd_u = (n1 > 0.f && n2 > 0.f) ? sqrtf(fmaxf(var, 0.f)) : 0.f;
  z.dT = fabsf(fminf(Tp, Tm) - np * (np + 1.f) * 0.25f);
  const float wvar = np * (np + 1.f) * (2.f * np + 1.f) * (1.f / 24.f) - wtie * (1.f / 48.f);
  z.sd_t = np > 0.f ? sqrtf(fmaxf(wvar, 0.f)) : 0.f;
  return z;
}

template <bool SMALL>
__global__ __launch_bounds__(256) void rank_tests_kernel(const RankArgs a) {
  const int w = wave_id(), lane = lane_id();
  const int n = blockIdx.x * (blockDim.x / FM_WAVE) + w;
  const int npool = a.nb + a.nc;
  const int npool4 = (npool + 3) & ~3;
  const int k = a.nb < a.nc ? a.nb : a.nc;
  const int k4 = (k + 3) & ~3;
  const int small_sz = SMALL ? FM_WAVE : 0;
  float* x = (float*)fm_rank_smem + (size_t)w * (small_sz + npool4 + k4 + FM_WAVE) + small_sz;
  float* dabs = x + npool4;
  float* Rf = dabs + k4;  // Friedman rank sums (<= 64 treatments)
  if (n >= a.N) return;  // wave-uniform; no block barrier below
  const float* b = a.base + (long long)n * a.ld_base;
  const float* c = a.cur + (long long)n * a.ld_cur;
  const bool want_fr = a.mode == 6 || a.p_friedman != nullptr;
  float R1, tie, R2, Tp, wtie, Tm, n1, n2, np, sb;  // R2: the sweep's (the tests need R1 only)
  float p_fr = 1.f, nblk = 0.f;
  if constexpr (SMALL) {
    const float bv = lane < a.nb ? b[lane] : fm_nan();
    const float cv = lane < a.nc ? c[lane] : fm_nan();
    float dv = fm_nan();
    if (lane < k) {
      const float d = cv - bv;
      if (d == d && d != 0.f) dv = d;
    }
    // one exact integer reduction for the three counts (7 bits each)
    const int cnt = wave_allsum_i((bv == bv ? 1 : 0) | (cv == cv ? 1 << 8 : 0) | (dv == dv ? 1 << 16 : 0));
    n1 = (float)(cnt & 0xff);
    n2 = (float)((cnt >> 8) & 0xff);
    np = (float)((cnt >> 16) & 0xff);
    sb = a.base_mean ? wave_allsum(bv == bv ? bv : 0.f) : 0.f;
    if (want_fr) {  // Friedman reads the pooled windows staged as the sweep stages them
      for (int i = lane; i < npool4; i += FM_WAVE) x[i] = i < a.nb ? b[i] : (i < npool ? c[i - a.nb] : fm_nan());
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      friedman_wave(a, x, Rf, p_fr, nblk);
    }
    small_ranks(bv, cv, dv, (unsigned*)(x - small_sz), lane, (int)n1, (int)n2, (int)np, R1, tie, Tp, Tm, wtie);
  } else {

  // stage pooled sample (NaN pads the vector tail) and |d| of aligned pairs
  float cnt_b = 0.f, cnt_c = 0.f, sum_b = 0.f;
  for (int i = lane; i < npool4; i += FM_WAVE) {
    float v = fm_nan();
    if (i < a.nb) v = b[i];
    else if (i < npool) v = c[i - a.nb];
    x[i] = v;
    if (v == v) {
      if (i < a.nb) { cnt_b += 1.f; sum_b += v; }
      else cnt_c += 1.f;
    }
  }
  float npairs = 0.f;
  for (int i = lane; i < k4; i += FM_WAVE) {
    float v = fm_nan();
    if (i < k) {
      const float d = c[i] - b[i];
      if (d == d && d != 0.f) { v = fabsf(d); npairs += 1.f; }
    }
    dabs[i] = v;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  n1 = wave_sum(cnt_b);
  n2 = wave_sum(cnt_c);
  np = wave_sum(npairs);
  sb = a.base_mean ? wave_sum(sum_b) : 0.f;

  // --- Friedman (time blocks x pods) on the staged windows
  if (want_fr) friedman_wave(a, x, Rf, p_fr, nblk);

  // --- MW / Kruskal share the pooled ranks
  const int nbv = a.nb;
  rank_sweep(x, npool4, [nbv](int i) { return i < nbv; }, R1, tie, R2);

  // --- Wilcoxon: ranks of |d| over nonzero pairs, group = positive d
  rank_sweep(dabs, k4, [c, b](int i) { return (c[i] - b[i]) > 0.f; }, Tp, wtie, Tm);
  }
  const float nn = n1 + n2;

  if (lane != 0) return;
  if (!a.pvals && a.z_crit > 0.f && a.mode >= 1 && a.mode <= 5) {
    // decisions only (the product tick): p < alpha <=> |z| > z_crit, no erfc
    const float zc = a.z_crit;
    const RankZ z = rank_z(R1, tie, Tp, Tm, wtie, n1, n2, np);
    bool rej_mw = z.sd_u > 0.f && z.dU - 0.5f > zc * z.sd_u;
    bool rej_k = z.sd_u > 0.f && z.dU > zc * z.sd_u;
    bool rej_w = z.sd_t > 0.f && z.dT > zc * z.sd_t;
    const float nsmall = fminf(n1, n2);
    const bool ran_mw = nsmall >= (float)a.min_mw, ran_w = np >= (float)a.min_wilcoxon;
    const bool ran_k = nsmall >= (float)a.min_kruskal;
    rej_mw &= ran_mw;
    rej_w &= ran_w;
    rej_k &= ran_k;
    bool d = false;
    switch (a.mode) {
      case 1: d = (ran_mw || ran_w || ran_k) && (!ran_mw || rej_mw) && (!ran_w || rej_w) && (!ran_k || rej_k); break;
      case 2: d = rej_mw || rej_w || rej_k; break;
      case 3: d = rej_mw; break;
      case 4: d = rej_w; break;
      default: d = rej_k; break;
    }
    a.differs[n] = d ? 1 : 0;
    if (a.base_mean) a.base_mean[n] = n1 > 0.f ? sb / n1 : fm_nan();
    if (a.p_friedman) {
      a.p_friedman[2 * (long long)n + 0] = p_fr;
      a.p_friedman[2 * (long long)n + 1] = nblk;
    }
    if (a.counts) {
      a.counts[3 * (long long)n + 0] = n1;
      a.counts[3 * (long long)n + 1] = n2;
      a.counts[3 * (long long)n + 2] = np;
    }
    return;
  }
  // Mann-Whitney U (two-sided, continuity, tie-corrected), Kruskal-Wallis (2 groups, chi^2(1)),
  // Wilcoxon signed rank (no continuity correction): see rank_z
  const RankZ z = rank_z(R1, tie, Tp, Tm, wtie, n1, n2, np);
  const float p_mw = z.sd_u > 0.f ? fminf(2.f * norm_sf((z.dU - 0.5f) / z.sd_u), 1.f) : 1.f;
  const float p_kw = z.sd_u > 0.f ? fminf(2.f * norm_sf(z.dU / z.sd_u), 1.f) : 1.f;
  const float p_w = z.sd_t > 0.f ? fminf(2.f * norm_sf(z.dT / z.sd_t), 1.f) : 1.f;
  const float nsmall = fminf(n1, n2);
  const bool ran_mw = nsmall >= (float)a.min_mw;
  const bool ran_w = np >= (float)a.min_wilcoxon;
  const bool ran_k = nsmall >= (float)a.min_kruskal;
  const bool rej_mw = ran_mw && p_mw < a.alpha;
  const bool rej_w = ran_w && p_w < a.alpha;
  const bool rej_k = ran_k && p_kw < a.alpha;
  bool d = false;
  switch (a.mode) {
    case 1: d = (ran_mw || ran_w || ran_k) && (!ran_mw || rej_mw) && (!ran_w || rej_w) && (!ran_k || rej_k); break;
    case 2: d = rej_mw || rej_w || rej_k; break;
    case 3: d = rej_mw; break;
    case 4: d = rej_w; break;
    case 5: d = rej_k; break;
    case 6: d = nblk >= (float)a.min_friedman && p_fr < a.alpha; break;
    default: d = false;
  }
  a.differs[n] = d ? 1 : 0;
  if (a.base_mean) a.base_mean[n] = n1 > 0.f ? sb / n1 : fm_nan();
  if (a.p_friedman) {
    a.p_friedman[2 * (long long)n + 0] = p_fr;
    a.p_friedman[2 * (long long)n + 1] = nblk;
  }
  if (a.pvals) {
    a.pvals[3 * (long long)n + 0] = p_mw;
    a.pvals[3 * (long long)n + 1] = p_w;
    a.pvals[3 * (long long)n + 2] = p_kw;
  }
  if (a.counts) {
    a.counts[3 * (long long)n + 0] = n1;
    a.counts[3 * (long long)n + 1] = n2;
    a.counts[3 * (long long)n + 2] = np;
  }
}

static bool rank_small(int nb, int nc) {
  return nb <= FM_WAVE && nc <= FM_WAVE && !getenv("FOREMAST_RANK_SWEEP");
}

extern "C" size_t fm_rank_lds_bytes(int nb, int nc) {
  const int npool4 = (nb + nc + 3) & ~3;
  const int k = nb < nc ? nb : nc;
  const int k4 = (k + 3) & ~3;
  const int small_sz = rank_small(nb, nc) ? FM_WAVE : 0;
  return (size_t)4 * (small_sz + npool4 + k4 + FM_WAVE) * 4;
}

extern "C" int fm_rank_tests(const RankArgs* a, hipStream_t st) {
  if (a->N <= 0) return 0;
  const size_t lds = fm_rank_lds_bytes(a->nb, a->nc);
  if (lds > 64 * 1024 || a->nb <= 0 || a->nc <= 0) return (int)hipErrorInvalidValue;
  if ((a->mode == 6 || a->p_friedman) &&
      (a->pods_b <= 0 || a->pods_c <= 0 || a->nb % a->pods_b || a->nc % a->pods_c || a->pods_b + a->pods_c > FM_WAVE))
    return (int)hipErrorInvalidValue;
  dim3 grid((a->N + 3) / 4), block(256);
  if (rank_small(a->nb, a->nc))
    hipLaunchKernelGGL(rank_tests_kernel<true>, grid, block, lds, st, *a);
  else
    hipLaunchKernelGGL(rank_tests_kernel<false>, grid, block, lds, st, *a);
  return (int)hipGetLastError();
}
