// K2/K3 fast path: branch-free time-parallel smoothing fit for geometries
// where every active lane owns exactly K steps of a segment (seg = L*K,
// L <= 64), e.g. Holt-Winters with a daily season of 1440 = 60 lanes x 24.
//
// Same semantics and outputs as smooth_fit_kernel (smoothing.hip); what
// differs is the schedule:
//  * the staged series lives in LDS lane-chunked ([seg][64][KP]) so each
//    lane pulls its K values of a segment with 16-byte ds_reads
//    (48-byte lane stride for K=24 bf16: conflict-free);
//  * the per-step loops carry no per-lane guards (idle lanes >= L compute
//    garbage that is masked once per segment), so a whole segment is one
//    basic block the scheduler can interleave;
//  * pass 1 of season k+1 (its local affine map, which needs season k's
//    updated seasonal state) is fused into pass 2 of season k: two
//    independent dependency chains per step;
//  * the cross-lane affine scan uses DPP (row_shr 1/2/4/8, row_bcast 15/31,
//    wave_shr 1) instead of LDS permutes, end-of-segment state is a
//    v_readlane;
//  * per-wave best seasonal state is kept in LDS, not registers.
#include "common.h"
#include "detect.h"
#include "args.h"

#include <cstdlib>
#include <type_traits>

extern __shared__ __attribute__((aligned(16))) char fm_hw_smem[];

namespace {

enum { MODE_ES = 0, MODE_DES = 1, MODE_HW = 2 };

template <int CTRL, int RM>
__device__ __forceinline__ float dppf(float old, float src) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src), CTRL, RM, 0xf, false));
}
template <int CTRL, int RM>
__device__ __forceinline__ v2f dpp2(float old, v2f src) {
  v2f r;
  r.x = dppf<CTRL, RM>(old, src.x);
  r.y = dppf<CTRL, RM>(old, src.y);
  return r;
}
__device__ __forceinline__ float rdlane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

template <typename V> __device__ __forceinline__ V splatv(float a);
template <> __device__ __forceinline__ float splatv<float>(float a) { return a; }
template <> __device__ __forceinline__ v2f splatv<v2f>(float a) { return splat2(a); }

template <int CTRL, int RM>
__device__ __forceinline__ float dppv(float old, float src) { return dppf<CTRL, RM>(old, src); }
template <int CTRL, int RM>
__device__ __forceinline__ v2f dppv(float old, v2f src) { return dpp2<CTRL, RM>(old, src); }

__device__ __forceinline__ float rdlanev(float v, int l) { return rdlane(v, l); }
__device__ __forceinline__ v2f rdlanev(v2f v, int l) { v2f r; r.x = rdlane(v.x, l); r.y = rdlane(v.y, l); return r; }
__device__ __forceinline__ float wave_sumv(float v) { return wave_sum(v); }
__device__ __forceinline__ v2f wave_sumv(v2f v) { return wave_sum2(v); }
__device__ __forceinline__ float compv(float v, int) { return v; }
__device__ __forceinline__ float compv(v2f v, int c) { return c ? v.y : v.x; }

template <typename V>
struct Aff {
  V m11, m12, m21, m22, v1, v2;
};

// this = this ∘ q  (apply q first)
template <typename V>
__device__ __forceinline__ void compose(Aff<V>& a, const Aff<V>& q) {
  const V nv1 = a.m11 * q.v1 + a.m12 * q.v2 + a.v1;
  const V nv2 = a.m21 * q.v1 + a.m22 * q.v2 + a.v2;
  const V n11 = a.m11 * q.m11 + a.m12 * q.m21, n12 = a.m11 * q.m12 + a.m12 * q.m22;
  const V n21 = a.m21 * q.m11 + a.m22 * q.m21, n22 = a.m21 * q.m12 + a.m22 * q.m22;
  a.m11 = n11; a.m12 = n12; a.m21 = n21; a.m22 = n22; a.v1 = nv1; a.v2 = nv2;
}

template <int CTRL, int RM, typename V>
__device__ __forceinline__ void scan_round(Aff<V>& a) {
  Aff<V> q;
  q.m11 = dppv<CTRL, RM>(1.f, a.m11);
  q.m12 = dppv<CTRL, RM>(0.f, a.m12);
  q.m21 = dppv<CTRL, RM>(0.f, a.m21);
  q.m22 = dppv<CTRL, RM>(1.f, a.m22);
  q.v1 = dppv<CTRL, RM>(0.f, a.v1);
  q.v2 = dppv<CTRL, RM>(0.f, a.v2);
  compose(a, q);
}

// inclusive wave scan of affine maps (lane j: f_j ∘ ... ∘ f_0), then shift by
// one lane (exclusive); lane 0 gets the identity.
template <typename V>
__device__ __forceinline__ void wave_exclusive_scan(Aff<V>& a) {
  scan_round<0x111, 0xf>(a);  // row_shr:1
  scan_round<0x112, 0xf>(a);  // row_shr:2
  scan_round<0x114, 0xf>(a);  // row_shr:4
  scan_round<0x118, 0xf>(a);  // row_shr:8
  scan_round<0x142, 0xa>(a);  // row_bcast:15 → rows 1, 3
  scan_round<0x143, 0xc>(a);  // row_bcast:31 → rows 2, 3
  a.m11 = dppv<0x138, 0xf>(1.f, a.m11);  // wave_shr:1
  a.m12 = dppv<0x138, 0xf>(0.f, a.m12);
  a.m21 = dppv<0x138, 0xf>(0.f, a.m21);
  a.m22 = dppv<0x138, 0xf>(1.f, a.m22);
  a.v1 = dppv<0x138, 0xf>(0.f, a.v1);
  a.v2 = dppv<0x138, 0xf>(0.f, a.v2);
}

// ---- register image of one lane's K values of a segment ---------------------------
template <typename TIN, int K>
struct YRegs {
  static constexpr int KP = (sizeof(TIN) == 2) ? ((K + 7) / 8) * 8 : ((K + 3) / 4) * 4;
  static constexpr int NW = KP * sizeof(TIN) / 4;  // 32-bit words
  unsigned w[NW];
  __device__ __forceinline__ void load(const TIN* lds) {
    const uint4* p = (const uint4*)lds;
#pragma unroll
    for (int q = 0; q < NW / 4; ++q) {
      const uint4 v = p[q];
      w[4 * q + 0] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
  }
  __device__ __forceinline__ float get(int i) const {
    if (sizeof(TIN) == 2) {
      const unsigned x = w[i >> 1];
      return __uint_as_float((i & 1) ? (x & 0xffff0000u) : (x << 16));
    }
    return __uint_as_float(w[i]);
  }
};

// State in (f, b) coordinates: f = level + trend (the one-step forecast),
// b = trend.  Update:  e = u - f;  f' = (f + b) + c1 e;  b' = b + c2 e  with
// c1 = alpha (1 + beta), c2 = alpha beta — a 2-deep dependency per step
// (t = f + b issues beside e = u - f).
template <int K, typename Y, typename V>
__device__ __forceinline__ void pass1_fast(const Y& y, const V* s, V c1, V c2, V& v1, V& v2) {
  v1 = splatv<V>(0.f);
  v2 = splatv<V>(0.f);
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const V t = v1 + v2;
    const V e = (splatv<V>(y.get(i)) - s[i]) - v1;
    v1 = t + c1 * e;
    v2 = v2 + c2 * e;
  }
}

// general local map (segment contains NaN): NaN steps are x' = [[1,1],[0,1]] x
template <int K, typename Y, typename V>
__device__ __forceinline__ void pass1_slow(const Y& y, const V* s, V c1, V c2, Aff<V>& a) {
  const V one = splatv<V>(1.f), zero = splatv<V>(0.f);
  const V omc1 = one - c1;
  a.m11 = one; a.m12 = zero; a.m21 = zero; a.m22 = one; a.v1 = zero; a.v2 = zero;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const float yi = y.get(i);
    const bool ok = (yi == yi);
    const V a11 = ok ? omc1 : one;  // a12 = a22 = 1
    const V a21 = ok ? -c2 : zero;
    const V u = ok ? (splatv<V>(yi) - s[i]) : zero;
    const V n11 = a11 * a.m11 + a.m21, n12 = a11 * a.m12 + a.m22;
    const V n21 = a21 * a.m11 + a.m21, n22 = a21 * a.m12 + a.m22;
    const V nv1 = a11 * a.v1 + a.v2 + (ok ? c1 * u : zero);
    const V nv2 = a21 * a.v1 + a.v2 + (ok ? c2 * u : zero);
    a.m11 = n11; a.m12 = n12; a.m21 = n21; a.m22 = n22; a.v1 = nv1; a.v2 = nv2;
  }
}

// pass 2 of this segment (true start state x1/x2), optionally fused with the
// fast pass 1 of the next segment.
template <int K, int MODE, bool MASK, bool FUSE, typename Y, typename V>
__device__ __forceinline__ void pass2(const Y& y, const Y& yn, V* s, V c1, V c2, V g1a, V& x1, V& x2, V& sse,
                                      V& p1, V& p2) {
  if (FUSE) { p1 = splatv<V>(0.f); p2 = splatv<V>(0.f); }
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const V t = x1 + x2;
    const float yi = y.get(i);
    V e = (splatv<V>(yi) - s[i]) - x1;
    if (MASK) e = (yi == yi) ? e : splatv<V>(0.f);
    x1 = t + c1 * e;
    x2 = x2 + c2 * e;
    if (MODE == MODE_HW) s[i] = s[i] + g1a * e;
    sse = sse + e * e;
    if (FUSE) {
      const V tn = p1 + p2;
      const V en = (splatv<V>(yn.get(i)) - s[i]) - p1;
      p1 = tn + c1 * en;
      p2 = p2 + c2 * en;
    }
  }
}


// ---- table-driven fast path (variant 3) ---------------------------------------------
// Per combo pair the host precomputes (float, [combo0, combo1] interleaved):
//   [0..5]            c1, c2, g1a
//   [6 .. 6+4K)       W_i = A^(K-1-i) c  as (W1_i, W2_i) pairs   (pass-1 weights)
//   [6+4K .. +40)     B^1, B^2, B^4, B^8, B^16 (B = A^K), each m11 m12 m21 m22
// so pass 1 is  v = sum_i W_i u_i  (3 ops/step) and the cross-lane scan only
// carries the state vector with wave-uniform matrices.
template <int K>
struct PairTab {
  static constexpr int W0 = 6;
  static constexpr int B0 = 6 + 4 * K;
  static constexpr int SIZE = ((B0 + 40) + 15) / 16 * 16;
};

__device__ __forceinline__ v2f ldv2(const float* p) { return *(const v2f*)p; }
// constant address space: wave-uniform table reads become s_load (SGPR operands)
typedef const __attribute__((address_space(4))) float* cfp;
__device__ __forceinline__ v2f ldv2(cfp p) { return *(const __attribute__((address_space(4))) v2f*)p; }

struct Mat2 { v2f a, b, c, d; };
__device__ __forceinline__ Mat2 ldmat(const float* p) {
  Mat2 m; m.a = ldv2(p); m.b = ldv2(p + 2); m.c = ldv2(p + 4); m.d = ldv2(p + 6); return m;
}
__device__ __forceinline__ Mat2 ldmat(cfp p) {
  Mat2 m; m.a = ldv2(p); m.b = ldv2(p + 2); m.c = ldv2(p + 4); m.d = ldv2(p + 6); return m;
}
__device__ __forceinline__ void matvec(const Mat2& m, v2f x1, v2f x2, v2f& y1, v2f& y2) {
  y1 = m.a * x1 + m.b * x2;
  y2 = m.c * x1 + m.d * x2;
}
__device__ __forceinline__ Mat2 matmul(const Mat2& p, const Mat2& q) {
  Mat2 r;
  r.a = p.a * q.a + p.b * q.c; r.b = p.a * q.b + p.b * q.d;
  r.c = p.c * q.a + p.d * q.c; r.d = p.c * q.b + p.d * q.d;
  return r;
}

template <int CTRL>
__device__ __forceinline__ void row_round(v2f& w1, v2f& w2, const Mat2& Bd) {
  const v2f q1 = dpp2<CTRL, 0xf>(0.f, w1);
  const v2f q2 = dpp2<CTRL, 0xf>(0.f, w2);
  w1 = w1 + Bd.a * q1 + Bd.b * q2;
  w2 = w2 + Bd.c * q1 + Bd.d * q2;
}

// Exclusive scan of X_j = B X_{j-1} + v_j over lanes (X_{-1} = x0); returns the
// start state of this lane.  Bj = B^(lane & 15) (per lane, precomputed).
__device__ __forceinline__ void uniform_exclusive_scan(const float* tab_b, v2f v1, v2f v2, v2f x01, v2f x02,
                                                       const Mat2& Bj, int lane, v2f& s1, v2f& s2) {
  const Mat2 B1 = ldmat(tab_b), B2 = ldmat(tab_b + 8), B4 = ldmat(tab_b + 16), B8 = ldmat(tab_b + 24),
             B16 = ldmat(tab_b + 32);
  // within-row exclusive prefix
  v2f w1 = dpp2<0x111, 0xf>(0.f, v1);
  v2f w2 = dpp2<0x111, 0xf>(0.f, v2);
  row_round<0x111>(w1, w2, B1);
  row_round<0x112>(w1, w2, B2);
  row_round<0x114>(w1, w2, B4);
  row_round<0x118>(w1, w2, B8);
  // row-end states from zero: E = B w + v at lanes 15, 31, 47
  v2f e1, e2;
  matvec(B1, w1, w2, e1, e2);
  e1 = e1 + v1;
  e2 = e2 + v2;
  v2f Y01 = x01, Y02 = x02, t1, t2;
  const int row = lane >> 4;
  v2f p1 = x01, p2 = x02;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const v2f E1 = rdlanev(e1, 16 * r + 15), E2 = rdlanev(e2, 16 * r + 15);
    matvec(B16, Y01, Y02, t1, t2);
    Y01 = t1 + E1;
    Y02 = t2 + E2;
    if (row == r + 1) { p1 = Y01; p2 = Y02; }
  }
  matvec(Bj, p1, p2, s1, s2);
  s1 = s1 + w1;
  s2 = s2 + w2;
}

template <int K, int MODE, bool MASK, typename Y>
__device__ __forceinline__ void pass2_tab(const Y& y, const Y& yn, v2f* s, v2f c1, v2f c2, v2f g1a,
                                          const float* W, v2f& x1, v2f& x2, v2f& sse, v2f& p1, v2f& p2) {
  p1 = splat2(0.f);
  p2 = splat2(0.f);
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const v2f t = x1 + x2;
    const float yi = y.get(i);
    v2f e = (splat2(yi) - s[i]) - x1;
    if (MASK) e = (yi == yi) ? e : splat2(0.f);
    x1 = t + c1 * e;
    x2 = x2 + c2 * e;
    if (MODE == MODE_HW) s[i] = s[i] + g1a * e;
    sse = sse + e * e;
    const v2f un = splat2(yn.get(i)) - s[i];
    p1 = p1 + ldv2(W + 4 * i) * un;
    p2 = p2 + ldv2(W + 4 * i + 2) * un;
  }
}

// ---- variant 4 helpers: one series per 32-lane half-wave -----------------------------

// bf16 values streamed from LDS 8 at a time (one ds_read_b128 per chunk), the next
// chunk in flight while this one is consumed; the empty asm keeps the compiler from
// hoisting every chunk (and its unpacked floats) to the top of the season.
struct Chunk8 {
  uint4 w;
  __device__ __forceinline__ float get(int i) const {
    const unsigned x = (i >> 1) == 0 ? w.x : (i >> 1) == 1 ? w.y : (i >> 1) == 2 ? w.z : w.w;
    return __uint_as_float((i & 1) ? (x & 0xffff0000u) : (x << 16));
  }
};
__device__ __forceinline__ void fence_sched() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);  // nor may the machine scheduler move ALU work across
}
// Constant-space loads are invariant, so LLVM hoists them out of every loop (and past
// asm memory clobbers) — for a 180-float table that spills SGPRs.  Re-deriving the
// pointer through an opaque asm per season / chunk keeps each load where it is used.
__device__ __forceinline__ cfp launder(cfp p) {
  asm volatile("" : "+s"(p));
  return p;
}
// the pair table as a constant-address-space pointer (uniform: scalar loads)
__device__ __forceinline__ cfp const_ptr(const float* p) {
  return (cfp)(__builtin_amdgcn_readfirstlane((int)((unsigned long long)p)) & 0xffffffffull |
               ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned long long)p >> 32)) << 32));
}

// fused: pass 2 of this season (true start state x) + table pass 1 of the next one.
template <int K, bool MASK, bool FUSE>
__device__ __forceinline__ void pass2_stream(const bf16_t* yc, const bf16_t* yn, v2f* s, v2f c1, v2f c2, v2f g1a,
                                             cfp W, v2f& x1, v2f& x2, v2f& sse, v2f& p1, v2f& p2) {
  constexpr int NCH = (K + 7) / 8;
  const uint4* pc = (const uint4*)yc;
  const uint4* pn = (const uint4*)yn;
  if (FUSE) { p1 = splat2(0.f); p2 = splat2(0.f); }
  fence_sched();  // the variants share loads: keep them from being merged above the branch
  // y chunks (LDS) and pass-1 weights (scalar loads, 8 steps = 16 SGPR pairs) are
  // fetched one chunk ahead, so no wait on lgkmcnt lands right after its load
  Chunk8 cc, cn, nc, nn;
  v2f wc[16], wn[16];
  cn.w = pc[0];
  if (FUSE) {
    nn.w = pn[0];
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (r < 2 * K) wn[r] = ldv2(W + 2 * r);
  }
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    cc = cn;
    if (FUSE) {
      nc = nn;
#pragma unroll
      for (int r = 0; r < 16; ++r) wc[r] = wn[r];
      // wait for this chunk's operands BEFORE the next chunk's loads are issued
      // (scalar loads complete out of order: any use waits for lgkmcnt(0))
      asm volatile("" ::"v"(cc.w.x), "v"(nc.w.x), "s"(wc[0].x));
    }
    if (q + 1 < NCH) {
      cn.w = pc[q + 1];
      if (FUSE) {
        W = launder(W);
        nn.w = pn[q + 1];
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (16 * (q + 1) + r < 2 * K) wn[r] = ldv2(W + 32 * (q + 1) + 2 * r);
      }
    }
    fence_sched();
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int i = 8 * q + r;
      if (i < K) {
        const v2f t = x1 + x2;
        const float yi = cc.get(r);
        v2f e = (splat2(yi) - s[i]) - x1;
        if (MASK) e = (yi == yi) ? e : splat2(0.f);
        x1 = t + c1 * e;
        x2 = x2 + c2 * e;
        s[i] = s[i] + g1a * e;
        sse = sse + e * e;
        if (FUSE) {
          const v2f un = splat2(nc.get(r)) - s[i];
          p1 = p1 + wc[2 * r] * un;
          p2 = p2 + wc[2 * r + 1] * un;
        }
      }
    }
    fence_sched();
  }
}

// table pass 1 (NaN-free season): v = sum_i W_i (y_i - s_i)
template <int K>
__device__ __forceinline__ void pass1_stream(const bf16_t* yc, const v2f* s, cfp W, v2f& p1, v2f& p2) {
  constexpr int NCH = (K + 7) / 8;
  const uint4* pc = (const uint4*)yc;
  p1 = splat2(0.f);
  p2 = splat2(0.f);
  fence_sched();
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    Chunk8 c;
    c.w = pc[q];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int i = 8 * q + r;
      if (i < K) {
        const v2f un = splat2(c.get(r)) - s[i];
        p1 = p1 + ldv2(W + 4 * i) * un;
        p2 = p2 + ldv2(W + 4 * i + 2) * un;
      }
    }
    fence_sched();
  }
}

// value of lane 31 (half 0) / lane 63 (half 1): the end state of the half's season
__device__ __forceinline__ v2f half_last(v2f x, int half) {
  const v2f lo = rdlanev(x, 31), hi = rdlanev(x, 63);
  return half ? hi : lo;
}

// Exclusive scan X_j = B X_{j-1} + v_j over the 32 lanes of each half (X_{-1} = x0
// of that half); Bj = B^(lane & 15).  Four in-row DPP rounds, then rows 1 / 3 take
// the row-0 / row-2 end state through row_bcast:15 — the halves never mix.
__device__ __forceinline__ void half_uniform_scan(cfp tab_b, v2f v1, v2f v2, v2f x01, v2f x02,
                                                  const Mat2& Bj, bool odd_row, v2f& s1, v2f& s2) {
  const Mat2 B1 = ldmat(tab_b), B2 = ldmat(tab_b + 8), B4 = ldmat(tab_b + 16), B8 = ldmat(tab_b + 24),
             B16 = ldmat(tab_b + 32);
  v2f w1 = dpp2<0x111, 0xf>(0.f, v1);
  v2f w2 = dpp2<0x111, 0xf>(0.f, v2);
  row_round<0x111>(w1, w2, B1);
  row_round<0x112>(w1, w2, B2);
  row_round<0x114>(w1, w2, B4);
  row_round<0x118>(w1, w2, B8);
  v2f e1, e2;  // end state of each lane from zero; lanes 15 / 47 close rows 0 / 2
  matvec(B1, w1, w2, e1, e2);
  e1 = e1 + v1;
  e2 = e2 + v2;
  const v2f E1 = dpp2<0x142, 0xa>(0.f, e1), E2 = dpp2<0x142, 0xa>(0.f, e2);
  v2f y1, y2;
  matvec(B16, x01, x02, y1, y2);
  y1 = odd_row ? y1 + E1 : x01;
  y2 = odd_row ? y2 + E2 : x02;
  matvec(Bj, y1, y2, s1, s2);
  s1 = s1 + w1;
  s2 = s2 + w2;
}

// DPP move with BOUND_CTRL: lanes without a source read 0, so no zeroed "old" register
// has to be materialised per move (variant 4 spends a v_mov per DPP on it)
template <int CTRL, int RM>
__device__ __forceinline__ v2f dppz2(v2f src) {
  v2f r;
  r.x = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(src.x), CTRL, RM, 0xf, true));
  r.y = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(src.y), CTRL, RM, 0xf, true));
  return r;
}
template <int CTRL>
__device__ __forceinline__ void row_round_z(v2f& w1, v2f& w2, const Mat2& Bd) {
  const v2f q1 = dppz2<CTRL, 0xf>(w1);
  const v2f q2 = dppz2<CTRL, 0xf>(w2);
  w1 = w1 + Bd.a * q1 + Bd.b * q2;
  w2 = w2 + Bd.c * q1 + Bd.d * q2;
}
// half_uniform_scan with BOUND_CTRL moves (rows 0 / 2 never read the row_bcast result) and
// B^1..B^8 already in registers (only B^16 is loaded here; it is first used after the four
// row rounds)
__device__ __forceinline__ void half_uniform_scan_pre(const Mat2* Bp, cfp tab_b, v2f v1, v2f v2, v2f x01, v2f x02,
                                                      const Mat2& Bj, bool odd_row, v2f& s1, v2f& s2) {
  const Mat2 B16 = ldmat(tab_b + 32);
  v2f w1 = dppz2<0x111, 0xf>(v1);
  v2f w2 = dppz2<0x111, 0xf>(v2);
  row_round_z<0x111>(w1, w2, Bp[0]);
  row_round_z<0x112>(w1, w2, Bp[1]);
  row_round_z<0x114>(w1, w2, Bp[2]);
  row_round_z<0x118>(w1, w2, Bp[3]);
  v2f e1, e2;
  matvec(Bp[0], w1, w2, e1, e2);
  e1 = e1 + v1;
  e2 = e2 + v2;
  const v2f E1 = dppz2<0x142, 0xa>(e1), E2 = dppz2<0x142, 0xa>(e2);
  v2f y1, y2;
  matvec(B16, x01, x02, y1, y2);
  y1 = odd_row ? y1 + E1 : x01;
  y2 = odd_row ? y2 + E2 : x02;
  matvec(Bj, y1, y2, s1, s2);
  s1 = s1 + w1;
  s2 = s2 + w2;
}

// hw_q_block's scan: one series per 16-lane row, so the four row rounds are the whole scan
// (X_{-1} = x0 of the row's series; Bj = B^(lane & 15))
__device__ __forceinline__ void row_uniform_scan_pre(const Mat2* Bp, v2f v1, v2f v2, v2f x01, v2f x02,
                                                     const Mat2& Bj, v2f& s1, v2f& s2) {
  v2f w1 = dppz2<0x111, 0xf>(v1);
  v2f w2 = dppz2<0x111, 0xf>(v2);
  row_round_z<0x111>(w1, w2, Bp[0]);
  row_round_z<0x112>(w1, w2, Bp[1]);
  row_round_z<0x114>(w1, w2, Bp[2]);
  row_round_z<0x118>(w1, w2, Bp[3]);
  matvec(Bj, x01, x02, s1, s2);
  s1 = s1 + w1;
  s2 = s2 + w2;
}

// General (per-lane matrix) exclusive affine scan within each 32-lane half.
template <typename V>
__device__ __forceinline__ void half_exclusive_scan(Aff<V>& a, int j) {
  scan_round<0x111, 0xf>(a);  // row_shr:1
  scan_round<0x112, 0xf>(a);  // row_shr:2
  scan_round<0x114, 0xf>(a);  // row_shr:4
  scan_round<0x118, 0xf>(a);  // row_shr:8
  scan_round<0x142, 0xa>(a);  // row_bcast:15 → rows 1, 3
  a.m11 = dppv<0x138, 0xf>(1.f, a.m11);  // wave_shr:1 (lane 32 is fixed below)
  a.m12 = dppv<0x138, 0xf>(0.f, a.m12);
  a.m21 = dppv<0x138, 0xf>(0.f, a.m21);
  a.m22 = dppv<0x138, 0xf>(1.f, a.m22);
  a.v1 = dppv<0x138, 0xf>(0.f, a.v1);
  a.v2 = dppv<0x138, 0xf>(0.f, a.v2);
  if (j == 0) {
    const V one = splatv<V>(1.f), zero = splatv<V>(0.f);
    a.m11 = one; a.m12 = zero; a.m21 = zero; a.m22 = one; a.v1 = zero; a.v2 = zero;
  }
}

}  // namespace

// ---- variant 4: two series per wave ----------------------------------------------------
// For a season m = 32 K (daily 1440 = 32 x 45) each 32-lane half of a wave walks one
// series: lane j owns phases [jK, (j+1)K).  Against variant 3 (one series per wave,
// 60 lanes x 24 steps) the per-season scan is four in-row DPP rounds + one row_bcast
// and is amortised over 45 steps instead of 24: ~12 VALU ops per step for two grid
// points instead of ~17.5.  A workgroup (4 waves, 2 per SIMD) owns two series staged
// once in LDS; every wave fits a quarter of the grid pairs for both.  Only the first
// HALF_HB best seasonal phases are kept (enough for forecast horizons 1..hmax <= K), so
// this variant does not produce season_out (the host falls back to variant 3 then).
constexpr int HALF_HB = 16;

// One workgroup's work on the series pair (n0, n0 + 1).  GENERAL = false is the
// straight-line NaN-free path: a pair with a gap in a fitted season is appended to
// `deferred` and left to the GENERAL = true launch (per-lane affine scan, masked
// steps), so the common path carries no NaN branches and no register copies at joins.
template <int K, bool GENERAL>
__device__ __forceinline__ void hw_half_block(const SmoothArgs& a, int hmax, int n0, int* deferred) {
  using YR = YRegs<bf16_t, K>;
  constexpr int KP = YR::KP;
  constexpr int TS = PairTab<K>::SIZE;
  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  const int half = lane >> 5, j = lane & 31;
  const bool odd_row = ((lane >> 4) & 1) != 0;
  const int nseg = a.Tp / a.seg, m = a.m;

  // ---- LDS: ys[2][nseg][32][KP] | segnan[2][nseg] + nvs[2] | bests[4][2][HB] | wbest[4][2][4]
  bf16_t* ys = (bf16_t*)fm_hw_smem;
  size_t off = ((size_t)2 * nseg * 32 * KP * sizeof(bf16_t) + 15) & ~(size_t)15;
  int* segnan = (int*)(fm_hw_smem + off);
  float* nvs = (float*)(segnan + 2 * nseg);
  off += ((size_t)(2 * nseg + 2) * 4 + 15) & ~(size_t)15;
  float* bests = (float*)(fm_hw_smem + off);
  off += (size_t)4 * 2 * HALF_HB * 4;
  float* wbest = (float*)(fm_hw_smem + off);

  for (int i = tid; i < 2 * nseg + 2; i += blockDim.x) segnan[i] = 0;  // also nvs = 0.f
  const int head = a.head_dev ? *a.head_dev : a.head;
  __syncthreads();

  // ---- stage both series: logical padded index p = pk*K + i, pk = sg*32 + lane -------
  // 16 independent loads in flight per thread per batch (a dependent load per
  // element would serialise ~80 HBM round trips per workgroup)
  constexpr int U = 16;
  for (int r = 0; r < 2; ++r) {
    const int n = n0 + r;
    const bool real = n < a.N;
    const bf16_t* row = (const bf16_t*)a.hist + (long long)(real ? n : 0) * a.ld;
    float nv = 0.f;
    for (int p0 = tid; p0 < a.Tp; p0 += U * (int)blockDim.x) {
      bf16_t v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int p = p0 + u * (int)blockDim.x;
        v[u] = 0;  // the padding series of an odd N is zeros (keeps the wave on the fast path)
        if (real && p < a.Tp) {
          v[u] = 0x7fc0;
          const int t = p - a.pad;
          if (t >= 0) {
            int c = head + t;
            if (c >= a.ring_len) c -= a.ring_len;
            v[u] = row[c];
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int p = p0 + u * (int)blockDim.x;
        if (p < a.Tp) {
          const int pk = p / K, i = p - pk * K;
          ys[((size_t)r * nseg * 32 + pk) * KP + i] = v[u];
          const float f = bf16_to_f32(v[u]);
          if (f != f) atomicOr(&segnan[r * nseg + (pk >> 5)], 1);
          else if (p >= m) nv += 1.f;
        }
      }
    }
    nv = wave_sum(nv);
    if (lane == 0) atomicAdd(&nvs[r], nv);
  }
  __syncthreads();

  const bf16_t* myys = ys + ((size_t)half * nseg * 32 + j) * KP;
  auto yseg = [&](int sg) { return myys + (size_t)sg * 32 * KP; };
  auto seg_nan = [&](int sg) { return (segnan[sg] | segnan[nseg + sg]) != 0; };

  // ---- initial state of my half's series (season means) ------------------------------
  float l0, b0;
  {
    YR y0, y1;
    y0.load(yseg(0));
    y1.load(yseg(1));
    float s0 = 0.f, q0 = 0.f, s1 = 0.f, q1 = 0.f;
#pragma unroll
    for (int i = 0; i < K; ++i) {
      const float u = y0.get(i), v = y1.get(i);
      if (u == u) { s0 += u; q0 += 1.f; }
      if (v == v) { s1 += v; q1 += 1.f; }
    }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
      s0 += __shfl_xor(s0, o, FM_WAVE);
      q0 += __shfl_xor(q0, o, FM_WAVE);
      s1 += __shfl_xor(s1, o, FM_WAVE);
      q1 += __shfl_xor(q1, o, FM_WAVE);
    }
    l0 = q0 > 0.f ? s0 / q0 : 0.f;
    b0 = ((q1 > 0.f ? s1 / q1 : 0.f) - l0) / (float)m;
  }

  bool allfast = true;  // no NaN in the fitted seasons of either series
  for (int sg = 1; sg < nseg; ++sg) allfast = allfast && !seg_nan(sg);
  if (!GENERAL && !allfast) {
    if (tid == 0) {
      const int q = atomicAdd(deferred, 1);
      if (q < (a.N + 1) / 2) deferred[1 + q] = n0;  // a stale count can never write past the pair list
    }
    return;
  }
  float bestSSE = __builtin_huge_valf();
  int bestIdx = 0x7fffffff;
  float bestL = l0, bestB = b0;
  float* mybest = bests + (w * 2 + half) * HALF_HB;
  const int npairs = (a.G + 1) / 2;
  const int nwaves = blockDim.x / FM_WAVE;

  for (int pi = w; pi < npairs; pi += nwaves) {
    const int c0 = 2 * pi;
    const int c1i = (2 * pi + 1 < a.G) ? 2 * pi + 1 : c0;
    const cfp tab = const_ptr(a.pair_tab + (size_t)pi * TS);
    const v2f c1 = ldv2(tab), c2 = ldv2(tab + 2), g1a = ldv2(tab + 4);
    const cfp W = tab + PairTab<K>::W0;
    const cfp tb = tab + PairTab<K>::B0;
    const v2f one = splat2(1.f), zero = splat2(0.f);
    Mat2 Bj;  // B^(lane & 15)
    Bj.a = one; Bj.b = zero; Bj.c = zero; Bj.d = one;
#pragma unroll
    for (int bit = 0; bit < 4; ++bit) {
      const Mat2 Bb = ldmat(tb + 8 * bit);
      const Mat2 r = matmul(Bj, Bb);
      if ((lane >> bit) & 1) Bj = r;
    }

    v2f s[K];
    {
      YR y0;
      y0.load(yseg(0));
#pragma unroll
      for (int i = 0; i < K; ++i) {
        const float y = y0.get(i);
        s[i] = splat2(y == y ? y - l0 : 0.f);
      }
    }
    v2f X1 = splat2(l0 + b0), X2 = splat2(b0), sse = zero;  // (f, b) at the season start

    Aff<v2f> loc;
    if constexpr (!GENERAL) {
      // NaN-free seasons (the common case): one straight-line path, so the seasonal
      // state keeps its registers across seasons (no phi copies at a join)
      pass1_stream<K>(yseg(1), s, W, loc.v1, loc.v2);
      for (int sg = 1; sg < nseg - 1; ++sg) {
        v2f x1, x2;
        half_uniform_scan(launder(tb), loc.v1, loc.v2, X1, X2, Bj, odd_row, x1, x2);
        pass2_stream<K, false, true>(yseg(sg), yseg(sg + 1), s, c1, c2, g1a, launder(W), x1, x2, sse, loc.v1,
                                     loc.v2);
        X1 = half_last(x1, half);
        X2 = half_last(x2, half);
      }
      v2f x1, x2, d1, d2;
      half_uniform_scan(tb, loc.v1, loc.v2, X1, X2, Bj, odd_row, x1, x2);
      pass2_stream<K, false, false>(yseg(nseg - 1), yseg(nseg - 1), s, c1, c2, g1a, W, x1, x2, sse, d1, d2);
      X1 = half_last(x1, half);
      X2 = half_last(x2, half);
    } else {
      bool locfast = !seg_nan(1);
      if (locfast) {
        pass1_stream<K>(yseg(1), s, W, loc.v1, loc.v2);
      } else {
        YR y1;
        y1.load(yseg(1));
        pass1_slow<K>(y1, s, c1, c2, loc);
      }
      for (int sg = 1; sg < nseg; ++sg) {
        v2f x1, x2;
        if (locfast) {
          half_uniform_scan(tb, loc.v1, loc.v2, X1, X2, Bj, odd_row, x1, x2);
        } else {
          half_exclusive_scan(loc, j);
          x1 = loc.m11 * X1 + loc.m12 * X2 + loc.v1;
          x2 = loc.m21 * X1 + loc.m22 * X2 + loc.v2;
        }
        const bool has_next = sg + 1 < nseg;
        const bool mask = seg_nan(sg);
        const bool next_fast = has_next && !seg_nan(sg + 1);
        const bf16_t* yc = yseg(sg);
        const bf16_t* yn = yseg(has_next ? sg + 1 : sg);
        if (next_fast) {
          if (mask) pass2_stream<K, true, true>(yc, yn, s, c1, c2, g1a, W, x1, x2, sse, loc.v1, loc.v2);
          else pass2_stream<K, false, true>(yc, yn, s, c1, c2, g1a, W, x1, x2, sse, loc.v1, loc.v2);
          locfast = true;
        } else {
          v2f d1, d2;
          if (mask) pass2_stream<K, true, false>(yc, yn, s, c1, c2, g1a, W, x1, x2, sse, d1, d2);
          else pass2_stream<K, false, false>(yc, yn, s, c1, c2, g1a, W, x1, x2, sse, d1, d2);
          if (has_next) {
            YR y1;
            y1.load(yn);
            pass1_slow<K>(y1, s, c1, c2, loc);
          }
          locfast = false;
        }
        X1 = half_last(x1, half);
        X2 = half_last(x2, half);
      }
    }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
      sse.x += __shfl_xor(sse.x, o, FM_WAVE);
      sse.y += __shfl_xor(sse.y, o, FM_WAVE);
    }
    const bool upd0 = (sse.x < bestSSE || (sse.x == bestSSE && c0 < bestIdx));
    if (upd0) { bestSSE = sse.x; bestIdx = c0; bestL = X1.x - X2.x; bestB = X2.x; }
    const bool upd1 = (c1i != c0) && (sse.y < bestSSE || (sse.y == bestSSE && c1i < bestIdx));
    if (upd1) { bestSSE = sse.y; bestIdx = c1i; bestL = X1.y - X2.y; bestB = X2.y; }
    if (j == 0 && (upd0 || upd1)) {
#pragma unroll
      for (int i = 0; i < K && i < HALF_HB; ++i)
        if (i < hmax) mybest[i] = upd1 ? s[i].y : s[i].x;
    }
  }

  // ---- arg-min across the 4 waves; wave r finishes series n0 + r ----------------------
  if (j == 0) {
    float* wb = wbest + (w * 2 + half) * 4;
    wb[0] = bestSSE;
    wb[1] = __int_as_float(bestIdx);
    wb[2] = bestL;
    wb[3] = bestB;
  }
  __syncthreads();
  if (w >= 2) return;
  const int r = w, n = n0 + r;
  if (n >= a.N) return;
  const int nw = blockDim.x / FM_WAVE;
  int win = 0;
  for (int q = 1; q < nw; ++q) {
    const float sq = wbest[(q * 2 + r) * 4], sw = wbest[(win * 2 + r) * 4];
    const int iq = __float_as_int(wbest[(q * 2 + r) * 4 + 1]), iw = __float_as_int(wbest[(win * 2 + r) * 4 + 1]);
    if (sq < sw || (sq == sw && iq < iw)) win = q;
  }
  const float* wb = wbest + (win * 2 + r) * 4;
  const float gSSE = wb[0], gL = wb[2], gB = wb[3];
  const int gIdx = __float_as_int(wb[1]);
  const float nvr = nvs[r];
  const float sig = sqrtf(gSSE / fmaxf(nvr, 1.f));
  if (lane == 0) {
    a.level[n] = gL;
    a.trend[n] = gB;
    a.sigma[n] = sig;
    a.best[n] = gIdx;
  }
  const float* sb = bests + (win * 2 + r) * HALF_HB;
  const int Tp = a.Tp;
  if (a.season_hb && lane < hmax) a.season_hb[(long long)n * HALF_HB + lane] = sb[lane];
  if (a.nvalid_out && lane == 0) a.nvalid_out[n] = nvr;
  detect_epilogue_wave(a.det, n, sig, nvr, [&](int h) {
    int ph = (Tp - 1 + h) % m;
    if (ph < 0) ph += m;
    ph = ph < HALF_HB ? ph : HALF_HB - 1;  // host guarantees ph < hmax; clamp keeps LDS reads in bounds
    return gL + (float)h * gB + sb[ph];
  }, gIdx);
}

template <int K>
__global__ __launch_bounds__(256, 2) void hw_half_kernel(const SmoothArgs a, int hmax, int* deferred) {
  hw_half_block<K, false>(a, hmax, blockIdx.x * 2, deferred);
}

// persistent over the pairs deferred by hw_half_kernel (count in deferred[0]).
// Self-cleaning: the workspace is int32 [2 + ceil(N / 2)] = {count, pairs..., done};
// every workgroup counts itself in `done` after it has read the count, and the last
// one resets count and done to 0, so the next fit needs no memset launch (the host
// allocates the workspace zeroed).
template <int K>
__global__ __launch_bounds__(256, 2) void hw_half_general_kernel(const SmoothArgs a, int hmax, int* deferred) {
  const int cnt = min(deferred[0], (a.N + 1) / 2);
  // nothing deferred (gap-free shard, the common case): count and done are already 0, so
  // no workgroup needs to count itself — skip the 512 same-address atomics
  if (cnt == 0) return;
  for (int q = blockIdx.x; q < cnt; q += gridDim.x) {
    hw_half_block<K, true>(a, hmax, deferred[1 + q], nullptr);
    __syncthreads();  // LDS is reused by the next pair
  }
  __syncthreads();  // every thread of this workgroup has read the count
  if (threadIdx.x == 0) {
    int* done = deferred + 1 + (a.N + 1) / 2;
    if (atomicAdd(done, 1) == (int)gridDim.x - 1) {
      *done = 0;
      deferred[0] = 0;
    }
  }
}

// ---- variant 5: residual-state walk ------------------------------------------------------
// Per phase i the walker keeps D_i = y_{k,i} - s_i, the observation of the season being
// walked minus its seasonal state, instead of s_i.  Then
//   e = D - f,   s' = s + g e   =>   D' = D + (y_{k+1,i} - y_{k,i}) - g e,
// and D' is exactly the next season's pass-1 input u = y_{k+1} - s'.  The LDS image holds
// D^(1) (season 1 minus the initial seasonal state) and the season-to-season differences
// in fp32, so a step is 9 packed ops (e, f+b, f, b, sse, D+dy, D-ge, two pass-1 FMAs) with
// no bf16 unpacking — variant 4 spends 12 (two unpacks, y-s, -f, un).  The image is twice
// the bf16 one (fp32) but holds one season fewer: 2 series x 6 x 1440 x 4 B = 72 KiB per
// workgroup, two workgroups per CU.  Series pairs with a NaN past season 0 are deferred
// to hw_half_general_kernel exactly as in variant 4.
constexpr int D_CHUNK = 260;  // floats per 8-step chunk: 256 + 4 pad (see dl_off)
template <int K>
struct DLay {
  static constexpr int NCH = (K + 7) / 8;
  static constexpr int KP = NCH * 8;
  static constexpr int SEASON = D_CHUNK * NCH;  // floats per (series, season): [q][h][j][4] + pad
};
// float offset of step i of lane j inside a season block: lanes are 16 B apart within a
// half-chunk, so each ds_read_b128 lane group hits 16 distinct 16-B slots (no conflicts).
// Chunk q starts 4 floats further than 256 q: the stage phase writes, per instruction, the
// ~6 steps i = i0 + 8k of one lane from 6 threads, which without the pad all hit bank
// 4 j + (i & 3); with it they land 4 banks apart (at most 2-way, lanes 4 apart with
// chunks 4 apart).
__device__ __forceinline__ int dl_off(int i, int j) {
  return (i >> 3) * D_CHUNK + ((i >> 2) & 1) * 128 + j * 4 + (i & 3);
}

constexpr int D_WAVES = 4;   // waves per hw_d workgroup (launched with 256 threads)
constexpr int D_MAXSEG = 7;  // seasons staged per series (LDS budget: 6 fp32 blocks)

struct Chunk8f {
  float4 lo, hi;
  __device__ __forceinline__ float get(int r) const {
    switch (r) {
      case 0: return lo.x; case 1: return lo.y; case 2: return lo.z; case 3: return lo.w;
      case 4: return hi.x; case 5: return hi.y; case 6: return hi.z; default: return hi.w;
    }
  }
  __device__ __forceinline__ void load(const float* p) {  // p: chunk base + j*4
    lo = *(const float4*)p;
    hi = *(const float4*)(p + 128);
  }
};

// a + {pair[SEL], pair[SEL]}: VOP3P op_sel picks either 32-bit half of an aligned pair
// for both lanes, so the odd elements of a float4 need no register copy (LLVM only
// folds the even ones)
template <int SEL>
__device__ __forceinline__ v2f pk_add_bcast(v2f a, v2f pair) {
  v2f r;
  if (SEL == 0) asm("v_pk_add_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r) : "v"(a), "v"(pair));
  else asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(r) : "v"(a), "v"(pair));
  return r;
}
template <int R>
__device__ __forceinline__ v2f chunk_pair(const Chunk8f& c) {
  const float4 q = R < 4 ? c.lo : c.hi;
  v2f p;
  if ((R & 3) < 2) { p.x = q.x; p.y = q.y; } else { p.x = q.z; p.y = q.w; }
  return p;
}
template <int R>
__device__ __forceinline__ v2f add_dy(v2f d, const Chunk8f& c) { return pk_add_bcast<R & 1>(d, chunk_pair<R>(c)); }

// end state of each half's season (lane 31 / lane 63) to every lane of the half:
// one ds_bpermute per register (its latency hides under the next season's row rounds)
__device__ __forceinline__ v2f half_last_bp(v2f x, int src_addr) {
  v2f r;
  r.x = __int_as_float(__builtin_amdgcn_ds_bpermute(src_addr, __float_as_int(x.x)));
  r.y = __int_as_float(__builtin_amdgcn_ds_bpermute(src_addr, __float_as_int(x.y)));
  return r;
}

// sum over each 32-lane half, valid in lanes 31 and 63 only: DPP row scans (row_shr
// 1/2/4/8) then row_bcast:15 into rows 1 / 3.  One fixed tree of adds, so a sum of
// larger operands is never smaller (the grid branch and bound relies on it).
__device__ __forceinline__ v2f half_sum_last(v2f v) {
  // v_add_f32 with a DPP source (LLVM would re-pack separate adds into v_pk_add_f32,
  // which takes no DPP operand); s_nop 1 covers the VALU-write -> DPP-read hazard.
  // row_bcast:15 writes rows 1 / 3 only: rows 0 / 2 keep their value.
  asm volatile(
      "s_nop 1\n"
      "v_add_f32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_add_f32_dpp %1, %1, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "s_nop 1\n"
      "v_add_f32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_add_f32_dpp %1, %1, %1 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "s_nop 1\n"
      "v_add_f32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_add_f32_dpp %1, %1, %1 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "s_nop 1\n"
      "v_add_f32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_add_f32_dpp %1, %1, %1 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "s_nop 1\n"
      "v_add_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
      "v_add_f32_dpp %1, %1, %1 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
      "s_nop 1"
      : "+v"(v.x), "+v"(v.y));
  return v;
}

// sum over each 16-lane row, valid in lanes 15 / 31 / 47 / 63 (hw_q_block: a series per
// row): the first four rounds of half_sum_last, the same fixed tree within a row
__device__ __forceinline__ v2f row_sum_last(v2f v) {
  asm volatile(
      "s_nop 1\n"
      "v_add_f32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_add_f32_dpp %1, %1, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "s_nop 1\n"
      "v_add_f32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_add_f32_dpp %1, %1, %1 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "s_nop 1\n"
      "v_add_f32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_add_f32_dpp %1, %1, %1 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "s_nop 1\n"
      "v_add_f32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_add_f32_dpp %1, %1, %1 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "s_nop 1"
      : "+v"(v.x), "+v"(v.y));
  return v;
}

// {pair[SEL], pair[SEL]} in one v_pk_mov_b32 (two v_mov_b32 otherwise); the result is a
// 64-bit register pair from the start: left as one 32-bit value used twice, the season
// loop's D registers were re-paired by 48 copies on every iteration
template <int SEL>
__device__ __forceinline__ v2f pk_splat(v2f pair) {
  v2f r;
  if (SEL == 0) asm volatile("v_pk_mov_b32 %0, %1, %1 op_sel:[0,0]" : "=v"(r) : "v"(pair));
  else asm volatile("v_pk_mov_b32 %0, %1, %1 op_sel:[1,1]" : "=v"(r) : "v"(pair));
  return r;
}
template <int K, int R>
__device__ __forceinline__ void d_pass1_steps(int q, const Chunk8f& cc, const v2f* wc, v2f* D, v2f& p1, v2f& p2) {
  if constexpr (R < 8) {
    const int i = 8 * q + R;
    if (i < K) {
      D[i] = pk_splat<R & 1>(chunk_pair<R>(cc));
      p1 = p1 + wc[2 * R] * D[i];
      p2 = p2 + wc[2 * R + 1] * D[i];
    }
    d_pass1_steps<K, R + 1>(q, cc, wc, D, p1, p2);
  }
}

// pass 1 of season 1: D_i = splat(D1_i), v = sum_i W_i D1_i.  A chunk's 16 weight pairs
// are requested together (one wait per chunk; loaded one at a time, each waited for
// before the next, they left the pass on the scalar cache's latency) and the next LDS
// chunk is in flight while this one is summed
template <int K>
__device__ __forceinline__ void d_pass1(const float* blk, cfp W, v2f* D, v2f& p1, v2f& p2) {
  constexpr int NCH = (K + 7) / 8;
  p1 = splat2(0.f);
  p2 = splat2(0.f);
  Chunk8f cc, cn;
  cn.load(blk);
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    v2f wc[16];
    W = launder(W);
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (16 * q + r < 2 * K) wc[r] = ldv2(W + 32 * q + 2 * r);
    cc = cn;
    if (q + 1 < NCH) cn.load(blk + (q + 1) * D_CHUNK);
    fence_sched();
    d_pass1_steps<K, 0>(q, cc, wc, D, p1, p2);
    fence_sched();
  }
}

// e with both grid points' components zeroed where bit `bit` of `keep` is clear (keep:
// the lane's valid-step bits): a missing observation's step carries the forecast
// (e = 0: no SSE term, no seasonal update).  v_bfe_i32 + two v_and_b32.
__device__ __forceinline__ v2f keep_if(v2f e, unsigned keep, int bit) {
  const int mk = ((int)(keep << (31 - bit))) >> 31;  // -1: observed, 0: missing
  v2f r;
  r.x = __int_as_float(__float_as_int(e.x) & mk);
  r.y = __int_as_float(__float_as_int(e.y) & mk);
  return r;
}

// the 8 steps of chunk q (compile-time r: the Δ operand's register half is static).
// Gapped seasons (hw_dg_block): M2 masks this season's missing steps (keep bits k2 of the
// chunk's word); R1 runs the next season's pass 1 as the masked recurrence from a zero
// state (p = the lane's end state from zero: its affine offset, exact with gaps) instead
// of the table sum, whose uniform weights assume every step observed (keep bits k1).
template <int K, bool FUSE, int R, bool M2 = false, bool R1 = false>
__device__ __forceinline__ void d_steps(int q, const Chunk8f& cc, v2f* D, v2f c1, v2f c2, v2f g1a, const v2f* wc,
                                        v2f& x1, v2f& x2, v2f& sse, v2f& p1, v2f& p2, unsigned k2 = 0u,
                                        unsigned k1 = 0u) {
  if constexpr (R < 8) {
    const int i = 8 * q + R;
    if (i < K) {
      v2f e = D[i] - x1;
      if (M2) e = keep_if(e, k2, i & 31);
      const v2f t = x1 + x2;
      x1 = t + c1 * e;
      x2 = x2 + c2 * e;
      sse = sse + e * e;
      if (FUSE) {
        D[i] = add_dy<R>(D[i], cc) - g1a * e;
        if (R1) {
          const v2f tz = p1 + p2;
          const v2f ez = keep_if(D[i] - p1, k1, i & 31);
          p1 = tz + c1 * ez;
          p2 = p2 + c2 * ez;
        } else {
          p1 = p1 + wc[2 * R] * D[i];
          p2 = p2 + wc[2 * R + 1] * D[i];
        }
      } else if (i < HALF_HB) {
        D[i] = D[i] - g1a * e;
      }
    }
    d_steps<K, FUSE, R + 1, M2, R1>(q, cc, D, c1, c2, g1a, wc, x1, x2, sse, p1, p2, k2, k1);
  }
}

// pass 2 of a season from its true start state (x1, x2) = (f, b); FUSE: D advances to the
// next season (dy block `blk`) and feeds that season's pass 1; !FUSE (last season): only
// the first HALF_HB phases are advanced (they carry the forecast's seasonal terms).
// FUSE also prefetches the next scan's B^1, B^2, B^4, B^8 (scalar loads) during the last
// chunk, when the pass-1 weight registers of a next chunk are not needed: the scan then
// starts without waiting on the scalar cache.
// chunk 0 of a fused season (its dy chunk and pass-1 weights)
template <int K>
__device__ __forceinline__ void d_chunk0(const float* blk, cfp W, Chunk8f& c, v2f* w) {
  c.load(blk);
#pragma unroll
  for (int r = 0; r < 16; ++r)
    if (r < 2 * K) w[r] = ldv2(W + 2 * r);
}

template <int K, bool FUSE, bool M2 = false, bool R1 = false, int L = 32>
__device__ __forceinline__ void d_pass2(const float* blk, v2f* D, v2f c1, v2f c2, v2f g1a, cfp W, v2f& x1,
                                        v2f& x2, v2f& sse, v2f& p1, v2f& p2, cfp tb = nullptr,
                                        Mat2* Bn = nullptr, bool chk = false, const unsigned* ubp = nullptr,
                                        int* alive = nullptr, const Chunk8f* c0 = nullptr, const v2f* w0 = nullptr,
                                        unsigned k2lo = 0u, unsigned k2hi = 0u, unsigned k1lo = 0u,
                                        unsigned k1hi = 0u) {
  constexpr int NCH = (K + 7) / 8;
  constexpr bool WTS = FUSE && !R1;  // table pass 1: the chunk's weights
  if (FUSE) { p1 = splat2(0.f); p2 = splat2(0.f); }
  fence_sched();
  Chunk8f cc, cn;
  v2f wc[16], wn[16];
  // the prune bound, read at the season's start and compared at its last chunk (its LDS
  // round trip hides under the walk; a bound read early is only larger: it prunes less,
  // never wrongly)
  unsigned ub = 0x7f800000u;
  if (FUSE && chk) ub = __hip_atomic_load(ubp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (WTS) {
    if (c0) {  // chunk 0 was requested before the scan (its latency hides under it)
      cn = *c0;
#pragma unroll
      for (int r = 0; r < 16; ++r) wn[r] = w0[r];
    } else {
      d_chunk0<K>(blk, W, cn, wn);
    }
  } else if (FUSE) {
    cn.load(blk);
  }
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    if (FUSE && q + 1 == NCH && chk) {
      // grid branch and bound (hw_d_block): the SSE before the season's last chunk is a
      // lower bound of the pair's final SSE.  Checked here, before the B prefetch, where
      // the scalar registers of the next chunk's weights are free.
      // Only lanes 31 / 63 hold their half's sum and vote; the wave keeps the pair while
      // either of them does (the caller's __any).
      const v2f s = L == 32 ? half_sum_last(sse) : row_sum_last(sse);  // the same sum as the final SSE
      const float U = __uint_as_float(ub);
      int v = ((lane_id() & (L - 1)) == L - 1 && !(s.x > U && s.y > U)) ? 1 : 0;
      asm volatile("" : "+v"(v));  // the flag lives in a VGPR: no scalar register across the loop
      *alive = v;
    }
    if (WTS) {
      cc = cn;
#pragma unroll
      for (int r = 0; r < 16; ++r) wc[r] = wn[r];
      asm volatile("" ::"v"(cc.lo.x), "v"(cc.hi.x), "s"(wc[0].x));
      if (q + 1 < NCH) {
        W = launder(W);
        cn.load(blk + (q + 1) * D_CHUNK);
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (16 * (q + 1) + r < 2 * K) wn[r] = ldv2(W + 32 * (q + 1) + 2 * r);
      } else if (Bn) {
        tb = launder(tb);
#pragma unroll
        for (int b = 0; b < 4; ++b) Bn[b] = ldmat(tb + 8 * b);
      }
    } else if (FUSE) {  // recurrence pass 1: dy chunks only (the next scan is the general one)
      cc = cn;
      asm volatile("" ::"v"(cc.lo.x), "v"(cc.hi.x));
      if (q + 1 < NCH) cn.load(blk + (q + 1) * D_CHUNK);
    }
    fence_sched();
    // chunk q's steps 8q .. 8q + 7 lie in one 32-bit word of the lane's keep bits
    d_steps<K, FUSE, 0, M2, R1>(q, cc, D, c1, c2, g1a, wc, x1, x2, sse, p1, p2, q < 4 ? k2lo : k2hi,
                                q < 4 ? k1lo : k1hi);
    fence_sched();
  }
  // retire the B prefetch here (it landed during the last chunk) so the wait the compiler
  // needs for it is not placed after the caller's end-state ds_bpermutes
  if (WTS && Bn) {
    asm volatile("" ::"s"(Bn[0].a.x), "s"(Bn[3].d.y));
    fence_sched();
  }
}

// k-th grid pair of a block's queue: the (at most two, distinct) hint pairs packed in hp
// first, then [lo, ...) in order without them
__device__ __forceinline__ int hint_pair_at(int k, int lo, unsigned hp) {
  const int h0 = (int)(hp & 0xffffu), h1 = (int)(hp >> 16);
  const int nh = (h0 != 0xffff) + (h1 != 0xffff);
  if (k < nh) return (k == 0 && h0 != 0xffff) ? h0 : h1;
  int r = lo + k - nh;
  const int a0 = h0 < h1 ? h0 : h1, a1 = h0 < h1 ? h1 : h0;  // 0xffff sorts last, past every pair
  r += r >= a0 ? 1 : 0;
  r += r >= a1 ? 1 : 0;
  return r;
}

// Split tail (see fm_hw_d_fit): a workgroup may fit only the grid pairs [pi_lo, pi_hi)
// of its series pair; its per-series best then goes to slot `slot` of `cand` (half
// `hid`), and whichever half arrives second merges the two and finishes the series.
constexpr int CAND_FLOATS = 4 + HALF_HB;  // SSE, index bits, level, trend, seasonal phases

template <int K, bool PRUNE>
__device__ __forceinline__ void hw_d_block(const SmoothArgs& a, int hmax, int n0, int* deferred, int pi_lo,
                                           int pi_hi, int slot, int hid, int* cnt, float* cand, int hints) {
  constexpr int SEA = DLay<K>::SEASON;
  constexpr int TS = PairTab<K>::SIZE;
  constexpr int NMW = (32 * K + 31) / 32;  // season-0 validity bitmask words per series
  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  const int half = lane >> 5, j = lane & 31;
  const bool odd_row = ((lane >> 4) & 1) != 0;
  const int nseg = a.Tp / a.seg, m = a.m, ns1 = nseg - 1;

  // ---- LDS: dl[2][ns1][SEA] | vmask[2][NMW] | stat[4 waves][2][4] | flag | ylast[2][HB] | bests[4][2][HB] | wbest[4][2][4]
  //          | ubound[4]
  float* dl = (float*)fm_hw_smem;
  unsigned* vmask = (unsigned*)(dl + (size_t)2 * ns1 * SEA);
  float* stat = (float*)(vmask + 2 * NMW);
  int* flag = (int*)(stat + 8 * D_WAVES);
  float* ylast = (float*)(flag + 4);
  float* bests = ylast + 2 * HALF_HB;
  float* wbest = bests + 4 * 2 * HALF_HB;
  // [0..1] per-series SSE bound, [2] pair queue, [3] hint pairs (lo16 | hi16, 0xffff = none)
  unsigned* ubound = (unsigned*)(wbest + 4 * 2 * 4);

  // a pair the gapped kernel took in the last fit (its gap is almost always still in the
  // window: the ring moved a few columns) goes straight back to it, without staging here
  int* gflags = deferred + 4 + (a.N + 1) / 2;
  if (__builtin_amdgcn_readfirstlane(gflags[n0 >> 1])) {
    if (tid == 0 && hid == 0) {
      const int q = atomicAdd(deferred, 1);
      if (q < (a.N + 1) / 2) deferred[1 + q] = n0;
    }
    return;
  }
  for (int i = tid; i < 2 * NMW + 8 * D_WAVES + 4; i += blockDim.x) vmask[i] = 0u;  // vmask, stat, flag
  if (tid < 3) ubound[tid] = tid < 2 ? 0x7f800000u : 0u;  // +inf, +inf, queue 0
  if (tid == 3) {
    // hints: the grid pairs that won the previous fit of these series (a.best still holds it: only
    // this block -- or, split, the second arriver of its two halves -- rewrites it, at the
    // end) go first, so the branch and bound starts from a near-optimal bound
    unsigned hp[2] = {0xffffu, 0xffffu};
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int b = (hints && n0 + r < a.N) ? a.best[n0 + r] : -1;
      const int q = (b >= 0 && b < a.G) ? b / 2 : -1;
      if (q >= pi_lo && q < pi_hi && (r == 0 || (unsigned)q != hp[0])) hp[r] = (unsigned)q;
    }
    ubound[3] = hp[0] | (hp[1] << 16);
  }
  const int head = a.head_dev ? *a.head_dev : a.head;
  __syncthreads();

  // ---- stage: one thread per (series, 8 consecutive phases), all seasons of them in ------
  // flight at once.  Aligned rings (R, m, ld multiples of 8, 16-B row base): the phase
  // groups are shifted by phi = (pad - head) mod 8 so that each season's 8 columns are
  // one aligned 16-byte chunk (one load per season, no per-element address math);
  // otherwise one clamped 2-byte load per element.
  {
    constexpr int GRP = 8;
    const int R = a.ring_len;
    const bool al = (R % GRP == 0) && (m % GRP == 0) && (a.ld % GRP == 0) &&
                    ((((unsigned long long)a.hist) & 15ull) == 0);
    const int phi = al ? (((a.pad - head) % GRP) + GRP) % GRP : 0;
    const int ostart = phi ? phi - GRP : 0;
    const int ngrp = (m - ostart + GRP - 1) / GRP;
    float s0 = 0.f, c0 = 0.f, s1 = 0.f, c1 = 0.f, s0b = 0.f, c0b = 0.f, s1b = 0.f, c1b = 0.f;
    int bad = 0;
    for (int g = tid; g < 2 * ngrp; g += blockDim.x) {
      const int r = g >= ngrp ? 1 : 0, o0 = ostart + (g - r * ngrp) * GRP;
      const int n = n0 + r;
      const bool real = n < a.N;
      const bf16_t* row = (const bf16_t*)a.hist + (long long)(real ? n : 0) * a.ld;
      float y[D_MAXSEG][GRP];
      if (al) {
#pragma unroll
        for (int k = 0; k < D_MAXSEG; ++k) {
          const int t0 = k * m + o0 - a.pad;  // logical index of element 0 (multiple-of-8 column)
          int c = (head + t0) % R;
          c += c < 0 ? R : 0;
          uint4 w = make_uint4(0u, 0u, 0u, 0u);
          if (k < nseg) w = *(const uint4*)(row + c);  // k < nseg is block-uniform
          const unsigned ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
          for (int u = 0; u < GRP; ++u) {
            const unsigned x = ww[u >> 1];
            const float v = __uint_as_float((u & 1) ? (x & 0xffff0000u) : (x << 16));
            const bool ok = real && k < nseg;
            // the padding series of an odd N is zeros (keeps the pair on the fast path)
            y[k][u] = ok ? (t0 + u >= 0 ? v : fm_nan()) : 0.f;
          }
        }
      } else {
#pragma unroll
        for (int k = 0; k < D_MAXSEG; ++k) {
#pragma unroll
          for (int u = 0; u < GRP; ++u) {
            // branch-free: every load is issued (clamped to a valid column) and the value
            // selected afterwards, so all of them are in flight before the first wait
            const bool ok = real && k < nseg && o0 + u < m;
            const int t = k * m + o0 + u - a.pad;
            const bool pos = t >= 0;
            int c = head + ((ok && pos) ? t : 0);
            c -= (c >= R) ? R : 0;
            const float v = bf16_to_f32(row[c]);
            y[k][u] = ok ? (pos ? v : fm_nan()) : 0.f;
          }
        }
      }
      // (lane, step) of the group's first in-range phase; later phases step from it
      const int ob = o0 > 0 ? o0 : 0;
      const int jjb = ob / K, ib = ob - jjb * K;
      unsigned vlo = 0u, vhi = 0u;  // season-0 validity bits for words o0 >> 5 and (o0 + 7) >> 5
#pragma unroll
      for (int u = 0; u < GRP; ++u) {
        const int o = o0 + u;
        if (o >= 0 && o < m) {
          int i = ib + (o - ob), jj = jjb;
          if (i >= K) { i -= K; ++jj; }
          const bool v0 = y[0][u] == y[0][u];
          float* blk = dl + (size_t)r * ns1 * SEA + dl_off(i, jj);
          blk[0] = v0 ? y[1][u] - y[0][u] : y[1][u];  // + l0 for valid y0 once the means are known
          if (v0) {
            if ((o >> 5) == ((o0 < 0 ? 0 : o0) >> 5)) vlo |= 1u << (o & 31);
            else vhi |= 1u << (o & 31);
          }
#pragma unroll
          for (int k = 1; k < D_MAXSEG - 1; ++k)
            if (k < ns1) blk[(size_t)k * SEA] = y[k + 1][u] - y[k][u];
#pragma unroll
          for (int k = 1; k < D_MAXSEG; ++k)
            if (k < nseg && y[k][u] != y[k][u]) bad = 1;
          if (o < HALF_HB) {
            float yl = y[1][u];
#pragma unroll
            for (int k = 2; k < D_MAXSEG; ++k)
              if (k == ns1) yl = y[k][u];
            ylast[r * HALF_HB + o] = yl;
          }
          const bool v1 = y[1][u] == y[1][u];
          const float y0v = v0 ? y[0][u] : 0.f, y0c = v0 ? 1.f : 0.f;
          const float y1v = v1 ? y[1][u] : 0.f, y1c = v1 ? 1.f : 0.f;
          if (r == 0) { s0 += y0v; c0 += y0c; s1 += y1v; c1 += y1c; }
          else { s0b += y0v; c0b += y0c; s1b += y1v; c1b += y1c; }
        }
      }
      const int wlo = (o0 < 0 ? 0 : o0) >> 5;
      if (vlo) atomicOr(&vmask[r * NMW + wlo], vlo);
      if (vhi) atomicOr(&vmask[r * NMW + wlo + 1], vhi);
    }
    s0 = wave_sum(s0); c0 = wave_sum(c0); s1 = wave_sum(s1); c1 = wave_sum(c1);
    s0b = wave_sum(s0b); c0b = wave_sum(c0b); s1b = wave_sum(s1b); c1b = wave_sum(c1b);
    // per-wave slots summed in wave order below: a float atomicAdd's order would make l0 / b0
    // (and a beta = 0 fit's trend) differ in the last bit from run to run
    if (lane == 0) {
      float* sw = stat + 8 * w;
      sw[0] = s0; sw[1] = c0; sw[2] = s1; sw[3] = c1;
      sw[4] = s0b; sw[5] = c0b; sw[6] = s1b; sw[7] = c1b;
    }
    if (bad) atomicOr(flag, 1);
  }
  __syncthreads();
  if (*flag) {  // block-uniform: a gap past season 0 — the gapped kernel takes the pair
    if (tid == 0 && hid == 0) {
      const int q = atomicAdd(deferred, 1);
      if (q < (a.N + 1) / 2) deferred[1 + q] = n0;  // a stale count can never write past the pair list
      gflags[n0 >> 1] = 1;
    }
    return;
  }
  float l0r[2], b0r[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    float st[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int v = 0; v < D_WAVES; ++v)
#pragma unroll
      for (int u = 0; u < 4; ++u) st[u] += stat[8 * v + 4 * r + u];
    l0r[r] = st[1] > 0.f ? st[0] / st[1] : 0.f;
    b0r[r] = ((st[3] > 0.f ? st[2] / st[3] : 0.f) - l0r[r]) / (float)m;
  }
  // D^(1) = y1 - s0 with s0 = y0 - l0 where y0 is valid (0 elsewhere)
  for (int col = tid; col < 2 * m; col += blockDim.x) {
    const int r = col >= m ? 1 : 0, o = col - r * m;
    if ((vmask[r * NMW + (o >> 5)] >> (o & 31)) & 1u) {
      const int jj = o / K, i = o - jj * K;
      dl[(size_t)r * ns1 * SEA + dl_off(i, jj)] += l0r[r];
    }
  }
  __syncthreads();

  const float l0 = half ? l0r[1] : l0r[0], b0 = half ? b0r[1] : b0r[0];
  const float* mydl = dl + (size_t)half * ns1 * SEA + j * 4;
  const int last_addr = ((lane & 32) | 31) << 2;  // bpermute source: lane 31 / 63
  float bestSSE = __builtin_huge_valf();
  int bestIdx = 0x7fffffff;
  float bestL = l0, bestB = b0;
  float* mybest = bests + (w * 2 + half) * HALF_HB;
  const int nwaves = blockDim.x / FM_WAVE;
  // Exact branch and bound over the grid (PRUNE): ubound[half] is the smallest
  // complete SSE any wave of this block has found for that series.  A per-lane SSE only
  // grows (fl(s + e*e) >= s) and the DPP half sum is one fixed tree of adds, monotone in
  // its operands, so a pair whose partial sum in season sg already exceeds the bound
  // (strictly, for both series and both grid points) ends above it and can never be the
  // argmin or tie it: the wave drops it and takes the next pair from the block's queue.
  // Queue order: the hint pairs (previous winners), then the rest in grid order.
  const int npb = pi_hi - pi_lo;
  // the hint pairs are fixed for the block: read once (an LDS round trip per pair otherwise)
  const unsigned hints_pp = (unsigned)__builtin_amdgcn_readfirstlane((int)ubound[3]);
  for (int k = w; k < npb;) {
    const int pi = hint_pair_at(k, pi_lo, hints_pp);
    const int c0 = 2 * pi;
    const int c1i = (2 * pi + 1 < a.G) ? 2 * pi + 1 : c0;
    const cfp tab = const_ptr(a.pair_tab + (size_t)pi * TS);
    const v2f c1 = ldv2(tab), c2 = ldv2(tab + 2), g1a = ldv2(tab + 4);
    const cfp W = tab + PairTab<K>::W0;
    const cfp tb = tab + PairTab<K>::B0;
    const v2f one = splat2(1.f), zero = splat2(0.f);
    Mat2 Bj;  // B^(lane & 15)
    Mat2 Bp[4];  // B^1, B^2, B^4, B^8 of the next scan
    Bj.a = one; Bj.b = zero; Bj.c = zero; Bj.d = one;
#pragma unroll
    for (int bit = 0; bit < 4; ++bit) Bp[bit] = ldmat(tb + 8 * bit);
    fence_sched();  // all four requested before the first is used: one scalar-cache wait, not four
#pragma unroll
    for (int bit = 0; bit < 4; ++bit) {
      const Mat2 r = matmul(Bj, Bp[bit]);
      if ((lane >> bit) & 1) Bj = r;
    }
    v2f D[K];
    v2f X1 = splat2(l0 + b0), X2 = splat2(b0), sse = zero;  // (f, b) at the season start
    v2f p1, p2;
    d_pass1<K>(mydl, W, D, p1, p2);
    int alive = 1;  // per lane: 0 once this lane's partial SSEs exceed the bound (read wave-wide)
    for (int sg = 1; sg < nseg - 1; ++sg) {
      v2f x1, x2;
      Chunk8f c0;
      v2f w0[16];
      d_chunk0<K>(mydl + (size_t)sg * SEA, launder(W), c0, w0);  // in flight during the scan
      half_uniform_scan_pre(Bp, launder(tb), p1, p2, X1, X2, Bj, odd_row, x1, x2);
      d_pass2<K, true>(mydl + (size_t)sg * SEA, D, c1, c2, g1a, launder(W), x1, x2, sse, p1, p2, tb, Bp,
                       PRUNE, ubound + half, &alive, &c0, w0);
      X1 = half_last_bp(x1, last_addr);
      X2 = half_last_bp(x2, last_addr);
      if (PRUNE && !__any(alive)) break;
    }
    if (!PRUNE || __any(alive)) {
      v2f x1, x2, d1, d2;
      half_uniform_scan_pre(Bp, tb, p1, p2, X1, X2, Bj, odd_row, x1, x2);
      d_pass2<K, false>(mydl, D, c1, c2, g1a, W, x1, x2, sse, d1, d2);
      X1 = half_last_bp(x1, last_addr);
      X2 = half_last_bp(x2, last_addr);
      sse = half_sum_last(sse);
      sse = half_last_bp(sse, last_addr);  // lane 31 / 63 -> the whole half
      const bool upd0 = (sse.x < bestSSE || (sse.x == bestSSE && c0 < bestIdx));
      if (upd0) { bestSSE = sse.x; bestIdx = c0; bestL = X1.x - X2.x; bestB = X2.x; }
      const bool upd1 = (c1i != c0) && (sse.y < bestSSE || (sse.y == bestSSE && c1i < bestIdx));
      if (upd1) { bestSSE = sse.y; bestIdx = c1i; bestL = X1.y - X2.y; bestB = X2.y; }
      if (j == 0 && (upd0 || upd1)) {
        const float* yl = ylast + half * HALF_HB;
#pragma unroll
        for (int i = 0; i < K && i < HALF_HB; ++i)
          if (i < hmax) mybest[i] = yl[i] - (upd1 ? D[i].y : D[i].x);
      }
      // publish the bound (SSE >= 0: float order is unsigned-int order; a NaN never lowers it)
      if (PRUNE && j == 0 && (upd0 || upd1))
        __hip_atomic_fetch_min(ubound + half, __float_as_uint(bestSSE), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // next pair: the first round is static (pi_lo + w), later ones come from the queue
    int q = 0;
    if (lane == 0)
      q = __hip_atomic_fetch_add(ubound + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    k = nwaves + __builtin_amdgcn_readfirstlane(q);
  }

  // ---- arg-min across the 4 waves; wave r finishes series n0 + r ----------------------
  if (j == 0) {
    float* wb = wbest + (w * 2 + half) * 4;
    wb[0] = bestSSE;
    wb[1] = __int_as_float(bestIdx);
    wb[2] = bestL;
    wb[3] = bestB;
  }
  __syncthreads();
  if (w >= 2) return;
  const int r = w, n = n0 + r;
  if (n >= a.N) return;
  int win = 0;
  for (int q = 1; q < nwaves; ++q) {
    const float sq = wbest[(q * 2 + r) * 4], sw = wbest[(win * 2 + r) * 4];
    const int iq = __float_as_int(wbest[(q * 2 + r) * 4 + 1]), iw = __float_as_int(wbest[(win * 2 + r) * 4 + 1]);
    if (sq < sw || (sq == sw && iq < iw)) win = q;
  }
  const float* wb = wbest + (win * 2 + r) * 4;
  float gSSE = wb[0], gL = wb[2], gB = wb[3];
  int gIdx = __float_as_int(wb[1]);
  float* sb = bests + (win * 2 + r) * HALF_HB;
  if (slot >= 0) {
    // publish this half's best: system-scope (sc0 sc1) stores, which write through every
    // cache level, drained before the device-scope arrival count; the second arriver reads
    // them with system-scope loads, which bypass its XCD's L2 (an agent-scope sc1 load
    // could hit a line left there by an earlier call: the L2 is per XCD)
    float* mine = cand + (((size_t)slot * 2 + hid) * 2 + r) * CAND_FLOATS;
    if (lane < HALF_HB) __hip_atomic_store(&mine[4 + lane], sb[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (lane == 0) {
      __hip_atomic_store(&mine[0], gSSE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&mine[1], __int_as_float(gIdx), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&mine[2], gL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&mine[3], gB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int prev = 0;
    if (lane == 0) prev = __hip_atomic_fetch_add(&cnt[slot * 2 + r], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    prev = __shfl(prev, 0, FM_WAVE);
    if (prev == 0) return;  // first half in: the other one finishes this series
    // second arriver: the last user of this counter in the launch resets it for the next one
    if (lane == 0) __hip_atomic_store(&cnt[slot * 2 + r], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float* oth = cand + (((size_t)slot * 2 + (1 - hid)) * 2 + r) * CAND_FLOATS;
    const float oSSE = __hip_atomic_load(&oth[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const int oIdx = __float_as_int(__hip_atomic_load(&oth[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (oSSE < gSSE || (oSSE == gSSE && oIdx < gIdx)) {  // same tie rule as the in-block argmin
      gSSE = oSSE;
      gIdx = oIdx;
      gL = __hip_atomic_load(&oth[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      gB = __hip_atomic_load(&oth[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (lane < HALF_HB) sb[lane] = __hip_atomic_load(&oth[4 + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
  }
  const float nvr = (float)(ns1 * m);  // fast path: every sample past season 0 is valid
  const float sig = sqrtf(gSSE / fmaxf(nvr, 1.f));
  if (lane == 0) {
    a.level[n] = gL;
    a.trend[n] = gB;
    a.sigma[n] = sig;
    a.best[n] = gIdx;
  }
  const int Tp = a.Tp;
  if (a.season_hb && lane < hmax) a.season_hb[(long long)n * HALF_HB + lane] = sb[lane];
  if (a.nvalid_out && lane == 0) a.nvalid_out[n] = nvr;
  detect_epilogue_wave(a.det, n, sig, nvr, [&](int h) {
    int ph = (Tp - 1 + h) % m;
    if (ph < 0) ph += m;
    ph = ph < HALF_HB ? ph : HALF_HB - 1;  // host guarantees ph < hmax; clamp keeps LDS reads in bounds
    return gL + (float)h * gB + sb[ph];
  }, gIdx);
}

// Workgroups [0, n_full) fit whole series pairs 0..n_full-1; the rest are split-tail
// halves: workgroup n_full + 2 s + h fits half h of the grid of pair n_full + s.
template <int K, bool PRUNE>
__global__ __launch_bounds__(256, 2) void hw_d_kernel(const SmoothArgs a, int hmax, int* deferred, int n_full,
                                                     int* cnt, float* cand, int hints) {
  const int b = blockIdx.x;
  const int npairs = (a.G + 1) / 2;
  if (b < n_full) {
    hw_d_block<K, PRUNE>(a, hmax, 2 * b, deferred, 0, npairs, -1, 0, cnt, cand, hints);
    return;
  }
  const int item = b - n_full, slot = item >> 1, h = item & 1, mid = npairs / 2;
  hw_d_block<K, PRUNE>(a, hmax, 2 * (n_full + slot), deferred, h ? mid : 0, h ? npairs : mid, slot, h, cnt, cand,
                       hints);
}


// ---- variant 5 at short seasons: hw_q_kernel (four series per wave) ---------------------------
// A daily season m = 16 K (the 300 s step: 288 = 16 x 18) walked by 16 lanes per series, four
// series per wave (one per DPP row) and per workgroup.  Against the 32-lane layout at K = 9
// the per-season fixed work -- the lane scan, its B loads, the end-state broadcast, the prune
// vote -- is spread over 18 steps instead of 9 and the scan loses its cross-row stage.  Same
// residual-state walk and table pass 1 as hw_d_block (d_pass1 / d_pass2 are lane-count
// agnostic; the prune vote sums over a row, L = 16), same outputs.  A quad with a gap past
// season 0 goes, as its two series pairs, to the 32-lane gapped kernel (hw_dg_kernel<m / 32>,
// launched with its own pair table); the hints are those of the first two series (the
// branch and bound is exact in any order).
constexpr int Q_S = 4;  // series per wave / workgroup
template <int K, bool PRUNE>
__device__ __forceinline__ void hw_q_block(const SmoothArgs& a, int hmax, int n0, int* deferred, int hints) {
  constexpr int SEA = DLay<K>::SEASON;
  constexpr int TS = PairTab<K>::SIZE;
  constexpr int M = 16 * K;
  constexpr int NMW = (M + 31) / 32;
  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  const int sid = lane >> 4, j = lane & 15;
  const int nseg = a.Tp / a.seg, m = a.m, ns1 = nseg - 1;

  // ---- LDS: dl[4][ns1][SEA] | vmask[4][NMW] | stat[4 waves][4][4] | flag | ylast[4][HB] | bests[4][4][HB]
  //          | wbest[4][4][4] | ubound[4] | queue | hints
  float* dl = (float*)fm_hw_smem;
  unsigned* vmask = (unsigned*)(dl + (size_t)Q_S * ns1 * SEA);
  float* stat = (float*)(vmask + Q_S * NMW);
  int* flag = (int*)(stat + 4 * Q_S * D_WAVES);
  float* ylast = (float*)(flag + 4);
  float* bests = ylast + Q_S * HALF_HB;
  float* wbest = bests + 4 * Q_S * HALF_HB;
  unsigned* ubound = (unsigned*)(wbest + 4 * Q_S * 4);  // [0..3] bounds, [4] queue, [5] hints

  const int P = (a.N + 1) / 2;
  int* gflags = deferred + 4 + P;
  const int pa = n0 >> 1, pb = (n0 + 2 < a.N) ? pa + 1 : -1;  // the quad's two series pairs
  const auto defer = [&]() {
    if (tid == 0) {
      const int q = atomicAdd(deferred, pb >= 0 ? 2 : 1);
      if (q < P) deferred[1 + q] = n0;
      if (pb >= 0 && q + 1 < P) deferred[2 + q] = n0 + 2;
      gflags[pa] = 1;
      if (pb >= 0) gflags[pb] = 1;
    }
  };
  if (__builtin_amdgcn_readfirstlane(gflags[pa] | (pb >= 0 ? gflags[pb] : 0))) {
    defer();
    return;
  }
  for (int i = tid; i < Q_S * NMW + 4 * Q_S * D_WAVES + 4; i += blockDim.x) vmask[i] = 0u;  // vmask, stat, flag
  if (tid < Q_S + 1) ubound[tid] = tid < Q_S ? 0x7f800000u : 0u;  // +inf per series, queue 0
  if (tid == Q_S + 1) {
    unsigned hp[2] = {0xffffu, 0xffffu};
    const int npairs = (a.G + 1) / 2;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int b = (hints && n0 + r < a.N) ? a.best[n0 + r] : -1;
      const int q = (b >= 0 && b < a.G) ? b / 2 : -1;
      if (q >= 0 && q < npairs && (r == 0 || (unsigned)q != hp[0])) hp[r] = (unsigned)q;
    }
    ubound[Q_S + 1] = hp[0] | (hp[1] << 16);
  }
  const int head = a.head_dev ? *a.head_dev : a.head;
  __syncthreads();

  // ---- stage: one thread per (series, 8 consecutive phases), all seasons of them in flight
  {
    constexpr int GRP = 8;
    const int R = a.ring_len;
    const bool al = (R % GRP == 0) && (m % GRP == 0) && (a.ld % GRP == 0) &&
                    ((((unsigned long long)a.hist) & 15ull) == 0);
    const int phi = al ? (((a.pad - head) % GRP) + GRP) % GRP : 0;
    const int ostart = phi ? phi - GRP : 0;
    const int ngrp = (m - ostart + GRP - 1) / GRP;
    float acc[Q_S][4];
#pragma unroll
    for (int r = 0; r < Q_S; ++r)
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[r][u] = 0.f;
    int bad = 0;
    for (int g = tid; g < Q_S * ngrp; g += blockDim.x) {
      const int r = g / ngrp, o0 = ostart + (g - r * ngrp) * GRP;
      const int n = n0 + r;
      const bool real = n < a.N;
      const bf16_t* row = (const bf16_t*)a.hist + (long long)(real ? n : 0) * a.ld;
      float y[D_MAXSEG][GRP];
      if (al) {
#pragma unroll
        for (int k = 0; k < D_MAXSEG; ++k) {
          const int t0 = k * m + o0 - a.pad;
          int c = (head + t0) % R;
          c += c < 0 ? R : 0;
          uint4 wv = make_uint4(0u, 0u, 0u, 0u);
          if (k < nseg) wv = *(const uint4*)(row + c);
          const unsigned ww[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
          for (int u = 0; u < GRP; ++u) {
            const unsigned x = ww[u >> 1];
            const float v = __uint_as_float((u & 1) ? (x & 0xffff0000u) : (x << 16));
            const bool ok = real && k < nseg;
            y[k][u] = ok ? (t0 + u >= 0 ? v : fm_nan()) : 0.f;
          }
        }
      } else {
#pragma unroll
        for (int k = 0; k < D_MAXSEG; ++k) {
#pragma unroll
          for (int u = 0; u < GRP; ++u) {
            const bool ok = real && k < nseg && o0 + u < m;
            const int t = k * m + o0 + u - a.pad;
            const bool pos = t >= 0;
            int c = head + ((ok && pos) ? t : 0);
            c -= (c >= R) ? R : 0;
            const float v = bf16_to_f32(row[c]);
            y[k][u] = ok ? (pos ? v : fm_nan()) : 0.f;
          }
        }
      }
      float s0 = 0.f, c0 = 0.f, s1 = 0.f, c1 = 0.f;
#pragma unroll
      for (int u = 0; u < GRP; ++u) {
        const int o = o0 + u;
        if (o >= 0 && o < m) {
          const int jj = o / K, i = o - jj * K;
          const bool v0 = y[0][u] == y[0][u];
          float* blk = dl + (size_t)r * ns1 * SEA + dl_off(i, jj);
          blk[0] = v0 ? y[1][u] - y[0][u] : y[1][u];  // + l0 for valid y0 once the means are known
          if (v0) atomicOr(&vmask[r * NMW + (o >> 5)], 1u << (o & 31));
#pragma unroll
          for (int k = 1; k < D_MAXSEG - 1; ++k)
            if (k < ns1) blk[(size_t)k * SEA] = y[k + 1][u] - y[k][u];
#pragma unroll
          for (int k = 1; k < D_MAXSEG; ++k)
            if (k < nseg && y[k][u] != y[k][u]) bad = 1;
          if (o < HALF_HB) {
            float yl = y[1][u];
#pragma unroll
            for (int k = 2; k < D_MAXSEG; ++k)
              if (k == ns1) yl = y[k][u];
            ylast[r * HALF_HB + o] = yl;
          }
          const bool v1 = y[1][u] == y[1][u];
          s0 += v0 ? y[0][u] : 0.f;
          c0 += v0 ? 1.f : 0.f;
          s1 += v1 ? y[1][u] : 0.f;
          c1 += v1 ? 1.f : 0.f;
        }
      }
#pragma unroll
      for (int q = 0; q < Q_S; ++q)
        if (q == r) { acc[q][0] += s0; acc[q][1] += c0; acc[q][2] += s1; acc[q][3] += c1; }
    }
    // per-wave slots summed in wave order below (deterministic, see hw_d_block)
#pragma unroll
    for (int q = 0; q < Q_S; ++q)
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[q][u] = wave_sum(acc[q][u]);
    if (lane == 0) {
      float* sw = stat + 4 * Q_S * w;
#pragma unroll
      for (int q = 0; q < Q_S; ++q)
#pragma unroll
        for (int u = 0; u < 4; ++u) sw[4 * q + u] = acc[q][u];
    }
    if (bad) atomicOr(flag, 1);
  }
  __syncthreads();
  if (*flag) {  // block-uniform: a gap past season 0 — the 32-lane gapped kernel takes both pairs
    defer();
    return;
  }
  float l0r[Q_S], b0r[Q_S];
#pragma unroll
  for (int r = 0; r < Q_S; ++r) {
    float st[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int v = 0; v < D_WAVES; ++v)
#pragma unroll
      for (int u = 0; u < 4; ++u) st[u] += stat[4 * Q_S * v + 4 * r + u];
    l0r[r] = st[1] > 0.f ? st[0] / st[1] : 0.f;
    b0r[r] = ((st[3] > 0.f ? st[2] / st[3] : 0.f) - l0r[r]) / (float)m;
  }
  for (int col = tid; col < Q_S * m; col += blockDim.x) {
    const int r = col / m, o = col - r * m;
    if ((vmask[r * NMW + (o >> 5)] >> (o & 31)) & 1u) {
      const int jj = o / K, i = o - jj * K;
      dl[(size_t)r * ns1 * SEA + dl_off(i, jj)] += l0r[r];
    }
  }
  __syncthreads();

  const float l0 = sid == 0 ? l0r[0] : sid == 1 ? l0r[1] : sid == 2 ? l0r[2] : l0r[3];
  const float b0 = sid == 0 ? b0r[0] : sid == 1 ? b0r[1] : sid == 2 ? b0r[2] : b0r[3];
  const float* mydl = dl + (size_t)sid * ns1 * SEA + j * 4;
  const int last_addr = ((lane & 48) | 15) << 2;  // bpermute source: lane 15 of the row
  float bestSSE = __builtin_huge_valf();
  int bestIdx = 0x7fffffff;
  float bestL = l0, bestB = b0;
  float* mybest = bests + (w * Q_S + sid) * HALF_HB;
  const int nwaves = blockDim.x / FM_WAVE;
  const int npb = (a.G + 1) / 2;
  const unsigned hints_pp = (unsigned)__builtin_amdgcn_readfirstlane((int)ubound[Q_S + 1]);
  for (int k = w; k < npb;) {
    const int pi = hint_pair_at(k, 0, hints_pp);
    const int c0 = 2 * pi;
    const int c1i = (2 * pi + 1 < a.G) ? 2 * pi + 1 : c0;
    const cfp tab = const_ptr(a.pair_tab + (size_t)pi * TS);
    const v2f c1 = ldv2(tab), c2 = ldv2(tab + 2), g1a = ldv2(tab + 4);
    const cfp W = tab + PairTab<K>::W0;
    const cfp tb = tab + PairTab<K>::B0;
    const v2f one = splat2(1.f), zero = splat2(0.f);
    Mat2 Bj;
    Mat2 Bp[4];
    Bj.a = one; Bj.b = zero; Bj.c = zero; Bj.d = one;
#pragma unroll
    for (int bit = 0; bit < 4; ++bit) Bp[bit] = ldmat(tb + 8 * bit);
    fence_sched();
#pragma unroll
    for (int bit = 0; bit < 4; ++bit) {
      const Mat2 r = matmul(Bj, Bp[bit]);
      if ((lane >> bit) & 1) Bj = r;
    }
    v2f D[K];
    v2f X1 = splat2(l0 + b0), X2 = splat2(b0), sse = zero;
    v2f p1, p2;
    d_pass1<K>(mydl, W, D, p1, p2);
    int alive = 1;
    for (int sg = 1; sg < nseg - 1; ++sg) {
      v2f x1, x2;
      Chunk8f c0;
      v2f w0[16];
      d_chunk0<K>(mydl + (size_t)sg * SEA, launder(W), c0, w0);
      row_uniform_scan_pre(Bp, p1, p2, X1, X2, Bj, x1, x2);
      d_pass2<K, true, false, false, 16>(mydl + (size_t)sg * SEA, D, c1, c2, g1a, launder(W), x1, x2, sse, p1, p2,
                                         tb, Bp, PRUNE, ubound + sid, &alive, &c0, w0);
      X1 = half_last_bp(x1, last_addr);
      X2 = half_last_bp(x2, last_addr);
      if (PRUNE && !__any(alive)) break;
    }
    if (!PRUNE || __any(alive)) {
      v2f x1, x2, d1, d2;
      row_uniform_scan_pre(Bp, p1, p2, X1, X2, Bj, x1, x2);
      d_pass2<K, false, false, false, 16>(mydl, D, c1, c2, g1a, W, x1, x2, sse, d1, d2);
      X1 = half_last_bp(x1, last_addr);
      X2 = half_last_bp(x2, last_addr);
      sse = row_sum_last(sse);
      sse = half_last_bp(sse, last_addr);  // lane 15 of the row -> the whole row
      const bool upd0 = (sse.x < bestSSE || (sse.x == bestSSE && c0 < bestIdx));
      if (upd0) { bestSSE = sse.x; bestIdx = c0; bestL = X1.x - X2.x; bestB = X2.x; }
      const bool upd1 = (c1i != c0) && (sse.y < bestSSE || (sse.y == bestSSE && c1i < bestIdx));
      if (upd1) { bestSSE = sse.y; bestIdx = c1i; bestL = X1.y - X2.y; bestB = X2.y; }
      if (j == 0 && (upd0 || upd1)) {
        const float* yl = ylast + sid * HALF_HB;
#pragma unroll
        for (int i = 0; i < K && i < HALF_HB; ++i)
          if (i < hmax) mybest[i] = yl[i] - (upd1 ? D[i].y : D[i].x);
      }
      if (PRUNE && j == 0 && (upd0 || upd1))
        __hip_atomic_fetch_min(ubound + sid, __float_as_uint(bestSSE), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    int q = 0;
    if (lane == 0)
      q = __hip_atomic_fetch_add(ubound + Q_S, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    k = nwaves + __builtin_amdgcn_readfirstlane(q);
  }

  // ---- arg-min across the 4 waves; wave r finishes series n0 + r ----------------------
  if (j == 0) {
    float* wb = wbest + (w * Q_S + sid) * 4;
    wb[0] = bestSSE;
    wb[1] = __int_as_float(bestIdx);
    wb[2] = bestL;
    wb[3] = bestB;
  }
  __syncthreads();
  if (w >= Q_S) return;
  const int r = w, n = n0 + r;
  if (n >= a.N) return;
  int win = 0;
  for (int q = 1; q < nwaves; ++q) {
    const float sq = wbest[(q * Q_S + r) * 4], sw = wbest[(win * Q_S + r) * 4];
    const int iq = __float_as_int(wbest[(q * Q_S + r) * 4 + 1]), iw = __float_as_int(wbest[(win * Q_S + r) * 4 + 1]);
    if (sq < sw || (sq == sw && iq < iw)) win = q;
  }
  const float* wb = wbest + (win * Q_S + r) * 4;
  const float gSSE = wb[0], gL = wb[2], gB = wb[3];
  const int gIdx = __float_as_int(wb[1]);
  const float* sb = bests + (win * Q_S + r) * HALF_HB;
  const float nvr = (float)(ns1 * m);  // fast path: every sample past season 0 is valid
  const float sig = sqrtf(gSSE / fmaxf(nvr, 1.f));
  if (lane == 0) {
    a.level[n] = gL;
    a.trend[n] = gB;
    a.sigma[n] = sig;
    a.best[n] = gIdx;
  }
  const int Tp = a.Tp;
  if (a.season_hb && lane < hmax) a.season_hb[(long long)n * HALF_HB + lane] = sb[lane];
  if (a.nvalid_out && lane == 0) a.nvalid_out[n] = nvr;
  detect_epilogue_wave(a.det, n, sig, nvr, [&](int h) {
    int ph = (Tp - 1 + h) % m;
    if (ph < 0) ph += m;
    ph = ph < HALF_HB ? ph : HALF_HB - 1;
    return gL + (float)h * gB + sb[ph];
  }, gIdx);
}

template <int K, bool PRUNE>
__global__ __launch_bounds__(256, 2) void hw_q_kernel(const SmoothArgs a, int hmax, int* deferred, int hints) {
  hw_q_block<K, PRUNE>(a, hmax, 4 * blockIdx.x, deferred, hints);
}

// ---- variant 5, gapped series: hw_dg_kernel ------------------------------------------------
// A series pair with a missing observation past season 0 leaves hw_d_kernel (which keeps its
// straight-line dense walk) for this kernel, persistent over the deferred list.  Same
// residual-state walk, same semantics as the fp64 reference (models/smoothing.py): a missing
// step carries the forecast (e = 0: no SSE term, no seasonal update) and sigma divides by the
// valid points.  Per season the pair takes the dense code unless that season has a gap:
//  * a missing y is imputed as 0 in the season-difference image (D = y* - s stays the exact
//    residual chain: y* never reaches an error, the step is masked) and flagged in a 64-bit
//    per-(series, season, lane) miss mask;
//  * pass 2 of a gapped season masks e at its missing steps (keep_if: 3 VALU per step);
//  * pass 1 of a gapped NEXT season runs as the masked recurrence from a zero state (4 ops per
//    step instead of the 2 of the table sum, whose uniform weights assume no gap): its end
//    state is the lane map's exact offset v; the map's matrix M is the product of the lane's
//    step matrices, A for an observed step and A_m = [[1, 1], [0, 1]] for a missing one,
//    assembled run by run from a table of A^0 .. A^K (lane_map);
//  * the season after such a pass 1 takes the general affine scan (per-lane M, v), the
//    others the uniform-matrix scan.
// So a pair pays the gap code only in the seasons that hold a gap (a 30-minute outage: one
// season), and the dense kernel is untouched.
template <int K>
__device__ __forceinline__ Mat2 pow_at(const float* pw, int n) {
  const float4 lo = *(const float4*)(pw + 8 * n), hi = *(const float4*)(pw + 8 * n + 4);
  Mat2 m;
  m.a.x = lo.x; m.a.y = lo.y; m.b.x = lo.z; m.b.y = lo.w;
  m.c.x = hi.x; m.c.y = hi.y; m.d.x = hi.z; m.d.y = hi.w;
  return m;
}

// The lane's season map matrix from its miss bits (bit i: step i missing): runs of observed
// steps are table powers A^n, a run of r missing steps is A_m^r = [[1, r], [0, 1]].  The
// loop runs as often as the lane of the wave with the most miss runs (usually 1-3).
template <int K>
__device__ __forceinline__ Mat2 lane_map(const float* pw, unsigned lo, unsigned hi) {
  unsigned long long b = ((unsigned long long)hi << 32) | lo;
  Mat2 M;
  M.a = splat2(1.f); M.b = splat2(0.f); M.c = splat2(0.f); M.d = splat2(1.f);
  int pos = 0;
  while (__any(b != 0ull)) {
    if (b != 0ull) {
      const int i0 = __builtin_ctzll(b);
      const unsigned long long rest = ~(b >> i0);
      const int r = rest ? __builtin_ctzll(rest) : 64 - i0;
      M = matmul(pow_at<K>(pw, i0 - pos), M);
      const v2f rr = splat2((float)r);
      M.a = M.a + rr * M.c;
      M.b = M.b + rr * M.d;
      pos = i0 + r;
      b = pos >= 64 ? 0ull : (b >> pos) << pos;
    }
  }
  return matmul(pow_at<K>(pw, K - pos), M);
}

// pass 1 of season 1 as the masked recurrence (D^(1) from LDS into the D registers)
template <int K, int R>
__device__ __forceinline__ void dg_pass1_steps(int q, const Chunk8f& cc, v2f* D, v2f c1, v2f c2, unsigned kw, v2f& p1,
                                               v2f& p2) {
  if constexpr (R < 8) {
    const int i = 8 * q + R;
    if (i < K) {
      D[i] = pk_splat<R & 1>(chunk_pair<R>(cc));
      const v2f t = p1 + p2;
      const v2f e = keep_if(D[i] - p1, kw, i & 31);
      p1 = t + c1 * e;
      p2 = p2 + c2 * e;
    }
    dg_pass1_steps<K, R + 1>(q, cc, D, c1, c2, kw, p1, p2);
  }
}
template <int K>
__device__ __forceinline__ void dg_pass1_rec(const float* blk, v2f* D, v2f c1, v2f c2, unsigned klo, unsigned khi,
                                             v2f& p1, v2f& p2) {
  constexpr int NCH = (K + 7) / 8;
  p1 = splat2(0.f);
  p2 = splat2(0.f);
  Chunk8f cc, cn;
  cn.load(blk);
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    cc = cn;
    if (q + 1 < NCH) cn.load(blk + (q + 1) * D_CHUNK);
    fence_sched();
    dg_pass1_steps<K, 0>(q, cc, D, c1, c2, q < 4 ? klo : khi, p1, p2);
    fence_sched();
  }
}

// one fused season of the gapped walk: pass 2 of season sg (masked if it has a gap) + pass 1
// of season sg + 1 (recurrence if IT has a gap); returns whether the next scan is general
template <int K>
__device__ __forceinline__ void dg_season(bool m2, bool r1, const float* blk, v2f* D, v2f c1, v2f c2, v2f g1a, cfp W,
                                          v2f& x1, v2f& x2, v2f& sse, v2f& p1, v2f& p2, cfp tb, Mat2* Bp,
                                          bool chk, const unsigned* ubp, int* alive, unsigned k2lo, unsigned k2hi,
                                          unsigned k1lo, unsigned k1hi) {
  // two variants, not four: a third or fourth copy of the 45-step walk spilled into the hot
  // blocks (-Rpass-analysis); a season that needs only one of the two masks runs the other
  // with every keep bit set (exact, a few ops per step dearer)
  if (!m2 && !r1)
    d_pass2<K, true, false, false>(blk, D, c1, c2, g1a, W, x1, x2, sse, p1, p2, tb, Bp, chk, ubp, alive);
  else
    d_pass2<K, true, true, true>(blk, D, c1, c2, g1a, W, x1, x2, sse, p1, p2, tb, nullptr, chk, ubp, alive, nullptr,
                                 nullptr, k2lo, k2hi, k1lo, k1hi);
}

template <int K, bool PRUNE>
__device__ __forceinline__ void hw_dg_block(const SmoothArgs& a, int hmax, int n0, int hints, int* gflags) {
  constexpr int SEA = DLay<K>::SEASON;
  constexpr int TS = PairTab<K>::SIZE;
  constexpr int NMW = (32 * K + 31) / 32;
  // thread / lane ids re-derived through an opaque asm per pair: the queue loop of
  // hw_dg_kernel then holds no lane-derived addresses across pairs (they spilled)
  int tid = threadIdx.x, lane = lane_id();
  asm volatile("" : "+v"(tid), "+v"(lane));
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = lane >> 5, j = lane & 31;
  const bool odd_row = ((lane >> 4) & 1) != 0;
  const int nseg = a.Tp / a.seg, m = a.m, ns1 = nseg - 1;
  const int npairs = (a.G + 1) / 2;

  // ---- LDS: the hw_d_block layout, then mbits[2][ns1][32][2] | segm[2][ns1] | nvc[2]
  float* dl = (float*)fm_hw_smem;
  unsigned* vmask = (unsigned*)(dl + (size_t)2 * ns1 * SEA);
  float* stat = (float*)(vmask + 2 * NMW);
  int* flag = (int*)(stat + 8 * D_WAVES);
  float* ylast = (float*)(flag + 4);
  float* bests = ylast + 2 * HALF_HB;
  float* wbest = bests + 4 * 2 * HALF_HB;
  unsigned* ubound = (unsigned*)(wbest + 4 * 2 * 4);
  unsigned* mbits = ubound + 4;
  int* segm = (int*)(mbits + 2 * ns1 * 64);
  float* nvc = (float*)(segm + 2 * ns1);

  for (int i = tid; i < 2 * NMW + 8 * D_WAVES + 4; i += blockDim.x) vmask[i] = 0u;
  for (int i = tid; i < 2 * ns1 * 64 + 2 * ns1 + 2; i += blockDim.x) mbits[i] = 0u;  // mbits, segm, nvc = 0.f
  if (tid < 3) ubound[tid] = tid < 2 ? 0x7f800000u : 0u;
  if (tid == 3) {
    unsigned hp[2] = {0xffffu, 0xffffu};
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int b = (hints && n0 + r < a.N) ? a.best[n0 + r] : -1;
      const int q = (b >= 0 && b < a.G) ? b / 2 : -1;
      if (q >= 0 && q < npairs && (r == 0 || (unsigned)q != hp[0])) hp[r] = (unsigned)q;
    }
    ubound[3] = hp[0] | (hp[1] << 16);
  }
  const int head = a.head_dev ? *a.head_dev : a.head;
  __syncthreads();

  // ---- stage (as hw_d_block: aligned rings in 16-byte season chunks, else per element) -----
  {
    constexpr int GRP = 8;
    const int R = a.ring_len;
    const bool al = (R % GRP == 0) && (m % GRP == 0) && (a.ld % GRP == 0) &&
                    ((((unsigned long long)a.hist) & 15ull) == 0);
    const int phi = al ? (((a.pad - head) % GRP) + GRP) % GRP : 0;
    const int ostart = phi ? phi - GRP : 0;
    const int ngrp = (m - ostart + GRP - 1) / GRP;
    float s0 = 0.f, c0 = 0.f, s1 = 0.f, c1 = 0.f, s0b = 0.f, c0b = 0.f, s1b = 0.f, c1b = 0.f;
    float nv0 = 0.f, nv1 = 0.f;
    for (int g = tid; g < 2 * ngrp; g += blockDim.x) {
      const int r = g >= ngrp ? 1 : 0, o0 = ostart + (g - r * ngrp) * GRP;
      const int n = n0 + r;
      const bool real = n < a.N;
      const bf16_t* row = (const bf16_t*)a.hist + (long long)(real ? n : 0) * a.ld;
      float y[D_MAXSEG][GRP];
      if (al) {
#pragma unroll
        for (int k = 0; k < D_MAXSEG; ++k) {
          const int t0 = k * m + o0 - a.pad;
          int c = (head + t0) % R;
          c += c < 0 ? R : 0;
          uint4 wv = make_uint4(0u, 0u, 0u, 0u);
          if (k < nseg) wv = *(const uint4*)(row + c);
          const unsigned ww[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
          for (int u = 0; u < GRP; ++u) {
            const unsigned x = ww[u >> 1];
            const float v = __uint_as_float((u & 1) ? (x & 0xffff0000u) : (x << 16));
            const bool ok = real && k < nseg;
            y[k][u] = ok ? (t0 + u >= 0 ? v : fm_nan()) : 0.f;
          }
        }
      } else {
#pragma unroll
        for (int k = 0; k < D_MAXSEG; ++k) {
#pragma unroll
          for (int u = 0; u < GRP; ++u) {
            const bool ok = real && k < nseg && o0 + u < m;
            const int t = k * m + o0 + u - a.pad;
            const bool pos = t >= 0;
            int c = head + ((ok && pos) ? t : 0);
            c -= (c >= R) ? R : 0;
            const float v = bf16_to_f32(row[c]);
            y[k][u] = ok ? (pos ? v : fm_nan()) : 0.f;
          }
        }
      }
      const int ob = o0 > 0 ? o0 : 0;
      const int jjb = ob / K, ib = ob - jjb * K;
      unsigned vlo = 0u, vhi = 0u;
#pragma unroll
      for (int u = 0; u < GRP; ++u) {
        const int o = o0 + u;
        if (o >= 0 && o < m) {
          int i = ib + (o - ob), jj = jjb;
          if (i >= K) { i -= K; ++jj; }
          const bool v0 = y[0][u] == y[0][u];
          const bool v1 = y[1][u] == y[1][u];
          // seasons >= 1: a missing y is flagged and imputed as 0 (y*), see above
#pragma unroll
          for (int k = 1; k < D_MAXSEG; ++k) {
            if (k < nseg) {
              if (y[k][u] != y[k][u]) {
                y[k][u] = 0.f;
                atomicOr(&mbits[((r * ns1 + (k - 1)) * 32 + jj) * 2 + (i >> 5)], 1u << (i & 31));
                segm[r * ns1 + (k - 1)] = 1;
              } else {
                if (r == 0) nv0 += 1.f; else nv1 += 1.f;
              }
            }
          }
          float* blk = dl + (size_t)r * ns1 * SEA + dl_off(i, jj);
          blk[0] = v0 ? y[1][u] - y[0][u] : y[1][u];  // D^(1) = y1* - s0; + l0 for valid y0 below
          if (v0) {
            if ((o >> 5) == ((o0 < 0 ? 0 : o0) >> 5)) vlo |= 1u << (o & 31);
            else vhi |= 1u << (o & 31);
          }
#pragma unroll
          for (int k = 1; k < D_MAXSEG - 1; ++k)
            if (k < ns1) blk[(size_t)k * SEA] = y[k + 1][u] - y[k][u];
          if (o < HALF_HB) {
            float yl = y[1][u];
#pragma unroll
            for (int k = 2; k < D_MAXSEG; ++k)
              if (k == ns1) yl = y[k][u];
            ylast[r * HALF_HB + o] = yl;
          }
          // season-1 mean: observed points only (the imputed 0s are not data)
          const float y0v = v0 ? y[0][u] : 0.f, y0c = v0 ? 1.f : 0.f;
          const float y1v = v1 ? y[1][u] : 0.f, y1c = v1 ? 1.f : 0.f;
          if (r == 0) { s0 += y0v; c0 += y0c; s1 += y1v; c1 += y1c; }
          else { s0b += y0v; c0b += y0c; s1b += y1v; c1b += y1c; }
        }
      }
      const int wlo = (o0 < 0 ? 0 : o0) >> 5;
      if (vlo) atomicOr(&vmask[r * NMW + wlo], vlo);
      if (vhi) atomicOr(&vmask[r * NMW + wlo + 1], vhi);
    }
    s0 = wave_sum(s0); c0 = wave_sum(c0); s1 = wave_sum(s1); c1 = wave_sum(c1);
    s0b = wave_sum(s0b); c0b = wave_sum(c0b); s1b = wave_sum(s1b); c1b = wave_sum(c1b);
    nv0 = wave_sum(nv0); nv1 = wave_sum(nv1);
    if (lane == 0) {
      float* sw = stat + 8 * w;
      sw[0] = s0; sw[1] = c0; sw[2] = s1; sw[3] = c1;
      sw[4] = s0b; sw[5] = c0b; sw[6] = s1b; sw[7] = c1b;
      atomicAdd(&nvc[0], nv0);  // integer-valued: exact in any order
      atomicAdd(&nvc[1], nv1);
    }
  }
  __syncthreads();
  float l0r[2], b0r[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    float st[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int v = 0; v < D_WAVES; ++v)
#pragma unroll
      for (int u = 0; u < 4; ++u) st[u] += stat[8 * v + 4 * r + u];
    l0r[r] = st[1] > 0.f ? st[0] / st[1] : 0.f;
    b0r[r] = ((st[3] > 0.f ? st[2] / st[3] : 0.f) - l0r[r]) / (float)m;
  }
  for (int col = tid; col < 2 * m; col += blockDim.x) {
    const int r = col >= m ? 1 : 0, o = col - r * m;
    if ((vmask[r * NMW + (o >> 5)] >> (o & 31)) & 1u) {
      const int jj = o / K, i = o - jj * K;
      dl[(size_t)r * ns1 * SEA + dl_off(i, jj)] += l0r[r];
    }
  }
  // gapped seasons of the pair (either series): bit sg for season sg (1 .. ns1)
  int segbits = 0;
  for (int k = 0; k < ns1; ++k) segbits |= (segm[k] | segm[ns1 + k]) ? (2 << k) : 0;
  segbits = __builtin_amdgcn_readfirstlane(segbits);
  if (segbits == 0 && tid == 0) gflags[n0 >> 1] = 0;  // gap-free now: hw_d_kernel stages it next time
  __syncthreads();

  const float l0 = half ? l0r[1] : l0r[0], b0 = half ? b0r[1] : b0r[0];
  const float* mydl = dl + (size_t)half * ns1 * SEA + j * 4;
  const unsigned* mymb = mbits + ((size_t)half * ns1 * 32 + j) * 2;  // + (sg - 1) * 64
  const int last_addr = ((lane & 32) | 31) << 2;
  float bestSSE = __builtin_huge_valf();
  int bestIdx = 0x7fffffff;
  float bestL = l0, bestB = b0;
  float* mybest = bests + (w * 2 + half) * HALF_HB;
  const int nwaves = blockDim.x / FM_WAVE;
  const float* powbase = a.pair_tab + (size_t)npairs * TS;  // [npairs][K + 1][8]: A^0 .. A^K
  const unsigned hints_pp = (unsigned)__builtin_amdgcn_readfirstlane((int)ubound[3]);
  for (int k = w; k < npairs;) {
    const int pi = hint_pair_at(k, 0, hints_pp);
    const int c0 = 2 * pi;
    const int c1i = (2 * pi + 1 < a.G) ? 2 * pi + 1 : c0;
    const cfp tab = const_ptr(a.pair_tab + (size_t)pi * TS);
    const v2f c1 = ldv2(tab), c2 = ldv2(tab + 2), g1a = ldv2(tab + 4);
    const cfp W = tab + PairTab<K>::W0;
    const cfp tb = tab + PairTab<K>::B0;
    const float* pw = powbase + (size_t)pi * (K + 1) * 8;
    const v2f one = splat2(1.f), zero = splat2(0.f);
    Mat2 Bj;
    Mat2 Bp[4];
    Bj.a = one; Bj.b = zero; Bj.c = zero; Bj.d = one;
#pragma unroll
    for (int bit = 0; bit < 4; ++bit) Bp[bit] = ldmat(tb + 8 * bit);
    fence_sched();
#pragma unroll
    for (int bit = 0; bit < 4; ++bit) {
      const Mat2 r = matmul(Bj, Bp[bit]);
      if ((lane >> bit) & 1) Bj = r;
    }
    v2f D[K];
    v2f X1 = splat2(l0 + b0), X2 = splat2(b0), sse = zero;
    v2f p1, p2;
    Aff<v2f> loc;
    bool general = (segbits & 2) != 0;
    if (general) {
      const unsigned mlo = mymb[0], mhi = mymb[1];
      dg_pass1_rec<K>(mydl, D, c1, c2, ~mlo, ~mhi, p1, p2);
      const Mat2 M = lane_map<K>(pw, mlo, mhi);
      loc.m11 = M.a; loc.m12 = M.b; loc.m21 = M.c; loc.m22 = M.d; loc.v1 = p1; loc.v2 = p2;
    } else {
      d_pass1<K>(mydl, W, D, p1, p2);
    }
    int alive = 1;
    for (int sg = 1; sg < ns1; ++sg) {
      v2f x1, x2;
      if (general) {
        half_exclusive_scan(loc, j);
        x1 = loc.m11 * X1 + loc.m12 * X2 + loc.v1;
        x2 = loc.m21 * X1 + loc.m22 * X2 + loc.v2;
      } else {
        half_uniform_scan_pre(Bp, launder(tb), p1, p2, X1, X2, Bj, odd_row, x1, x2);
      }
      const bool m2 = (segbits >> sg) & 1, r1 = (segbits >> (sg + 1)) & 1;
      const unsigned* mb2 = mymb + (size_t)(sg - 1) * 64;
      const unsigned* mb1 = mb2 + 64;
      const unsigned n2lo = mb2[0], n2hi = mb2[1], n1lo = mb1[0], n1hi = mb1[1];
      dg_season<K>(m2, r1, mydl + (size_t)sg * SEA, D, c1, c2, g1a, launder(W), x1, x2, sse, p1, p2, tb, Bp,
                   PRUNE, ubound + half, &alive, ~n2lo, ~n2hi, ~n1lo, ~n1hi);
      // the gapped variant ran pass 1 as the recurrence (whichever of its masks it needed):
      // the next scan takes the general lane maps
      general = m2 || r1;
      if (general) {
        const Mat2 M = lane_map<K>(pw, n1lo, n1hi);
        loc.m11 = M.a; loc.m12 = M.b; loc.m21 = M.c; loc.m22 = M.d; loc.v1 = p1; loc.v2 = p2;
      }
      X1 = half_last_bp(x1, last_addr);
      X2 = half_last_bp(x2, last_addr);
      if (PRUNE && !__any(alive)) break;
    }
    if (!PRUNE || __any(alive)) {
      v2f x1, x2, d1, d2;
      if (general) {
        half_exclusive_scan(loc, j);
        x1 = loc.m11 * X1 + loc.m12 * X2 + loc.v1;
        x2 = loc.m21 * X1 + loc.m22 * X2 + loc.v2;
      } else {
        half_uniform_scan_pre(Bp, tb, p1, p2, X1, X2, Bj, odd_row, x1, x2);
      }
      if ((segbits >> ns1) & 1) {
        const unsigned* mb2 = mymb + (size_t)(ns1 - 1) * 64;
        d_pass2<K, false, true, false>(mydl, D, c1, c2, g1a, W, x1, x2, sse, d1, d2, nullptr, nullptr, false,
                                       nullptr, nullptr, nullptr, nullptr, ~mb2[0], ~mb2[1]);
      } else {
        d_pass2<K, false>(mydl, D, c1, c2, g1a, W, x1, x2, sse, d1, d2);
      }
      X1 = half_last_bp(x1, last_addr);
      X2 = half_last_bp(x2, last_addr);
      sse = half_sum_last(sse);
      sse = half_last_bp(sse, last_addr);
      const bool upd0 = (sse.x < bestSSE || (sse.x == bestSSE && c0 < bestIdx));
      if (upd0) { bestSSE = sse.x; bestIdx = c0; bestL = X1.x - X2.x; bestB = X2.x; }
      const bool upd1 = (c1i != c0) && (sse.y < bestSSE || (sse.y == bestSSE && c1i < bestIdx));
      if (upd1) { bestSSE = sse.y; bestIdx = c1i; bestL = X1.y - X2.y; bestB = X2.y; }
      // the forecast's seasonal phases 0 .. hmax - 1 from the lanes that own them: lane 0 alone
      // while hmax <= K; at K = 9 (the gapped pairs of the 300 s step's quad path, which takes
      // horizons up to 16) phases 9 .. 15 are lane 1's
      if ((upd0 || upd1) && j * K < hmax) {
        const float* yl = ylast + half * HALF_HB;
#pragma unroll
        for (int i = 0; i < K && i < HALF_HB; ++i) {
          const int ph = j * K + i;
          if (ph < hmax && ph < HALF_HB) mybest[ph] = yl[ph] - (upd1 ? D[i].y : D[i].x);
        }
      }
      if (PRUNE && j == 0 && (upd0 || upd1))
        __hip_atomic_fetch_min(ubound + half, __float_as_uint(bestSSE), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    int q = 0;
    if (lane == 0)
      q = __hip_atomic_fetch_add(ubound + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    k = nwaves + __builtin_amdgcn_readfirstlane(q);
  }

  // ---- arg-min across the 4 waves; wave r finishes series n0 + r ----------------------
  if (j == 0) {
    float* wb = wbest + (w * 2 + half) * 4;
    wb[0] = bestSSE;
    wb[1] = __int_as_float(bestIdx);
    wb[2] = bestL;
    wb[3] = bestB;
  }
  __syncthreads();
  if (w >= 2) return;
  const int r = w, n = n0 + r;
  if (n >= a.N) return;
  int win = 0;
  for (int q = 1; q < nwaves; ++q) {
    const float sq = wbest[(q * 2 + r) * 4], sw = wbest[(win * 2 + r) * 4];
    const int iq = __float_as_int(wbest[(q * 2 + r) * 4 + 1]), iw = __float_as_int(wbest[(win * 2 + r) * 4 + 1]);
    if (sq < sw || (sq == sw && iq < iw)) win = q;
  }
  const float* wb = wbest + (win * 2 + r) * 4;
  const float gSSE = wb[0], gL = wb[2], gB = wb[3];
  const int gIdx = __float_as_int(wb[1]);
  const float* sb = bests + (win * 2 + r) * HALF_HB;
  const float nvr = nvc[r];
  const float sig = sqrtf(gSSE / fmaxf(nvr, 1.f));
  if (lane == 0) {
    a.level[n] = gL;
    a.trend[n] = gB;
    a.sigma[n] = sig;
    a.best[n] = gIdx;
  }
  const int Tp = a.Tp;
  if (a.season_hb && lane < hmax) a.season_hb[(long long)n * HALF_HB + lane] = sb[lane];
  if (a.nvalid_out && lane == 0) a.nvalid_out[n] = nvr;
  detect_epilogue_wave(a.det, n, sig, nvr, [&](int h) {
    int ph = (Tp - 1 + h) % m;
    if (ph < 0) ph += m;
    ph = ph < HALF_HB ? ph : HALF_HB - 1;
    return gL + (float)h * gB + sb[ph];
  }, gIdx);
}

// Persistent over the pairs hw_d_kernel deferred (count in deferred[0]); self-cleaning like
// hw_half_general_kernel: workspace int32 [4 + 2 ceil(N / 2)] = {count, pairs..., done, total,
// queue, per-pair gap flags...}; the last workgroup out adds the count to `total` (deferred
// pairs since allocation, for the records) and resets count, done and the queue.  A pair's
// flag is set by hw_d_kernel when it defers the pair and cleared here when the pair is found
// gap-free; hw_d_kernel hands flagged pairs over without staging them.
template <int K, bool PRUNE>
__global__ __launch_bounds__(256, 2) void hw_dg_kernel(const SmoothArgs a, int hmax, int* deferred, int hints) {
  const int cnt = min(deferred[0], (a.N + 1) / 2);
  if (cnt == 0) return;  // gap-free shard: count and done are already 0
  int* done = deferred + 1 + (a.N + 1) / 2;  // {done, total, queue}
  __shared__ int next;
  // pairs from a queue, not a static stride: their cost varies (gapped seasons, pruning)
  for (;;) {
    if (threadIdx.x == 0) next = atomicAdd(done + 2, 1);
    __syncthreads();
    const int q = next;
    __syncthreads();  // every thread has read `next` before thread 0 overwrites it
    if (q >= cnt) break;
    // the arguments through a pointer re-derived per pair (opaque to LLVM): values computed
    // from them inside the block are not hoisted out of the queue loop (held across it, they
    // spilled)
    const __attribute__((address_space(4))) SmoothArgs* ap =
        (const __attribute__((address_space(4))) SmoothArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    int hm = hmax, hi = hints;
    asm volatile("" : "+s"(ap), "+s"(hm), "+s"(hi));
    hw_dg_block<K, PRUNE>(*(const SmoothArgs*)ap, hm, deferred[1 + q], hi, done + 3);
    __syncthreads();  // LDS is reused by the next pair
  }
  if (threadIdx.x == 0) {
    if (atomicAdd(done, 1) == (int)gridDim.x - 1) {  // the last workgroup out resets the workspace
      done[1] += cnt;
      done[2] = 0;
      *done = 0;
      deferred[0] = 0;
    }
  }
}

extern "C" size_t fm_hw_dg_lds_bytes(int Tp, int seg, int K);

// A/B instrument (FOREMAST_HW_DG_ALL=1): every pair is listed for the gapped kernel, so its
// cost on gap-free seasons can be timed against hw_d_kernel's on the same data
__global__ void hw_dg_list_all_kernel(int* deferred, int pairs) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < pairs; q += gridDim.x * blockDim.x) deferred[1 + q] = 2 * q;
  if (blockIdx.x == 0 && threadIdx.x == 0) deferred[0] = pairs;
}

// the seasons variant 5 is instantiated for: m = 32 K, K steps per lane
// (1440 = 32 x 45: the 60 s step; 288 = 32 x 9: the 300 s step)
static bool d_supported_k(int K) { return K == 45 || K == 9; }

extern "C" size_t fm_hw_d_lds_bytes(int Tp, int seg, int K) {
  if (!d_supported_k(K) || seg <= 0) return (size_t)-1;
  const int nseg = Tp / seg;
  if (nseg < 2 || nseg > D_MAXSEG) return (size_t)-1;
  const int NMW = (32 * K + 31) / 32;
  const int season = D_CHUNK * ((K + 7) / 8);  // DLay<K>::SEASON
  return ((size_t)2 * (nseg - 1) * season + 2 * NMW + 8 * D_WAVES + 4 + 2 * HALF_HB + 4 * 2 * HALF_HB + 4 * 2 * 4 +
          4) * 4;
}

// hw_dg_block: the hw_d_block layout + per-(series, season, lane) 64-bit miss masks, per
// (series, season) gap flags and the two valid-point counts
// hw_q_kernel: seasons m = 16 K (K = 18: the 300 s step)
static bool q_supported_k(int K) { return K == 18; }

extern "C" size_t fm_hw_q_lds_bytes(int Tp, int seg, int K) {
  if (!q_supported_k(K) || seg != 16 * K) return (size_t)-1;
  const int nseg = Tp / seg;
  if (nseg < 2 || nseg > D_MAXSEG) return (size_t)-1;
  const int NMW = (16 * K + 31) / 32;
  const int season = D_CHUNK * ((K + 7) / 8);
  return ((size_t)Q_S * (nseg - 1) * season + Q_S * NMW + 4 * Q_S * D_WAVES + 4 + Q_S * HALF_HB +
          4 * Q_S * HALF_HB + 4 * Q_S * 4 + 8) * 4;
}

// Variant 5 at m = 16 K: hw_q_kernel over quads, then the gapped kernel at K / 2 (32 lanes x
// K / 2 steps) over the pairs it deferred, with `tab_g` = pair_table(grid, K / 2) (the
// 32-lane kernel's weights and powers).  Same workspace and contract as fm_hw_d_fit.
extern "C" int fm_hw_q_fit(const SmoothArgs* a, const float* tab_g, int hmax, int* deferred, hipStream_t st) {
  const int K = a->K;
  if (!q_supported_k(K) || a->seg != 16 * K || a->m != a->seg || a->Tp % a->seg != 0 || a->Tp / a->seg < 2 ||
      a->Tp / a->seg > D_MAXSEG || !a->pair_tab || !tab_g || a->season_out || hmax < 1 || hmax > K ||
      hmax > HALF_HB)
    return (int)hipErrorNotSupported;
  if (a->N <= 0) return 0;
  const size_t lds = fm_hw_q_lds_bytes(a->Tp, a->seg, K);
  const size_t dlds = fm_hw_dg_lds_bytes(a->Tp, a->seg, K / 2);
  if (lds > 80 * 1024 || dlds > 80 * 1024) return (int)hipErrorNotSupported;
  if (!deferred) return (int)hipErrorInvalidValue;
  const char* pe = getenv("FOREMAST_HW_PRUNE");
  const bool prune = !(pe && pe[0] == '0');
  const char* he = getenv("FOREMAST_HW_HINTS");
  const int hints = (prune && !(he && he[0] == '0')) ? 1 : 0;
  const int quads = (a->N + 3) / 4;
  if (prune)
    hipLaunchKernelGGL((hw_q_kernel<18, true>), dim3(quads), dim3(256), lds, st, *a, hmax, deferred, hints);
  else
    hipLaunchKernelGGL((hw_q_kernel<18, false>), dim3(quads), dim3(256), lds, st, *a, hmax, deferred, hints);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  SmoothArgs ag = *a;
  ag.pair_tab = tab_g;
  ag.K = K / 2;
  const int pairs = (a->N + 1) / 2;
  const int grid = pairs < 512 ? pairs : 512;
  if (prune)
    hipLaunchKernelGGL((hw_dg_kernel<9, true>), dim3(grid), dim3(256), dlds, st, ag, hmax, deferred, hints);
  else
    hipLaunchKernelGGL((hw_dg_kernel<9, false>), dim3(grid), dim3(256), dlds, st, ag, hmax, deferred, hints);
  return (int)hipGetLastError();
}

extern "C" size_t fm_hw_dg_lds_bytes(int Tp, int seg, int K) {
  const size_t base = fm_hw_d_lds_bytes(Tp, seg, K);
  if (base == (size_t)-1) return base;
  const int ns1 = Tp / seg - 1;
  return base + ((size_t)2 * ns1 * 64 + 2 * ns1 + 2) * 4;
}

// Deferred detection for HW variants 4/5: band, verdict, per-app counters and the K9
// anomaly list from the fitted parameters (one 16-lane row per series), with the same
// forecast as the fused epilogue: level + h * trend + season[(Tp - 1 + h) mod m].
__global__ __launch_bounds__(256) void hw_detect_params_kernel(const SmoothArgs a) {
  const int n = blockIdx.x * (blockDim.x / 16) + (threadIdx.x >> 4);
  if (n >= a.N) return;  // row-uniform
  const float gL = a.level[n], gB = a.trend[n], sig = a.sigma[n], nvr = a.nvalid_out[n];
  const float* sb = a.season_hb + (long long)n * HALF_HB;
  const int Tp = a.Tp, m = a.m;
  detect_epilogue_row(a.det, n, sig, nvr, [&](int h) {
    int ph = (Tp - 1 + h) % m;
    if (ph < 0) ph += m;
    ph = ph < HALF_HB ? ph : HALF_HB - 1;
    return gL + (float)h * gB + sb[ph];
  }, a.best ? a.best[n] : -1);
}

extern "C" int fm_hw_detect_params(const SmoothArgs* a, hipStream_t st) {
  if (a->N <= 0 || a->det.C <= 0) return 0;
  if (!a->season_hb || !a->nvalid_out || !a->level || !a->trend || !a->sigma || a->m <= 0)
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(hw_detect_params_kernel, dim3((a->N + 15) / 16), dim3(256), 0, st, *a);
  return (int)hipGetLastError();
}

extern "C" size_t fm_hw_half_lds_bytes(int Tp, int seg, int K) {
  if (K != 45) return (size_t)-1;
  constexpr int KP = 48;
  const int nseg = Tp / seg;
  size_t off = ((size_t)2 * nseg * 32 * KP * 2 + 15) & ~(size_t)15;
  off += ((size_t)(2 * nseg + 2) * 4 + 15) & ~(size_t)15;
  off += (size_t)4 * 2 * HALF_HB * 4;
  off += (size_t)4 * 2 * 4 * 4;
  return off;
}

// Variant 4 launcher: Holt-Winters, bf16 ring, season = seg = 32 K, pair table given,
// forecast horizons within 1..hmax (hmax <= min(K, HALF_HB)), no season_out.
// `deferred`: device int32 workspace of 2 + ceil(N / 2) entries, zero on entry (kept zero
// between launches by the general kernel).
extern "C" int fm_hw_half_fit(const SmoothArgs* a, int hmax, int* deferred, hipStream_t st) {
  const int K = a->K;
  if (K != 45 || a->seg != 32 * K || a->m != a->seg || a->Tp % a->seg != 0 || a->Tp / a->seg < 2 ||
      !a->pair_tab || a->season_out || hmax < 1 || hmax > K || hmax > HALF_HB)
    return (int)hipErrorNotSupported;
  if (a->N <= 0) return 0;
  const size_t lds = fm_hw_half_lds_bytes(a->Tp, a->seg, K);
  if (lds > 64 * 1024) return (int)hipErrorNotSupported;
  if (!deferred) return (int)hipErrorInvalidValue;
  const int pairs = (a->N + 1) / 2;
  hipLaunchKernelGGL((hw_half_kernel<45>), dim3(pairs), dim3(256), lds, st, *a, hmax, deferred);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL((hw_half_general_kernel<45>), dim3(pairs < 512 ? pairs : 512), dim3(256), lds, st, *a, hmax,
                     deferred);
  return (int)hipGetLastError();
}

// Split-tail plan: with P series pairs and `slots` resident workgroups, whole pairs run in
// ceil(P / slots) rounds and the last one can be nearly empty (12.5k series per GPU:
// 6250 pairs on 512 slots = 12.2 rounds).  Splitting the grid of the last S pairs in two
// halves (each a workgroup, merged by the second arriver) evens the tail; S is the
// candidate with the smallest modelled makespan (a half costs ~half a pair plus its
// staging).  Returns S (0 = no split).
extern "C" int fm_hw_d_split_plan(int pairs, int slots, int max_split) {
  if (pairs <= 0 || slots <= 0) return 0;
  auto cost = [&](int S) {
    const int full = pairs - S;
    return 2.0 * ((full + slots - 1) / slots) + 1.1 * ((2 * S + slots - 1) / slots);
  };
  int best = 0;
  double bc = cost(0);
  const int cands[3] = {pairs % slots, pairs % slots + slots, pairs};
  for (int S : cands) {
    if (S <= 0 || S > pairs || S > max_split) continue;
    const double c = cost(S);
    if (c < bc - 1e-9) { bc = c; best = S; }
  }
  return best;
}

// Variant 5 launcher: same contract as fm_hw_half_fit (deferred pairs go to the
// variant-4 general kernel), at most D_MAXSEG seasons.  `split_ws` (optional):
// int32 [2 * max_split] arrival counters followed by float [max_split * 2 * 2 *
// CAND_FLOATS] candidates; the counters must be zero on entry (they are left zero).
extern "C" int fm_hw_d_fit_split(const SmoothArgs* a, int hmax, int* deferred, int* split_ws, int max_split,
                                 int slots, hipStream_t st);
extern "C" int fm_hw_d_fit(const SmoothArgs* a, int hmax, int* deferred, hipStream_t st) {
  return fm_hw_d_fit_split(a, hmax, deferred, nullptr, 0, 0, st);
}

template <int K>
static hipError_t launch_d_fit(const SmoothArgs* a, int hmax, int* deferred, int* split_ws, int max_split, int slots,
                               hipStream_t st);

extern "C" int fm_hw_d_fit_split(const SmoothArgs* a, int hmax, int* deferred, int* split_ws, int max_split,
                                 int slots, hipStream_t st) {
  const int K = a->K;
  if (!d_supported_k(K) || a->seg != 32 * K || a->m != a->seg || a->Tp % a->seg != 0 || a->Tp / a->seg < 2 ||
      a->Tp / a->seg > D_MAXSEG || !a->pair_tab || a->season_out || hmax < 1 || hmax > K || hmax > HALF_HB)
    return (int)hipErrorNotSupported;
  if (a->N <= 0) return 0;
  if (fm_hw_d_lds_bytes(a->Tp, a->seg, K) > 80 * 1024 || fm_hw_dg_lds_bytes(a->Tp, a->seg, K) > 80 * 1024)
    return (int)hipErrorNotSupported;
  if (!deferred) return (int)hipErrorInvalidValue;
  return (int)(K == 45 ? launch_d_fit<45>(a, hmax, deferred, split_ws, max_split, slots, st)
                       : launch_d_fit<9>(a, hmax, deferred, split_ws, max_split, slots, st));
}

template <int K>
static hipError_t launch_d_fit(const SmoothArgs* a, int hmax, int* deferred, int* split_ws, int max_split, int slots,
                               hipStream_t st) {
  const size_t lds = fm_hw_d_lds_bytes(a->Tp, a->seg, K);
  const int pairs = (a->N + 1) / 2;
  const int S = (split_ws && max_split > 0 && a->G >= 2) ? fm_hw_d_split_plan(pairs, slots, max_split) : 0;
  // arrival counters are zero between launches: allocated zeroed, and the second arriver
  // of each (slot, row) resets its counter
  int* cnt = split_ws;
  float* cand = split_ws ? (float*)(split_ws + 2 * max_split) : nullptr;
  // FOREMAST_HW_PRUNE=0 turns the exact grid branch and bound off (A/B runs)
  const char* pe = getenv("FOREMAST_HW_PRUNE");
  const bool prune = !(pe && pe[0] == '0');
  const char* he = getenv("FOREMAST_HW_HINTS");  // previous winners first (=0: grid order)
  const int hints = (prune && !(he && he[0] == '0')) ? 1 : 0;
  const char* da = getenv("FOREMAST_HW_DG_ALL");
  if (da && da[0] == '1')
    hipLaunchKernelGGL(hw_dg_list_all_kernel, dim3((pairs + 255) / 256), dim3(256), 0, st, deferred, pairs);
  else if (prune)
    hipLaunchKernelGGL((hw_d_kernel<K, true>), dim3(pairs - S + 2 * S), dim3(256), lds, st, *a, hmax, deferred,
                       pairs - S, cnt, cand, hints);
  else
    hipLaunchKernelGGL((hw_d_kernel<K, false>), dim3(pairs - S + 2 * S), dim3(256), lds, st, *a, hmax, deferred,
                       pairs - S, cnt, cand, hints);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // gapped pairs: the variant-5 walk with masked seasons (FOREMAST_HW_GAPS=v4: the variant-4
  // general kernel instead, for A/B runs; daily season at 60 s only)
  const char* ge = getenv("FOREMAST_HW_GAPS");
  if (K == 45 && ge && ge[0] == 'v') {
    const size_t glds = fm_hw_half_lds_bytes(a->Tp, a->seg, K);
    if (glds > 64 * 1024) return hipErrorNotSupported;
    hipLaunchKernelGGL((hw_half_general_kernel<45>), dim3(pairs < 512 ? pairs : 512), dim3(256), glds, st, *a, hmax,
                       deferred);
    return hipGetLastError();
  }
  const size_t dlds = fm_hw_dg_lds_bytes(a->Tp, a->seg, K);
  int grid = pairs < 512 ? pairs : 512;
  const char* gg = getenv("FOREMAST_HW_DG_GRID");  // A/B: workgroups of the gapped kernel
  if (gg && atoi(gg) > 0) grid = atoi(gg) < pairs ? atoi(gg) : pairs;
  if (prune)
    hipLaunchKernelGGL((hw_dg_kernel<K, true>), dim3(grid), dim3(256), dlds, st, *a, hmax, deferred, hints);
  else
    hipLaunchKernelGGL((hw_dg_kernel<K, false>), dim3(grid), dim3(256), dlds, st, *a, hmax, deferred, hints);
  return hipGetLastError();
}

template <int K, int MODE, typename TIN, int NC, int MINW, bool TAB = false>
__global__ __launch_bounds__(256, MINW) void hw_scan_kernel(const SmoothArgs a) {
  static_assert(!TAB || NC == 2, "table path is packed-pair only");
  using V = typename std::conditional<NC == 2, v2f, float>::type;
  using YR = YRegs<TIN, K>;
  constexpr int KP = YR::KP;
  const int n = blockIdx.x;
  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  const int nwaves = blockDim.x / FM_WAVE;
  const int seg = a.seg;
  const int L = seg / K;  // active lanes
  const int nseg = a.Tp / seg;

  // ---- LDS carve: ys[nseg][64][KP] | bests[nwaves][64][KP] f32 | segnan | red | wbest ----
  size_t off = 0;
  TIN* ys = (TIN*)(fm_hw_smem + off);
  off += ((size_t)nseg * 64 * KP * sizeof(TIN) + 15) & ~(size_t)15;
  float* bests = (float*)(fm_hw_smem + off);
  if (MODE == MODE_HW) off += (size_t)nwaves * 64 * KP * 4;
  int* segnan = (int*)(fm_hw_smem + off);
  off += ((size_t)nseg * 4 + 15) & ~(size_t)15;
  float* red = (float*)(fm_hw_smem + off);
  off += 64 * 4;
  float* wbest = (float*)(fm_hw_smem + off);

  for (int i = tid; i < nseg; i += blockDim.x) segnan[i] = 0;
  __syncthreads();

  // ---- stage: logical padded index p = sg*seg + j*K + i → ys[sg][j][i] ----------------
  const TIN* row = (const TIN*)a.hist + (long long)n * a.ld;
  const int t0 = (MODE == MODE_HW) ? a.m : 0;
  float nv_local = 0.f;
  const int total = nseg * 64 * KP;
  for (int idx = tid; idx < total; idx += blockDim.x) {
    const int i = idx % KP;
    const int j = (idx / KP) & 63;
    const int sg = idx / (KP * 64);
    float v = fm_nan();
    if (i < K && j < L) {
      const int p = sg * seg + j * K + i;
      const int t = p - a.pad;
      if (t >= 0) {
        int c = a.head + t;
        if (c >= a.ring_len) c -= a.ring_len;
        v = to_f32<TIN>(row[c]);
      }
      const bool isn = (v != v);
      if (isn) atomicOr(&segnan[sg], 1);
      if (!isn && p >= t0) nv_local += 1.f;
    }
    ys[idx] = from_f32<TIN>(v);
  }
  const float n_valid = blk_sum(nv_local, red);

  // ---- initial state ----------------------------------------------------------------
  float l0 = 0.f, b0 = 0.f;
  if (MODE == MODE_HW) {
    float s0 = 0.f, c0 = 0.f, s1 = 0.f, c1 = 0.f;
    for (int q = tid; q < seg; q += blockDim.x) {
      const int j = q / K, i = q % K;
      const float y0 = to_f32<TIN>(ys[(0 * 64 + j) * KP + i]);
      const float y1 = to_f32<TIN>(ys[(1 * 64 + j) * KP + i]);
      if (y0 == y0) { s0 += y0; c0 += 1.f; }
      if (y1 == y1) { s1 += y1; c1 += 1.f; }
    }
    s0 = blk_sum(s0, red);
    c0 = blk_sum(c0, red);
    s1 = blk_sum(s1, red);
    c1 = blk_sum(c1, red);
    l0 = c0 > 0.f ? s0 / c0 : 0.f;
    b0 = ((c1 > 0.f ? s1 / c1 : 0.f) - l0) / (float)a.m;
  } else {
    // first valid value in logical order (segments, then lanes, then steps)
    int first = 0x7fffffff;
    for (int q = tid; q < nseg * seg; q += blockDim.x) {
      const int sg = q / seg, r = q % seg, j = r / K, i = r % K;
      const float y = to_f32<TIN>(ys[(sg * 64 + j) * KP + i]);
      if (y == y && q < first) first = q;
    }
    float f = (float)first;
    f = -blk_max(-f, red);
    const int fi = (int)f;
    if (fi < nseg * seg) {
      const int sg = fi / seg, r = fi % seg;
      l0 = to_f32<TIN>(ys[(sg * 64 + r / K) * KP + r % K]);
    }
  }

  const bool active = lane < L;
  float bestSSE = __builtin_huge_valf();
  int bestIdx = 0x7fffffff;
  float bestL = l0, bestB = b0;
  float* mybest = bests + ((size_t)w * 64 + lane) * KP;
  const int npairs = (a.G + NC - 1) / NC;
  const int sgA = (MODE == MODE_HW) ? 1 : 0;

  for (int pi = w; pi < npairs; pi += nwaves) {
    const int c0 = NC * pi;
    const int c1i = (NC == 2 && NC * pi + 1 < a.G) ? NC * pi + 1 : c0;
    V al, be, ga;
    if constexpr (NC == 2) {
      al.x = a.grid[3 * c0 + 0]; al.y = a.grid[3 * c1i + 0];
      be.x = a.grid[3 * c0 + 1]; be.y = a.grid[3 * c1i + 1];
      ga.x = a.grid[3 * c0 + 2]; ga.y = a.grid[3 * c1i + 2];
    } else {
      al = a.grid[3 * c0 + 0]; be = a.grid[3 * c0 + 1]; ga = a.grid[3 * c0 + 2];
    }
    const V one = splatv<V>(1.f), zero = splatv<V>(0.f);
    const V c2 = al * be, c1 = al + c2, g1a = ga * (one - al), omc1 = one - c1;
    const float* tab = nullptr;
    Mat2 Bj;
    if constexpr (TAB) {
      tab = a.pair_tab + (size_t)__builtin_amdgcn_readfirstlane(pi) * PairTab<K>::SIZE;
      // Bj = B^(lane & 15) by binary powering
      const float* tb = tab + PairTab<K>::B0;
      Bj.a = one; Bj.b = zero; Bj.c = zero; Bj.d = one;
#pragma unroll
      for (int bit = 0; bit < 4; ++bit) {
        const Mat2 Bb = ldmat(tb + 8 * bit);
        const Mat2 r = matmul(Bj, Bb);
        if ((lane >> bit) & 1) Bj = r;
      }
    }

    // A'^K for a full NaN-free lane chunk, A' = [[1-c1, 1], [-c2, 1]]
    Aff<V> P;
    P.m11 = one; P.m12 = zero; P.m21 = zero; P.m22 = one;
#pragma unroll
    for (int i = 0; i < K; ++i) {
      const V n11 = omc1 * P.m11 + P.m21, n12 = omc1 * P.m12 + P.m22;
      const V n21 = P.m21 - c2 * P.m11, n22 = P.m22 - c2 * P.m12;
      P.m11 = n11; P.m12 = n12; P.m21 = n21; P.m22 = n22;
    }

    // seasonal state: my phases of season 0, minus l0
    V s[K];
    {
      YR y0;
      y0.load(ys + ((size_t)0 * 64 + lane) * KP);
#pragma unroll
      for (int i = 0; i < K; ++i) {
        const float y = y0.get(i);
        s[i] = splatv<V>((MODE == MODE_HW && y == y) ? y - l0 : 0.f);
      }
    }
    V Lv = splatv<V>(l0 + b0), Bv = splatv<V>(b0), sse = zero;  // (f, b)

    // prologue: pass 1 of the first fitted segment
    YR ycur, ynext;
    ycur.load(ys + ((size_t)sgA * 64 + lane) * KP);
    Aff<V> loc;
    bool locfast = !segnan[sgA];
    if (locfast) {
      if constexpr (TAB) {
        loc.v1 = zero; loc.v2 = zero;
#pragma unroll
        for (int i = 0; i < K; ++i) {
          const V un = splatv<V>(ycur.get(i)) - s[i];
          loc.v1 = loc.v1 + ldv2(tab + PairTab<K>::W0 + 4 * i) * un;
          loc.v2 = loc.v2 + ldv2(tab + PairTab<K>::W0 + 4 * i + 2) * un;
        }
      } else {
        pass1_fast<K>(ycur, s, c1, c2, loc.v1, loc.v2);
      }
    } else {
      pass1_slow<K>(ycur, s, c1, c2, loc);
    }

    for (int sg = sgA; sg < nseg; ++sg) {
      V x1, x2;
      if (TAB && locfast) {
        if constexpr (TAB) uniform_exclusive_scan(tab + PairTab<K>::B0, loc.v1, loc.v2, Lv, Bv, Bj, lane, x1, x2);
      } else {
        if (locfast) { loc.m11 = P.m11; loc.m12 = P.m12; loc.m21 = P.m21; loc.m22 = P.m22; }
        wave_exclusive_scan(loc);
        x1 = loc.m11 * Lv + loc.m12 * Bv + loc.v1;
        x2 = loc.m21 * Lv + loc.m22 * Bv + loc.v2;
      }
      const bool has_next = sg + 1 < nseg;
      if (has_next) ynext.load(ys + ((size_t)(sg + 1) * 64 + lane) * KP);
      const bool mask = segnan[sg] != 0;
      const bool next_fast = has_next && !segnan[sg + 1];
      if (next_fast) {
        if constexpr (TAB) {
          if (mask) pass2_tab<K, MODE, true>(ycur, ynext, s, c1, c2, g1a, tab + PairTab<K>::W0, x1, x2, sse, loc.v1, loc.v2);
          else pass2_tab<K, MODE, false>(ycur, ynext, s, c1, c2, g1a, tab + PairTab<K>::W0, x1, x2, sse, loc.v1, loc.v2);
        } else {
          if (mask) pass2<K, MODE, true, true>(ycur, ynext, s, c1, c2, g1a, x1, x2, sse, loc.v1, loc.v2);
          else pass2<K, MODE, false, true>(ycur, ynext, s, c1, c2, g1a, x1, x2, sse, loc.v1, loc.v2);
        }
        locfast = true;
      } else {
        V d1, d2;
        if (mask) pass2<K, MODE, true, false>(ycur, ynext, s, c1, c2, g1a, x1, x2, sse, d1, d2);
        else pass2<K, MODE, false, false>(ycur, ynext, s, c1, c2, g1a, x1, x2, sse, d1, d2);
        if (has_next) pass1_slow<K>(ynext, s, c1, c2, loc);
        locfast = false;
      }
      Lv = rdlanev(x1, L - 1);
      Bv = rdlanev(x2, L - 1);
      ycur = ynext;
    }
    sse = active ? sse : zero;
    sse = wave_sumv(sse);
    const float s0v = compv(sse, 0), s1v = compv(sse, 1);
    bool upd0 = (s0v < bestSSE || (s0v == bestSSE && c0 < bestIdx));
    if (upd0) { bestSSE = s0v; bestIdx = c0; bestL = compv(Lv, 0) - compv(Bv, 0); bestB = compv(Bv, 0); }
    const bool upd1 = (c1i != c0) && (s1v < bestSSE || (s1v == bestSSE && c1i < bestIdx));
    if (upd1) { bestSSE = s1v; bestIdx = c1i; bestL = compv(Lv, 1) - compv(Bv, 1); bestB = compv(Bv, 1); }
    if (MODE == MODE_HW && (upd0 || upd1)) {
#pragma unroll
      for (int i = 0; i < K; ++i) mybest[i] = compv(s[i], upd1 ? 1 : 0);
    }
  }

  // ---- arg-min across waves ---------------------------------------------------------
  if (lane == 0) {
    wbest[4 * w + 0] = bestSSE;
    wbest[4 * w + 1] = __int_as_float(bestIdx);
    wbest[4 * w + 2] = bestL;
    wbest[4 * w + 3] = bestB;
  }
  __syncthreads();
  int win = 0;
  for (int i = 1; i < nwaves; ++i) {
    const float si = wbest[4 * i], sw = wbest[4 * win];
    const int ii = __float_as_int(wbest[4 * i + 1]), iw = __float_as_int(wbest[4 * win + 1]);
    if (si < sw || (si == sw && ii < iw)) win = i;
  }
  const float gSSE = wbest[4 * win];
  const int gIdx = __float_as_int(wbest[4 * win + 1]);
  const float gL = wbest[4 * win + 2], gB = wbest[4 * win + 3];
  const float sig = sqrtf(gSSE / fmaxf(n_valid, 1.f));
  if (tid == 0) {
    a.level[n] = gL;
    a.trend[n] = gB;
    a.sigma[n] = sig;
    a.best[n] = gIdx;
  }
  const float* sfin = bests + (size_t)win * 64 * KP;  // [lane][KP]: phase p → (p/K, p%K)
  if (MODE == MODE_HW && a.season_out) {
    for (int p = tid; p < a.m; p += blockDim.x) a.season_out[(long long)n * a.m + p] = sfin[(p / K) * KP + p % K];
  }
  const int Tp = a.Tp, m = a.m;
  detect_epilogue(a.det, n, sig, n_valid,
                  [&](int h) {
                    float f = gL + (float)h * gB;
                    if (MODE == MODE_HW) {
                      int ph = (Tp - 1 + h) % m;
                      if (ph < 0) ph += m;
                      f += sfin[(ph / K) * KP + ph % K];
                    }
                    return f;
                  },
                  red, gIdx);
}

template <int K>
static constexpr int kp_of(int bf16) {
  return bf16 ? ((K + 7) / 8) * 8 : ((K + 3) / 4) * 4;
}

extern "C" size_t fm_hw_scan_lds_bytes(int Tp, int seg, int K, int mode, int bf16) {
  int KP;
  switch (K) {
    case 8: KP = 8; break;
    case 12: KP = bf16 ? 16 : 12; break;
    case 16: KP = 16; break;
    case 24: KP = 24; break;
    case 32: KP = 32; break;
    default: return (size_t)-1;
  }
  const int nseg = Tp / seg;
  size_t off = ((size_t)nseg * 64 * KP * (bf16 ? 2 : 4) + 15) & ~(size_t)15;
  if (mode == MODE_HW) off += (size_t)4 * 64 * KP * 4;
  off += ((size_t)nseg * 4 + 15) & ~(size_t)15;
  off += 64 * 4 + 16 * 4;
  return off;
}

// variant: 0 = 1 combo/lane, >=3 waves/SIMD; 1 = 1 combo/lane, 2 waves/SIMD;
//          2 = 2 combos/lane (packed FP32), 2 waves/SIMD
template <int K, int MODE, int NC, int MINW, bool TAB = false>
static hipError_t launch_v(const SmoothArgs& a, int bf16, size_t lds, hipStream_t st) {
  if (bf16)
    hipLaunchKernelGGL((hw_scan_kernel<K, MODE, bf16_t, NC, MINW, TAB>), dim3(a.N), dim3(256), lds, st, a);
  else
    hipLaunchKernelGGL((hw_scan_kernel<K, MODE, float, NC, MINW, TAB>), dim3(a.N), dim3(256), lds, st, a);
  return hipGetLastError();
}

template <int K, int MODE>
static hipError_t launch_fast(const SmoothArgs& a, int bf16, size_t lds, hipStream_t st, int variant) {
  switch (variant) {
    case 1: return launch_v<K, MODE, 1, 2>(a, bf16, lds, st);
    case 2: return launch_v<K, MODE, 2, 2>(a, bf16, lds, st);
    case 3:
      if (!a.pair_tab) return hipErrorInvalidValue;
      return launch_v<K, MODE, 2, 2, true>(a, bf16, lds, st);
    default: return launch_v<K, MODE, 1, 3>(a, bf16, lds, st);
  }
}

template <int K, int MODE>
static hipError_t launch_fast0(const SmoothArgs& a, int bf16, size_t lds, hipStream_t st, int) {
  return launch_v<K, MODE, 1, 3>(a, bf16, lds, st);
}

// Returns hipErrorNotSupported when the geometry is not uniform (caller falls back).
extern "C" int fm_hw_scan_fit(const SmoothArgs* a, int mode, int bf16, int variant, hipStream_t st) {
  const int K = a->K;
  if (a->seg % K != 0 || a->seg / K > 64 || a->Tp % a->seg != 0) return (int)hipErrorNotSupported;
  const size_t lds = fm_hw_scan_lds_bytes(a->Tp, a->seg, K, mode, bf16);
  if (lds == (size_t)-1 || lds > 64 * 1024) return (int)hipErrorNotSupported;
  if (a->N <= 0) return 0;
  hipError_t e = hipErrorNotSupported;
  if (mode == MODE_HW) {
    switch (K) {
      case 8: e = launch_fast0<8, MODE_HW>(*a, bf16, lds, st, variant); break;
      case 12: e = launch_fast0<12, MODE_HW>(*a, bf16, lds, st, variant); break;
      case 16: e = launch_fast0<16, MODE_HW>(*a, bf16, lds, st, variant); break;
      case 24: e = launch_fast<24, MODE_HW>(*a, bf16, lds, st, variant); break;
      case 32: e = launch_fast0<32, MODE_HW>(*a, bf16, lds, st, variant); break;
      default: return (int)hipErrorNotSupported;
    }
  } else if (K == 16) {
    e = (mode == MODE_ES) ? launch_fast<16, MODE_ES>(*a, bf16, lds, st, variant)
                          : launch_fast<16, MODE_DES>(*a, bf16, lds, st, variant);
  } else {
    return (int)hipErrorNotSupported;
  }
  return (int)e;
}
