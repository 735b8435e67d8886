// K7: fused LSTM-autoencoder training pass (forward + backward through time)
// on MFMA, for the data-parallel trainer (foremast_amd/parallel/dp.py).
//
// Semantics = foremast_amd/models/lstm_ae.py, loss = mean over the batch of
// the per-window reconstruction MSE.  One 64-lane wave owns 32 windows
// (lane l: window l&31, hidden-unit half l>>5), exactly as the inference
// kernel (lstm.hip), and runs four phases back to back:
//
//   1. encoder forward  (40 MFMA / step, x + bias in the 5th k-step)
//   2. decoder forward  (+ read-out y_t, dL/dy_t)
//   3. decoder backward (t = T-1 .. 0)
//   4. encoder backward (t = T-1 .. 0), seeded by the decoder's dh/dc at t=0
//
// Forward saves the activated gates (i, f, g, o) and c_t per step in a
// lane-major fp32 scratch (layout below).  Backward
// recomputes nothing: per unit the cell gradient is lane-local, and
//   dh_{t-1} = W_hh^T · dgates_t
// is 32 MFMAs (2 M-tiles x 16 k-steps) whose B operand is the lane's own
// dgates (k ordered as the forward accumulator registers) and whose A
// operand is W_hh^T packed host-side so that the accumulator lands in the
// h register layout — no LDS transpose anywhere in the recurrence.
//
// Weight gradients are NOT reduced in the kernel: it streams dgates (bf16,
// PyTorch gate-row order) and the augmented inputs [h_{t-1}; x_t; 1] (bf16)
// to HBM as K-contiguous [rows, T*B] matrices (a wave's 32 windows write 64
// contiguous bytes per row), and the host forms
//   dW_aug = G · Haug^T   (one hipBLASLt GEMM per LSTM, K = T*B)
// in the "both operands K-contiguous" form hipBLASLt runs fastest.
// (A row-per-(t, window) layout with 16-byte stores made the kernel no
// faster and the GEMM 3.5x slower: measured, scripts/bench_lstm_kernels.py.)
// Scratch is float4-vectorised: per step a lane owns 40 float4 (gates i,f,g,o
// of unit u at float4 u, c of units 4k..4k+3 at float4 32+k), and every
// scratch access of a wave is one contiguous 1 KB segment.
#include "common.h"
#include "lstm_common.h"

struct LstmTrainArgs {
  const float* x;        // [B, T, F] normalised windows; B % 32 == 0
  int B;
  int T;
  int F;                 // 1..7
  int phases;            // bitmask (profiling): 1 enc fwd, 2 dec fwd, 4 dec bwd, 8 enc bwd; 0 = all
  const uint4* w_enc;    // forward A fragments [8][5][64] (bf16 x 8)
  const uint4* w_dec;
  const uint4* wt_enc;   // backward (W_hh^T) A fragments [2][16][64]
  const uint4* wt_dec;
  const float* w_out;    // [F][64]
  const float* b_out;    // [F]
  float* scratch;        // [waves][2][T][40][64] float4
  bf16_t* g_enc;         // [256][T*B]  dL/dgates, PyTorch row order
  bf16_t* g_dec;         // [256][T*B]
  bf16_t* h_enc;         // [80][T*B]   rows 0..63 h_{t-1}, 64..64+F-1 x_t (row 71 = 1 preset by host)
  bf16_t* h_dec;         // [80][(T+1)*B] block 0 = encoder final h, block t+1 = decoder h_t
  float* dy;             // [F][T*B]    dL/dy
  float* err;            // [B]         per-window reconstruction MSE
  float loss_scale;      // 2 / (B*T*F)
  int variant;           // 0: one wave per 32 windows; 1: two waves (hidden units split, LDS exchange)
  LstmRingSrc src;       // ring-direct input (x == null): sampled windows read from the history rings
};

extern __shared__ __attribute__((aligned(16))) char fm_lstm_train_smem[];

namespace {

using namespace fm_lstm;

constexpr int SV4 = 40;  // float4 per lane per step: 32 units x (i, f, g, o) + 32 c
constexpr int WT_FRAGS = 2 * 16;

__device__ __forceinline__ int unit_of(int tile, int hh, int q) {
  return 16 * (tile >> 1) + 8 * hh + 4 * (tile & 1) + q;
}

__device__ __forceinline__ bf16x8_t as_bf16x8(const uint4& v) {
  bf16x8_t r;
  __builtin_memcpy(&r, &v, 16);
  return r;
}

__device__ __forceinline__ f32x16 mfma_bf16(const uint4& a, const uint4& b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(a), as_bf16x8(b), c, 0, 0, 0);
}

__device__ __forceinline__ uint4 pack8(const float (&v)[8]) {
  uint4 r;
  r.x = pack_bf16x2(v[0], v[1]);
  r.y = pack_bf16x2(v[2], v[3]);
  r.z = pack_bf16x2(v[4], v[5]);
  r.w = pack_bf16x2(v[6], v[7]);
  return r;
}

__device__ __forceinline__ void stage(uint4* dst, const uint4* src, int n16) {
  for (int i = threadIdx.x; i < n16; i += blockDim.x) dst[i] = src[i];
}

// ---------------------------------------------------------------- forward
template <bool ENC>
__device__ __forceinline__ void fwd_phase(const LstmTrainArgs& a, const uint4* wlds, const float* wout,
                                          float4* scr, long long b, int hh, long long KB,
                                          float (&hreg)[32], float (&creg)[32], float& errsum) {
  const int lane = lane_id();
  const XPos xp = make_xpos(a.x, a.src, b, a.T, a.F);
  bf16_t* hbuf = ENC ? a.h_enc : a.h_dec;
  const long long ldh = ENC ? KB : KB + a.B;
  for (int t = 0; t < a.T; ++t) {
    const long long row = (long long)t * a.B + b;  // column of the [rows, T*B] matrices
    // augmented input [h_{t-1}; x_t; 1] for the weight-gradient GEMM
    if (ENC || t == 0) {
#pragma unroll
      for (int tt = 0; tt < TILES; ++tt)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          hbuf[(long long)unit_of(tt, hh, q) * ldh + row] = bf16_hw(hreg[4 * tt + q]);
    }
    uint4 hb[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = hreg[(2 * s + (j >> 2)) * 4 + (j & 3)];
      hb[s] = pack8(v);
    }
    uint4 xb;
    {
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (hh == 0) {
        if (ENC) {
#pragma unroll
          for (int f = 0; f < 7; ++f)
            if (f < a.F) {
              v[f] = load_x(a.src, xp, t, f, a.F);
              a.h_enc[(long long)(64 + f) * KB + row] = bf16_hw(v[f]);
            }
        }
        v[7] = 1.f;
      }
      xb = pack8(v);
    }
    int lo = lane;
    asm volatile("" : "+v"(lo));
    float4* srow = scr + (long long)t * SV4 * 64 + lane;
#pragma unroll
    for (int tp = 0; tp < TILES; tp += 2) {
      f32x16 acc0 = (f32x16){}, acc1 = (f32x16){};
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s) {
        const uint4 bfr = (s < 4) ? hb[s] : xb;
        acc0 = mfma_bf16(wlds[(tp * KSTEPS + s) * 64 + lo], bfr, acc0);
        acc1 = mfma_bf16(wlds[((tp + 1) * KSTEPS + s) * 64 + lo], bfr, acc1);
      }
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const f32x16& acc = e ? acc1 : acc0;
        float4 cv;
#pragma unroll
        for (int q = 0; q < 4; q += 2) {  // two units at a time: packed-FP32 activation arithmetic
          const f32x2_t gi = sigm2((f32x2_t){acc[q], acc[q + 1]}), gf = sigm2((f32x2_t){acc[4 + q], acc[5 + q]});
          const f32x2_t gg = tanh2((f32x2_t){acc[8 + q], acc[9 + q]});
          const f32x2_t go = sigm2((f32x2_t){acc[12 + q], acc[13 + q]});
          const int u = (tp + e) * 4 + q;
          const f32x2_t c = gf * (f32x2_t){creg[u], creg[u + 1]} + gi * gg;
          const f32x2_t h = go * tanh2(c);
          creg[u] = c.x;
          creg[u + 1] = c.y;
          hreg[u] = h.x;
          hreg[u + 1] = h.y;
          srow[u * 64] = make_float4(gi.x, gf.x, gg.x, go.x);
          srow[(u + 1) * 64] = make_float4(gi.y, gf.y, gg.y, go.y);
          (&cv.x)[q] = c.x;
          (&cv.x)[q + 1] = c.y;
        }
        srow[(32 + tp + e) * 64] = cv;
      }
    }
    if (!ENC) {
      // decoder output block t+1 (h_t) for dW_dec (as h_prev of step t+1) and dW_out
      const long long row1 = (long long)(t + 1) * a.B + b;
#pragma unroll
      for (int tt = 0; tt < TILES; ++tt)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          a.h_dec[(long long)unit_of(tt, hh, q) * ldh + row1] = bf16_hw(hreg[4 * tt + q]);
#pragma unroll
      for (int f = 0; f < 7; ++f) {
        if (f >= a.F) break;
        float p = 0.f;
#pragma unroll
        for (int tt = 0; tt < TILES; ++tt)
#pragma unroll
          for (int q = 0; q < 4; ++q) p += hreg[tt * 4 + q] * wout[f * H + unit_of(tt, hh, q)];
        p += __shfl_xor(p, 32, FM_WAVE);
        const float d = p + a.b_out[f] - load_x(a.src, xp, t, f, a.F);
        if (hh == 0) {
          errsum += d * d;
          a.dy[(long long)f * KB + row] = d * a.loss_scale;
        }
      }
    }
  }
}

// ---------------------------------------------------------------- backward
// c_prev of step t: scratch c of step t-1, or `c0` (per-unit registers) at t = 0.
template <bool ENC>
__device__ __forceinline__ void bwd_phase(const LstmTrainArgs& a, const uint4* wt, const float* wout,
                                          const float4* scr, const float (&c0)[32], long long b, int hh,
                                          long long KB, float (&dh)[32], float (&dc)[32]) {
  const int lane = lane_id();
  bf16_t* gbuf = ENC ? a.g_enc : a.g_dec;
  for (int t = a.T - 1; t >= 0; --t) {
    const long long row = (long long)t * a.B + b;
    if (!ENC) {
      // dL/dh_t += W_out^T dL/dy_t
#pragma unroll
      for (int f = 0; f < 7; ++f) {
        if (f >= a.F) break;
        const float dyf = a.dy[(long long)f * KB + row];
#pragma unroll
        for (int tt = 0; tt < TILES; ++tt)
#pragma unroll
          for (int q = 0; q < 4; ++q) dh[4 * tt + q] += dyf * wout[f * H + unit_of(tt, hh, q)];
      }
    }
    const float4* srow = scr + (long long)t * SV4 * 64 + lane;
    const float4* sprev = scr + (long long)(t - 1) * SV4 * 64 + lane;
    int lo = lane;
    asm volatile("" : "+v"(lo));
    f32x16 acc0 = (f32x16){}, acc1 = (f32x16){};  // dh_{t-1}: units of M-tile 0 / 1
#pragma unroll
    for (int tt = 0; tt < TILES; ++tt) {
      float dg[16];
      const float4 cv = srow[(32 + tt) * 64];
      float4 cpv;
      if (t > 0) cpv = sprev[(32 + tt) * 64];
      else cpv = make_float4(c0[4 * tt], c0[4 * tt + 1], c0[4 * tt + 2], c0[4 * tt + 3]);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int u = 4 * tt + q;
        const float4 gv = srow[u * 64];
        const float gi = gv.x, gf = gv.y, gg = gv.z, go = gv.w;
        const float c = (&cv.x)[q], cp = (&cpv.x)[q];
        const float tc = tanh_f(c);
        const float dcu = dc[u] + dh[u] * go * (1.f - tc * tc);
        dg[q] = dcu * gg * gi * (1.f - gi);            // i
        dg[4 + q] = dcu * cp * gf * (1.f - gf);        // f
        dg[8 + q] = dcu * gi * (1.f - gg * gg);        // g
        dg[12 + q] = dh[u] * tc * go * (1.f - go);     // o
        dc[u] = dcu * gf;
      }
      // dgates → HBM (PyTorch gate-row order: gate*64 + unit)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        gbuf[(long long)((r >> 2) * H + unit_of(tt, hh, r & 3)) * KB + row] = bf16_hw(dg[r]);
      // dh_{t-1} += W_hh^T[:, rows of this tile] · dgates (2 k-steps x 2 M-tiles)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = dg[8 * e + j];
        const uint4 bfr = pack8(v);
        const int ks = 2 * tt + e;
        acc0 = mfma_bf16(wt[(0 * 16 + ks) * 64 + lo], bfr, acc0);
        acc1 = mfma_bf16(wt[(1 * 16 + ks) * 64 + lo], bfr, acc1);
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      dh[r] = acc0[r];
      dh[16 + r] = acc1[r];
    }
  }
}

__global__ __launch_bounds__(64, 1) void lstm_ae_train_kernel(const LstmTrainArgs a) {
  const int lane = lane_id();
  const int hh = lane >> 5;
  const long long wave = blockIdx.x;
  const long long b = wave * 32 + (lane & 31);  // host guarantees B % 32 == 0
  const long long KB = (long long)a.T * a.B;
  uint4* wlds = (uint4*)fm_lstm_train_smem;
  float* wout = (float*)(fm_lstm_train_smem + FRAG_BYTES_BF16);
  float4* scr_enc = (float4*)a.scratch + wave * 2 * (long long)a.T * SV4 * 64;
  float4* scr_dec = scr_enc + (long long)a.T * SV4 * 64;

  for (int i = threadIdx.x; i < a.F * H; i += blockDim.x) wout[i] = a.w_out[i];
  stage(wlds, a.w_enc, FRAG_BYTES_BF16 / 16);
  __syncthreads();
  float hreg[32], creg[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) { hreg[i] = 0.f; creg[i] = 0.f; }
  float errsum = 0.f;
  const int ph = a.phases ? a.phases : 15;
  if (ph & 1) fwd_phase<true>(a, wlds, wout, scr_enc, b, hh, KB, hreg, creg, errsum);
  float c_enc[32];  // encoder final c = decoder c_prev at t = 0
#pragma unroll
  for (int i = 0; i < 32; ++i) c_enc[i] = creg[i];
  __syncthreads();
  stage(wlds, a.w_dec, FRAG_BYTES_BF16 / 16);
  __syncthreads();
  if (ph & 2) fwd_phase<false>(a, wlds, wout, scr_dec, b, hh, KB, hreg, creg, errsum);
  if (hh == 0) a.err[b] = errsum / (float)(a.T * a.F);

  // backward: decoder, then encoder
  __syncthreads();
  stage(wlds, a.wt_dec, WT_FRAGS * 64);
  __syncthreads();
  float dh[32], dc[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) { dh[i] = 0.f; dc[i] = 0.f; }
  if (ph & 4) bwd_phase<false>(a, wlds, wout, scr_dec, c_enc, b, hh, KB, dh, dc);
  __syncthreads();
  stage(wlds, a.wt_enc, WT_FRAGS * 64);
  __syncthreads();
  float zero[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) zero[i] = 0.f;
  if (ph & 8) bwd_phase<true>(a, wlds, wout, scr_enc, zero, b, hh, KB, dh, dc);
}


// ================================================================ variant 1
// Two waves per 32 windows: wave w owns gate tiles 4w..4w+3, i.e. hidden units
// 32w..32w+31 (both lane halves).  Per time step each wave issues half the
// MFMAs and half the cell math; the halves meet once per step through a
// double-buffered LDS exchange:
//  * forward: each wave publishes its two h B-fragments (k-steps 2w, 2w+1) and
//    its partial read-out; after one barrier the other wave's fragments
//    complete the next step's B operand;
//  * backward: each wave forms dh partials for BOTH M-tiles from its own
//    dgates k-steps, keeps its own M-tile and hands the other one over.
// Twice the waves in flight and half the dependency chain per wave per step.
constexpr int SV4H = 20;  // per wave per step: 16 units x (i,f,g,o) + 16 c

struct Xch {
  uint4* hb;    // [2 buf][2 wave][2 frag][64]
  float* y;     // [2 buf][2 wave][8][64]
  float* dh;    // [2 buf][2 wave][16][64]
};

template <bool ENC>
__device__ __forceinline__ void fwd_phase2(const LstmTrainArgs& a, const uint4* wlds, const float* wout, float4* scr,
                                           long long b, int hh, int w, long long KB, float (&hreg)[16],
                                           float (&creg)[16], float& errsum, const Xch& x) {
  const int lane = lane_id();
  const int TB = 4 * w;
  const XPos xp = make_xpos(a.x, a.src, b, a.T, a.F);
  bf16_t* hbuf = ENC ? a.h_enc : a.h_dec;
  const long long ldh = ENC ? KB : KB + a.B;
  // prologue: publish the initial h (zeros for the encoder, the encoder's final h for the decoder)
  // h as MFMA B fragments: k-steps 2w, 2w + 1 are this wave's units (hm), the other two the
  // other wave's (ho).  Kept as two arrays with compile-time indices: one array indexed by
  // the run-time wave id lived in scratch (four 16-byte scratch loads per time step)
  uint4 hm[2], ho[2];
  auto publish_h = [&](int buf) {
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = hreg[(2 * sl + (j >> 2)) * 4 + (j & 3)];
      const uint4 f = pack8(v);
      hm[sl] = f;
      x.hb[((buf * 2 + w) * 2 + sl) * 64 + lane] = f;
    }
  };
  auto collect_h = [&](int buf) {
    const int o = 1 - w;
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) ho[sl] = x.hb[((buf * 2 + o) * 2 + sl) * 64 + lane];
  };
  publish_h(1);
  __syncthreads();
  collect_h(1);
  for (int t = 0; t < a.T; ++t) {
    const int buf = t & 1;
    const long long row = (long long)t * a.B + b;
    if (ENC || t == 0) {
#pragma unroll
      for (int tl = 0; tl < 4; ++tl)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          hbuf[(long long)unit_of(TB + tl, hh, q) * ldh + row] = bf16_hw(hreg[4 * tl + q]);
    }
    uint4 xb;
    {
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (hh == 0) {
        if (ENC) {
#pragma unroll
          for (int f = 0; f < 7; ++f)
            if (f < a.F) {
              v[f] = load_x(a.src, xp, t, f, a.F);
              if (w == 0) a.h_enc[(long long)(64 + f) * KB + row] = bf16_hw(v[f]);
            }
        }
        v[7] = 1.f;
      }
      xb = pack8(v);
    }
    int lo = lane;
    asm volatile("" : "+v"(lo));
    float4* srow = scr + (long long)t * SV4H * 64 + lane;
#pragma unroll
    for (int tp = 0; tp < 4; tp += 2) {
      f32x16 acc0 = (f32x16){}, acc1 = (f32x16){};
#pragma unroll
      for (int k = 0; k < KSTEPS; ++k) {
        // k-step order: this wave's two h steps, the other wave's two, then x (h steps are
        // summed in a wave-dependent order; the weight fragment follows the step)
        const uint4 bfr = k < 2 ? hm[k] : k < 4 ? ho[k - 2] : xb;
        const int s = k < 4 ? ((k + 2 * w) & 3) : k;
        acc0 = mfma_bf16(wlds[((TB + tp) * KSTEPS + s) * 64 + lo], bfr, acc0);
        acc1 = mfma_bf16(wlds[((TB + tp + 1) * KSTEPS + s) * 64 + lo], bfr, acc1);
      }
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const f32x16& acc = e ? acc1 : acc0;
        float4 cv;
#pragma unroll
        for (int q = 0; q < 4; q += 2) {  // two units at a time: packed-FP32 activation arithmetic
          const f32x2_t gi = sigm2((f32x2_t){acc[q], acc[q + 1]}), gf = sigm2((f32x2_t){acc[4 + q], acc[5 + q]});
          const f32x2_t gg = tanh2((f32x2_t){acc[8 + q], acc[9 + q]});
          const f32x2_t go = sigm2((f32x2_t){acc[12 + q], acc[13 + q]});
          const int u = (tp + e) * 4 + q;
          const f32x2_t c = gf * (f32x2_t){creg[u], creg[u + 1]} + gi * gg;
          const f32x2_t h = go * tanh2(c);
          creg[u] = c.x;
          creg[u + 1] = c.y;
          hreg[u] = h.x;
          hreg[u + 1] = h.y;
          srow[u * 64] = make_float4(gi.x, gf.x, gg.x, go.x);
          srow[(u + 1) * 64] = make_float4(gi.y, gf.y, gg.y, go.y);
          (&cv.x)[q] = c.x;
          (&cv.x)[q + 1] = c.y;
        }
        srow[(16 + tp + e) * 64] = cv;
      }
    }
    float py[7];
    if (!ENC) {
      const long long row1 = (long long)(t + 1) * a.B + b;
#pragma unroll
      for (int tl = 0; tl < 4; ++tl)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          a.h_dec[(long long)unit_of(TB + tl, hh, q) * ldh + row1] = bf16_hw(hreg[4 * tl + q]);
#pragma unroll
      for (int f = 0; f < 7; ++f) {
        py[f] = 0.f;
        if (f >= a.F) continue;
        float p = 0.f;
#pragma unroll
        for (int tl = 0; tl < 4; ++tl)
#pragma unroll
          for (int q = 0; q < 4; ++q) p += hreg[tl * 4 + q] * wout[f * H + unit_of(TB + tl, hh, q)];
        p += __shfl_xor(p, 32, FM_WAVE);
        py[f] = p;
        x.y[((buf * 2 + w) * 8 + f) * 64 + lane] = p;
      }
    }
    publish_h(buf);
    __syncthreads();
    collect_h(buf);
    if (!ENC) {
#pragma unroll
      for (int f = 0; f < 7; ++f) {
        if (f >= a.F) break;
        const float y = py[f] + x.y[((buf * 2 + (1 - w)) * 8 + f) * 64 + lane] + a.b_out[f];
        const float d = y - load_x(a.src, xp, t, f, a.F);
        if (w == 0 && hh == 0) {
          errsum += d * d;
          a.dy[(long long)f * KB + row] = d * a.loss_scale;
        }
      }
    }
  }
}

template <bool ENC>
__device__ __forceinline__ void bwd_phase2(const LstmTrainArgs& a, const uint4* wt, const float* wout,
                                           const float4* scr, const float (&c0)[16], long long b, int hh, int w,
                                           long long KB, float (&dh)[16], float (&dc)[16], const Xch& x) {
  const int lane = lane_id();
  const int TB = 4 * w;
  bf16_t* gbuf = ENC ? a.g_enc : a.g_dec;
  for (int t = a.T - 1; t >= 0; --t) {
    const int buf = t & 1;
    const long long row = (long long)t * a.B + b;
    if (!ENC) {  // dy was written by wave 0 during the forward; phase barriers made it visible
#pragma unroll
      for (int f = 0; f < 7; ++f) {
        if (f >= a.F) break;
        const float dyf = a.dy[(long long)f * KB + row];
#pragma unroll
        for (int tl = 0; tl < 4; ++tl)
#pragma unroll
          for (int q = 0; q < 4; ++q) dh[4 * tl + q] += dyf * wout[f * H + unit_of(TB + tl, hh, q)];
      }
    }
    const float4* srow = scr + (long long)t * SV4H * 64 + lane;
    const float4* sprev = scr + (long long)(t - 1) * SV4H * 64 + lane;
    int lo = lane;
    asm volatile("" : "+v"(lo));
    f32x16 acc0 = (f32x16){}, acc1 = (f32x16){};
#pragma unroll
    for (int tl = 0; tl < 4; ++tl) {
      const int tt = TB + tl;
      float dg[16];
      const float4 cv = srow[(16 + tl) * 64];
      float4 cpv;
      if (t > 0) cpv = sprev[(16 + tl) * 64];
      else cpv = make_float4(c0[4 * tl], c0[4 * tl + 1], c0[4 * tl + 2], c0[4 * tl + 3]);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int u = 4 * tl + q;
        const float4 gv = srow[u * 64];
        const float gi = gv.x, gf = gv.y, gg = gv.z, go = gv.w;
        const float c = (&cv.x)[q], cp = (&cpv.x)[q];
        const float tc = tanh_f(c);
        const float dcu = dc[u] + dh[u] * go * (1.f - tc * tc);
        dg[q] = dcu * gg * gi * (1.f - gi);
        dg[4 + q] = dcu * cp * gf * (1.f - gf);
        dg[8 + q] = dcu * gi * (1.f - gg * gg);
        dg[12 + q] = dh[u] * tc * go * (1.f - go);
        dc[u] = dcu * gf;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r)
        gbuf[(long long)((r >> 2) * H + unit_of(tt, hh, r & 3)) * KB + row] = bf16_hw(dg[r]);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = dg[8 * e + j];
        const uint4 bfr = pack8(v);
        const int ks = 2 * tt + e;
        acc0 = mfma_bf16(wt[(0 * 16 + ks) * 64 + lo], bfr, acc0);
        acc1 = mfma_bf16(wt[(1 * 16 + ks) * 64 + lo], bfr, acc1);
      }
    }
    // keep my M-tile (units 32w..), hand the other partial to the other wave
    const f32x16& mine = w ? acc1 : acc0;
    const f32x16& theirs = w ? acc0 : acc1;
#pragma unroll
    for (int r = 0; r < 16; ++r) x.dh[((buf * 2 + w) * 16 + r) * 64 + lane] = theirs[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) dh[r] = mine[r] + x.dh[((buf * 2 + (1 - w)) * 16 + r) * 64 + lane];
  }
}

__global__ __launch_bounds__(128, 1) void lstm_ae_train_kernel2(const LstmTrainArgs a) {
  const int lane = lane_id();
  const int hh = lane >> 5;
  const int w = wave_id();
  const long long grp = blockIdx.x;
  const long long b = grp * 32 + (lane & 31);
  const long long KB = (long long)a.T * a.B;
  char* smem = fm_lstm_train_smem;
  uint4* wlds = (uint4*)smem;
  float* wout = (float*)(smem + FRAG_BYTES_BF16);
  Xch x;
  x.hb = (uint4*)(smem + FRAG_BYTES_BF16 + 7 * H * 4);
  x.y = (float*)(x.hb + 2 * 2 * 2 * 64);
  x.dh = x.y + 2 * 2 * 8 * 64;
  float4* base = (float4*)a.scratch + grp * 2 * 2 * (long long)a.T * SV4H * 64;
  float4* scr_enc = base + (0 * 2 + w) * (long long)a.T * SV4H * 64;
  float4* scr_dec = base + (1 * 2 + w) * (long long)a.T * SV4H * 64;

  for (int i = threadIdx.x; i < a.F * H; i += blockDim.x) wout[i] = a.w_out[i];
  stage(wlds, a.w_enc, FRAG_BYTES_BF16 / 16);
  __syncthreads();
  float hreg[16], creg[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) { hreg[i] = 0.f; creg[i] = 0.f; }
  float errsum = 0.f;
  const int ph = a.phases ? a.phases : 15;
  if (ph & 1) fwd_phase2<true>(a, wlds, wout, scr_enc, b, hh, w, KB, hreg, creg, errsum, x);
  float c_enc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) c_enc[i] = creg[i];
  __syncthreads();
  stage(wlds, a.w_dec, FRAG_BYTES_BF16 / 16);
  __syncthreads();
  if (ph & 2) fwd_phase2<false>(a, wlds, wout, scr_dec, b, hh, w, KB, hreg, creg, errsum, x);
  if (w == 0 && hh == 0) a.err[b] = errsum / (float)(a.T * a.F);
  __syncthreads();
  stage(wlds, a.wt_dec, WT_FRAGS * 64);
  __syncthreads();
  float dh[16], dc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) { dh[i] = 0.f; dc[i] = 0.f; }
  if (ph & 4) bwd_phase2<false>(a, wlds, wout, scr_dec, c_enc, b, hh, w, KB, dh, dc, x);
  __syncthreads();
  stage(wlds, a.wt_enc, WT_FRAGS * 64);
  __syncthreads();
  float zero[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) zero[i] = 0.f;
  if (ph & 8) bwd_phase2<true>(a, wlds, wout, scr_enc, zero, b, hh, w, KB, dh, dc, x);
}

}  // namespace

extern "C" size_t fm_lstm_train_lds_bytes(int F) { return (size_t)FRAG_BYTES_BF16 + (size_t)F * H * 4; }

static size_t lds_bytes_v1() {
  return (size_t)FRAG_BYTES_BF16 + 7 * H * 4 + 2 * 2 * 2 * 64 * 16 + (2 * 2 * 8 * 64 + 2 * 2 * 16 * 64) * 4;
}

extern "C" long long fm_lstm_train_scratch_floats(int B, int T) {
  return (long long)(B / 32) * 2 * T * SV4 * 64 * 4;
}

extern "C" long long fm_lstm_train_args_size() { return (long long)sizeof(LstmTrainArgs); }

extern "C" int fm_lstm_ae_train(const LstmTrainArgs* a, hipStream_t st) {
  if (a->B <= 0) return 0;
  if (a->B % 32 || a->F < 1 || a->F > 7 || a->T < 1) return (int)hipErrorInvalidValue;
  if (a->variant == 1)
    hipLaunchKernelGGL(lstm_ae_train_kernel2, dim3((unsigned)(a->B / 32)), dim3(128), lds_bytes_v1(), st, *a);
  else
    hipLaunchKernelGGL(lstm_ae_train_kernel, dim3((unsigned)(a->B / 32)), dim3(64),
                       fm_lstm_train_lds_bytes(a->F), st, *a);
  return (int)hipGetLastError();
}
