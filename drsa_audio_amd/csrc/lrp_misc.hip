// LRP engine kernels besides the 3x3 conv:
//   * dense head   (classifier Linear layers; Epsilon rule, reference constants.py:35-37)
//   * projection   (ProjectionModel virtual layers, reference modify_model.py:75-123, with the
//                   composite of explainer.py:198-203: Epsilon on invprojection, SubspaceHook mask,
//                   Epsilon on projection; SubspaceHook.backward = attribute.py:53-60)
//   * first layer  (WSquare / Flat backward, reference constants.py:29,42; zennit 0.5.1)
//   * denominator map of WSquare / Flat (input independent)
//   * heatmap split / per-subspace sums / descending sort (explainer.py:99-176)
#include "common.h"

#include <stdlib.h>
#include "lrp_conv.h"

namespace {

// ===========================================================================
// dense head: C[M][N] = A[M][K] B[K][N] on fp32 MFMA 16x16x4, 32x32 workgroup tile
//   forward : A = x,  B[k][n] = W[n][k];  z = acc + b;  optional a = relu(z)
//   backward: A[m][n] = g = prologue(R | seed, z), B[n][k] = W[n][k];  out = epilogue(acc, x, den)
// ===========================================================================
constexpr int LT = 32;   // workgroup tile (M and N)
constexpr int LK = 32;   // K chunk

struct LinArgs {
  const float* A;        // fwd: x [M][K]; bwd: R [M][Kg] (ignored when seed)
  const float* W;        // [Nout][Kin] (torch Linear weight)
  const float* bias;     // fwd
  const float* z;        // bwd: forward output of this layer [M][Kg]
  const int* cls;        // bwd seed: class per row (nullable -> not seed)
  const float* x;        // bwd: forward input of this layer [M][N]
  const float* den;      // bwd POST_DIV: next (lower) layer denominator, same indexing as out
  float* out;            // fwd: z [M][N]; bwd: R_in or g_next [M][N]
  float* out_relu;       // fwd: relu(z) (nullable)
  int M, N, K;           // GEMM dims
  int bwd;
  int one_hot, relu_mask, rule_eps, xmode, post;
  float eps, eps_post;
};

__global__ __launch_bounds__(256) void linear_kernel(LinArgs a) {
  __shared__ float As[LT][LK + 1];
  __shared__ float Bs[LK][LT + 1];
  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  const int m0 = blockIdx.x * LT, n0 = blockIdx.y * LT;
  const int wm = (w & 1) * 16, wn = (w >> 1) * 16;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < a.K; k0 += LK) {
    __syncthreads();
    for (int idx = tid; idx < LT * LK; idx += 256) {
      const int r = idx / LK, c = idx % LK;
      const int m = m0 + r, k = k0 + c;
      float v = 0.f;
      if (m < a.M && k < a.K) {
        if (!a.bwd) {
          v = a.A[(size_t)m * a.K + k];
        } else {
          // g = [z > 0]? R / stab(z) (rule Epsilon) or R (plain); R = seed or incoming relevance
          const float zz = a.z[(size_t)m * a.K + k];
          float R;
          if (a.cls) {
            const bool hit = (k == a.cls[m]);
            R = hit ? (a.one_hot ? 1.f : zz) : 0.f;
          } else {
            R = a.A[(size_t)m * a.K + k];
          }
          if (a.relu_mask && !(zz > 0.f)) R = 0.f;
          v = a.rule_eps ? R / stab(zz, a.eps) : R;
        }
      }
      As[r][c] = v;
    }
    for (int idx = tid; idx < LK * LT; idx += 256) {
      const int r = idx / LT, c = idx % LT;
      const int k = k0 + r, n = n0 + c;
      float v = 0.f;
      if (k < a.K && n < a.N) v = a.bwd ? a.W[(size_t)k * a.N + n] : a.W[(size_t)n * a.K + k];
      Bs[r][c] = v;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < LK; kk += 4) {
      const float av = As[wm + (lane & 15)][kk + (lane >> 4)];
      const float bv = Bs[kk + (lane >> 4)][wn + (lane & 15)];
      acc = mfma16(av, bv, acc);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + wm + (lane >> 4) * 4 + r, n = n0 + wn + (lane & 15);
    if (m >= a.M || n >= a.N) continue;
    const size_t o = (size_t)m * a.N + n;
    if (!a.bwd) {
      const float zz = acc[r] + (a.bias ? a.bias[n] : 0.f);
      a.out[o] = zz;
      if (a.out_relu) a.out_relu[o] = zz > 0.f ? zz : (zz != zz ? zz : 0.f);
    } else {
      float R = acc[r];
      if (a.xmode == XM_MUL) R = a.x[o] * R;
      if (a.post == POST_DIV) {
        const float xv = a.x[o];
        const float q = div_nb(R, stab(a.den[o], a.eps_post));
        R = (xv > 0.f) ? q : 0.f;
      } else if (a.post == POST_MASK) {
        R = (a.x[o] > 0.f) ? R : 0.f;
      }
      a.out[o] = R;
    }
  }
}

// Forward with K % 4 == 0 (the classifier input, K = 2048): 128-wide K chunks loaded as float4
// and the next chunk prefetched into registers while the current one runs, so the one
// k-ordered chain per output (oracle/lrp_exact.c:linear_exact) is no longer bound by one load
// round trip per 32 k.
constexpr int LFK = 128;

__global__ __launch_bounds__(256) void linear_fwd_kernel(LinArgs a) {
  __shared__ __attribute__((aligned(16))) float As[LT][LFK + 4];   // [m][k]
  __shared__ float Bs[LFK][LT + 1];                               // [k][n]
  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  const int m0 = blockIdx.x * LT, n0 = blockIdx.y * LT;
  const int wm = (w & 1) * 16, wn = (w >> 1) * 16;
  constexpr int NV = LT * LFK / 4 / 256;   // float4 per thread per operand
  float4 ra[NV], rb[NV];
#define LFWD_LOAD(K0)                                                                                     \
  _Pragma("unroll") for (int i = 0; i < NV; ++i) {                                                        \
    const int idx = tid + i * 256, r = idx / (LFK / 4), k = (K0) + (idx % (LFK / 4)) * 4;                 \
    const int m = m0 + r, n = n0 + r;                                                                     \
    const bool oa = m < a.M && k < a.K, ob = n < a.N && k < a.K;                                          \
    const float4 va = *reinterpret_cast<const float4*>(a.A + (oa ? (size_t)m * a.K + k : 0));             \
    const float4 vb = *reinterpret_cast<const float4*>(a.W + (ob ? (size_t)n * a.K + k : 0));             \
    ra[i] = oa ? va : make_float4(0.f, 0.f, 0.f, 0.f);                                                    \
    rb[i] = ob ? vb : make_float4(0.f, 0.f, 0.f, 0.f);                                                    \
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  LFWD_LOAD(0)
  for (int k0 = 0; k0 < a.K; k0 += LFK) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = tid + i * 256, r = idx / (LFK / 4), c = (idx % (LFK / 4)) * 4;
      *reinterpret_cast<float4*>(&As[r][c]) = ra[i];
      Bs[c][r] = rb[i].x; Bs[c + 1][r] = rb[i].y; Bs[c + 2][r] = rb[i].z; Bs[c + 3][r] = rb[i].w;
    }
    __syncthreads();
    if (k0 + LFK < a.K) { LFWD_LOAD(k0 + LFK) }
#pragma unroll
    for (int kk = 0; kk < LFK; kk += 4) {
      const float av = As[wm + (lane & 15)][kk + (lane >> 4)];
      const float bv = Bs[kk + (lane >> 4)][wn + (lane & 15)];
      acc = mfma16(av, bv, acc);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + wm + (lane >> 4) * 4 + r, n = n0 + wn + (lane & 15);
    if (m >= a.M || n >= a.N) continue;
    const size_t o = (size_t)m * a.N + n;
    const float zz = acc[r] + (a.bias ? a.bias[n] : 0.f);
    a.out[o] = zz;
    if (a.out_relu) a.out_relu[o] = zz > 0.f ? zz : (zz != zz ? zz : 0.f);
  }
#undef LFWD_LOAD
}

// Long K (the classifier input, K = 2048) with few output tiles (GTZAN: 512 x 128 = 256 16 x 16
// tiles): one wave per 16 x 16 output tile, so the grid covers the chip instead of 64 four-wave
// workgroups; K in 128-wide chunks staged through the wave's own LDS (a wave barrier, no workgroup
// barrier), the next chunk's 16 float4 loads in flight under the current chunk's 32 MFMAs.  The
// same single k-ordered chain per output as linear_fwd_kernel (bias added last): the same bits.
constexpr int L1K = 128;

__global__ __launch_bounds__(64) void linear_fwd_w1_kernel(LinArgs a) {
  __shared__ __attribute__((aligned(16))) float As[16][L1K + 4];   // [m][k]
  __shared__ float Bs[L1K][16 + 1];                                 // [k][n]
  const int lane = threadIdx.x;
  const int m0 = blockIdx.x * 16, n0 = blockIdx.y * 16;
  constexpr int NV = 16 * L1K / 4 / 64;   // float4 per lane per operand (8)
  float4 ra[NV], rb[NV];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = lane + i * 64, r = idx / (L1K / 4), k = k0 + (idx % (L1K / 4)) * 4;
      const int m = m0 + r, n = n0 + r;
      const bool oa = m < a.M && k < a.K, ob = n < a.N && k < a.K;
      const float4 va = *reinterpret_cast<const float4*>(a.A + (oa ? (size_t)m * a.K + k : 0));
      const float4 vb = *reinterpret_cast<const float4*>(a.W + (ob ? (size_t)n * a.K + k : 0));
      ra[i] = oa ? va : make_float4(0.f, 0.f, 0.f, 0.f);
      rb[i] = ob ? vb : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  load(0);
  for (int k0 = 0; k0 < a.K; k0 += L1K) {
    __builtin_amdgcn_wave_barrier();   // the previous chunk's LDS reads done (one wave: in order)
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = lane + i * 64, r = idx / (L1K / 4), c = (idx % (L1K / 4)) * 4;
      *reinterpret_cast<float4*>(&As[r][c]) = ra[i];
      Bs[c][r] = rb[i].x; Bs[c + 1][r] = rb[i].y; Bs[c + 2][r] = rb[i].z; Bs[c + 3][r] = rb[i].w;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the stores landed before this wave reads them
    __builtin_amdgcn_wave_barrier();
    if (k0 + L1K < a.K) load(k0 + L1K);
    // every operand of the chunk read before its chain (left to the scheduler each MFMA waits on
    // its own LDS round trip: one wave per SIMD has nothing else to hide it behind)
    float av[L1K / 4], bv[L1K / 4];
#pragma unroll
    for (int q = 0; q < L1K / 4; ++q) {
      av[q] = As[lane & 15][4 * q + (lane >> 4)];
      bv[q] = Bs[4 * q + (lane >> 4)][lane & 15];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < L1K / 4; ++q) acc = mfma16(av[q], bv[q], acc);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + (lane >> 4) * 4 + r, n = n0 + (lane & 15);
    if (m >= a.M || n >= a.N) continue;
    const size_t o = (size_t)m * a.N + n;
    const float zz = acc[r] + (a.bias ? a.bias[n] : 0.f);
    a.out[o] = zz;
    if (a.out_relu) a.out_relu[o] = zz > 0.f ? zz : (zz != zz ? zz : 0.f);
  }
}

// ===========================================================================
// projection forward: h = a_vec U, a' = h U^T, optional 2x2 max-pool of a'
//   a [B][d][H][W] -> h [B][d][H*W] (channel-major), ap [B][d][H][W], pooled + argmax
//   tile = 2 rows x 32 cols (64 pixels); a workgroup stages U once and walks PT tiles.
//   MFMA orientation D[channel][pixel]: lanes = pixels (coalesced I/O).
// Any d <= DP (DP = 16, 32, 64, 128): U and a are embedded in DP x DP / DP rows with zeros;
// the k chains run over d4 = round_up(d, 4) terms only, so for d % 4 == 0 (VGGish d = 100, 96)
// every value is the d-term chain of the unpadded product, bit for bit; outputs past d are
// computed (zeros) but not stored.
// ===========================================================================
// P = U U^T - I (d x d), the projection residual: each entry one float64 fma chain over k
// ascending (the products of two floats are exact in float64), minus the identity, rounded
// once to fp32.  P is symmetric bit for bit.  The projection kernels evaluate
//   a' = h U^T  as  a' = a + a P
// (equal in exact arithmetic): at a dead ReLU channel (a = 0) a' is then exact to its own
// rounding instead of carrying the O(1e-8) rounding noise of the d-term chain h U^T, which the
// invprojection's Epsilon(1e-6) amplifies into the subspace relevances.
__global__ __launch_bounds__(256) void projection_residual_kernel(const float* __restrict__ U, int d,
                                                                  float* __restrict__ P) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= d * d) return;
  const int r = i / d, c = i % d;
  double acc = 0.0;
  for (int k = 0; k < d; ++k) acc = fma((double)U[r * d + k], (double)U[c * d + k], acc);
  P[i] = (float)(acc - (r == c ? 1.0 : 0.0));
}

// MFMA A operand P[c][k] of lane (c, k), read as the symmetric P[k][c] so that the 16 lanes of a
// row group load 16 consecutive floats; zero outside the d x d matrix (padded embedding)
__device__ __forceinline__ float p_operand(const float* __restrict__ P, int d, int c, int k) {
  const bool ok = c < d && k < d;
  const float v = P[ok ? k * d + c : 0];
  return ok ? v : 0.f;
}

// P staged in LDS ([DP][DP + 16]: the four row groups of an MFMA operand read land on disjoint
// bank quarters), zero outside d x d; read transposed like p_operand
template <int DP>
__device__ __forceinline__ void stage_p(float* Ps, const float* __restrict__ P, int d, int tid) {
  constexpr int LP = DP + 16;
  for (int i = tid; i < DP * DP; i += 256) {
    const int k = i / DP, c = i % DP;
    const bool ok = k < d && c < d;
    const float v = P[ok ? k * d + c : 0];
    Ps[k * LP + c] = ok ? v : 0.f;
  }
}
template <int DP, bool PL>
__device__ __forceinline__ float p_op(const float* Ps, const float* __restrict__ P, int d, int c, int k) {
  if constexpr (PL) return Ps[k * (DP + 16) + c];
  else return p_operand(P, d, c, k);
}
template <int DP, bool PL>
constexpr size_t p_lds_floats() { return PL ? (size_t)DP * (DP + 16) : 0; }

constexpr int PT = 4;   // row-pair tiles per workgroup

template <int DP>
__device__ __forceinline__ void stage_u_padded(float* Us, const float* __restrict__ U, int d, int tid) {
  constexpr int LD = DP + 1;
  for (int i = tid; i < DP * DP; i += 256) {
    const int c = i / DP, j = i % DP;
    const bool ok = c < d && j < d;
    const float v = U[ok ? c * d + j : 0];
    Us[c * LD + j] = ok ? v : 0.f;
  }
}

// HOUT = false (the plan's default: projection_bwd recomputes h): only the residual GEMM
// delta = a P runs and U is not staged -- h = a U is needed by nobody (a' = a + delta).
template <int DP, bool PAD, bool PLDS, bool HOUT>
__global__ __launch_bounds__(256) void projection_fwd_kernel(const float* __restrict__ a, const float* __restrict__ U,
                                                            const float* __restrict__ Pm,
                                                            float* __restrict__ h, float* __restrict__ ap,
                                                            float* __restrict__ pooled, uint8_t* __restrict__ amax,
                                                            int d_in, int H, int W, int pool) {
  const int d = PAD ? d_in : DP;   // PAD = false: d == DP at compile time (no padding code)
  constexpr int P = 64, LD = DP + 1, PL = P + 4;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Us = sm;               // [DP][LD]   U[c][j] (HOUT only)
  float* as = Us + (HOUT ? DP * LD : 0);   // [DP][PL]   a tile, then a' tile
  float* Ps = as + DP * PL;     // [DP][DP + 16] P (when PLDS)
  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  const int b = blockIdx.y;
  const int TW = W < 32 ? W : 32, RPT = P / TW;      // tile = RPT rows x TW cols
  const int HW = H * W, xt = W / TW;
  const int d4 = (d + 3) & ~3;
  // per-sample bases + 32-bit per-lane offsets (saddr + voffset addressing; d * H * W < 2^31)
  const float* __restrict__ a_b = a + (size_t)b * d * HW;
  float* __restrict__ h_b = HOUT ? h + (size_t)b * d * HW : nullptr;
  float* __restrict__ ap_b = ap ? ap + (size_t)b * d * HW : nullptr;
  if constexpr (HOUT) stage_u_padded<DP>(Us, U, d, tid);
  if constexpr (PLDS) stage_p<DP>(Ps, Pm, d, tid);
  constexpr int NB = DP / 16;
  // unpadded DP <= 64: the residual's MFMA A operands (P[c][k], read as the symmetric P[k][c]) live
  // in registers for the whole launch: NB * DP / 4 floats per lane
  constexpr bool PREG = !PAD && !PLDS && DP <= 64;
  float preg[PREG ? NB * (DP / 4) : 1];
  if constexpr (PREG) {
#pragma unroll
    for (int jb = 0; jb < NB; ++jb)
#pragma unroll
      for (int ks = 0; ks < DP / 4; ++ks) preg[jb * (DP / 4) + ks] = Pm[(ks * 4 + (lane >> 4)) * DP + jb * 16 + (lane & 15)];
  }
  static_assert(P / 16 == 4, "one 16-pixel block per wave");
  // the a tile goes HBM -> registers one tile ahead (issued before the current tile's GEMMs),
  // then registers -> LDS at the top of its own iteration
  // (DP <= 64; at DP = 128 the 32 registers would cost a wave per SIMD)
  constexpr bool PFT = DP <= 64;
  constexpr int NPF = PFT ? DP * P / 256 : 1;
  const int ntiles = (H / RPT) * xt;
  float pf[NPF];
  auto fetch_tile = [&](int tile) {
    const int y0 = (tile / xt) * RPT, x0 = (tile % xt) * TW;
#pragma unroll
    for (int u = 0; u < (PFT ? NPF : 0); ++u) {
      const int i = tid + 256 * u, c = i / P, p = i % P;
      const bool ok = c < d;
      const float v = a_b[(ok ? c : 0) * HW + (y0 + p / TW) * W + x0 + p % TW];
      pf[u] = ok ? v : 0.f;
    }
  };
  if constexpr (PFT)
    if (blockIdx.x * PT < ntiles) fetch_tile(blockIdx.x * PT);
  for (int t = 0; t < PT; ++t) {
    const int tile = blockIdx.x * PT + t;
    if (tile >= ntiles) break;
    const int y0 = (tile / xt) * RPT, x0 = (tile % xt) * TW;
    __syncthreads();
    if constexpr (PFT) {
#pragma unroll
      for (int u = 0; u < NPF; ++u) {
        const int i = tid + 256 * u;
        as[(i / P) * PL + i % P] = pf[u];
      }
    } else {
      for (int i = tid; i < DP * P; i += 256) {
        const int c = i / P, p = i % P;
        const bool ok = c < d;
        const float v = a_b[(ok ? c : 0) * HW + (y0 + p / TW) * W + x0 + p % TW];
        as[c * PL + p] = ok ? v : 0.f;
      }
    }
    __syncthreads();
    if constexpr (PFT)
      if (t + 1 < PT && tile + 1 < ntiles) fetch_tile(tile + 1);
    // h[j][p] = sum_c U[c][j] a[c][p] and delta[c][p] = sum_k P[c][k] a[k][p]: wave w owns pixel
    // block w and runs the 2 NB output blocks as independent MFMA chains sharing the B operand read
    // (per element the single-chain k order); then a' = a + delta (= h U^T, residual form above)
    {
      f32x4 acc[NB], dl[NB];
#pragma unroll
      for (int jb = 0; jb < NB; ++jb) acc[jb] = dl[jb] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (PREG) {
#pragma unroll
        for (int k0 = 0; k0 < DP; k0 += 4) {
          const int c = k0 + (lane >> 4);
          const float bv = as[c * PL + w * 16 + (lane & 15)];
#pragma unroll
          for (int jb = 0; jb < NB; ++jb) {
            if constexpr (HOUT) acc[jb] = mfma16(Us[c * LD + jb * 16 + (lane & 15)], bv, acc[jb]);
            dl[jb] = mfma16(preg[jb * (DP / 4) + k0 / 4], bv, dl[jb]);
          }
        }
      } else {
#pragma unroll 2
        for (int k0 = 0; k0 < d4; k0 += 4) {
          const int c = k0 + (lane >> 4);
          const float bv = as[c * PL + w * 16 + (lane & 15)];
#pragma unroll
          for (int jb = 0; jb < NB; ++jb) {
            if constexpr (HOUT) acc[jb] = mfma16(Us[c * LD + jb * 16 + (lane & 15)], bv, acc[jb]);
            dl[jb] = mfma16(p_op<DP, PLDS>(Ps, Pm, d, jb * 16 + (lane & 15), c), bv, dl[jb]);
          }
        }
      }
      // every wave reads and writes only its own 16 pixel columns of the tile
#pragma unroll
      for (int jb = 0; jb < NB; ++jb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = jb * 16 + (lane >> 4) * 4 + r, p = w * 16 + (lane & 15);
          const int og = j * HW + (y0 + p / TW) * W + x0 + p % TW;
          if (HOUT && j < d) h_b[og] = acc[jb][r];
          const float v = as[j * PL + p] + dl[jb][r];
          as[j * PL + p] = v;   // a tile no longer needed: holds a' now
          if (ap_b && j < d) ap_b[og] = v;
        }
    }
    if (pool) {
      __syncthreads();
      const int H2 = H / 2, W2 = W / 2;
      const int CXN = TW / 2;
      for (int i = tid; i < d * 16; i += 256) {
        const int c = i / 16, cell = i % 16, cy = cell / CXN, cx = cell % CXN;
        const int p00 = (2 * cy) * TW + 2 * cx;
        const float v[4] = {as[c * PL + p00], as[c * PL + p00 + 1], as[c * PL + p00 + TW],
                            as[c * PL + p00 + TW + 1]};
        int am = 0;
        float m = v[0];
        for (int s4 = 1; s4 < 4; ++s4)
          if (v[s4] > m || (v[s4] != v[s4] && m == m)) { m = v[s4]; am = s4; }
        const int o = c * H2 * W2 + (y0 / 2 + cy) * W2 + x0 / 2 + cx;
        pooled[(size_t)b * d * H2 * W2 + o] = m;
        amax[(size_t)b * d * H2 * W2 + o] = (uint8_t)am;
      }
    }
  }
}

// ===========================================================================
// projection backward (per sample, fans out to K+1 relevance clones):
//   R_a'  = pool-backward(gp, argmax)               (or dense R when no pool follows)
//   g1    = R_a' / stab(a', eps_proj)               Epsilon on invprojection
//   R_h   = h (.) (g1 U)
//   g2    = R_h / stab(h, eps_proj)                  Epsilon on projection (after the mask)
//   clone 0: v = g2 U^T ; clone k: v = g2[block k-1] U[:, block k-1]^T   (SubspaceHook mask)
//   G_q   = [a > 0] (a (.) v) / stab(den, eps_den)   ReLU-backward + the conv rule's division below
// Tiles of 64 pixels (RPT rows x TW cols), lanes = pixels; one tile per workgroup.
// ===========================================================================
#ifndef DRSA_PT_BWD
#define DRSA_PT_BWD 1
#endif
constexpr int PT_BWD = DRSA_PT_BWD;   // tiles per workgroup (backward)
#ifndef PROJ_STAGE_UNROLL
#define PROJ_STAGE_UNROLL 1
#endif
#ifndef PROJ_CLONE_UNROLL
#define PROJ_CLONE_UNROLL 1
#endif

template <int DP, bool PAD>
__global__ __launch_bounds__(256) void projection_bwd_kernel(
    const float* __restrict__ gp, const uint8_t* __restrict__ amax, const float* __restrict__ ap,
    const float* __restrict__ h, const float* __restrict__ a, const float* __restrict__ den,
    const float* __restrict__ U, float* __restrict__ G, int d_in, int H, int W, int K, float eps_proj, float eps_den,
    int sparse, int has_den, int fanout) {
  const int d = PAD ? d_in : DP;
  constexpr int P = 64, LD = DP + 1, PL = P + 4;
  constexpr int NB = DP / 16, TILES = NB * (P / 16), QW = TILES / 4;   // 16x16 blocks; per wave
  // Per wave: pixel block pb = wave, channel blocks cb = 0..NB-1 (q = wave + 4 i).  Its h, a,
  // den values (MFMA output layout) are prefetched at the start, with the staging loads.
  // Rows c >= d (padded embedding) are zero in U and g1 and never stored.
  constexpr bool PF = DP <= 64;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Us = sm;               // [DP][LD]
  float* g1 = Us + DP * LD;     // [DP][PL]
  float* g2 = g1 + DP * PL;     // [DP][PL]
  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  const int b = blockIdx.y;
  const int TW = W < 32 ? W : 32, RPT = P / TW;
  const int HW = H * W, xt = W / TW;
  const int dk = d / K, d4 = (d + 3) & ~3;
  // fanout 1: K+1 clones (standard + K subspaces); 2: the K subspace clones only; 0: replicated rows
  const int nq = fanout == 1 ? (K + 1) : fanout == 2 ? K : 1;
  for (int t = 0; t < PT_BWD; ++t) {
    const int tile = blockIdx.x * PT_BWD + t;
    if (tile >= (H / RPT) * xt) break;
    const int y0 = (tile / xt) * RPT, x0 = (tile % xt) * TW;
    // this lane's pixel in its wave's 16-pixel block, and the channel rows it owns
    const int pl = w * 16 + (lane & 15);
    const size_t pixl = (size_t)(y0 + pl / TW) * W + x0 + pl % TW;
    float hv[PF ? QW * 4 : 1], av[PF ? QW * 4 : 1], dv[PF ? QW * 4 : 1];
    if constexpr (PF) {
#pragma unroll
      for (int i = 0; i < QW; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = i * 16 + (lane >> 4) * 4 + r;
          const bool ok = c < d;
          const size_t os = ((size_t)b * d + (ok ? c : 0)) * HW + pixl;
          const float hh = h[os], aa = a[os], dd = has_den ? den[os] : 1.f;
          hv[i * 4 + r] = ok ? hh : 0.f;
          av[i * 4 + r] = ok ? aa : 0.f;
          dv[i * 4 + r] = dd;
        }
    }
    __syncthreads();
    if (t == 0) stage_u_padded<DP>(Us, U, d, tid);
#pragma unroll PROJ_STAGE_UNROLL
    for (int i = tid; i < DP * P; i += 256) {
      const int c = i / P, p = i % P;
      const int y = y0 + p / TW, x = x0 + p % TW;
      const bool ok = c < d;
      const int cc = ok ? c : 0;
      float R;
      if (sparse) {
        const int H2 = H / 2, W2 = W / 2;
        const size_t q = ((size_t)b * d + cc) * H2 * W2 + (y >> 1) * W2 + (x >> 1);
        const float gv = gp[q];
        R = (amax[q] == (((y & 1) << 1) | (x & 1))) ? gv : 0.f;
      } else {
        R = gp[((size_t)b * d + cc) * HW + y * W + x];
      }
      const float v = R / stab(ap[((size_t)b * d + cc) * HW + y * W + x], eps_proj);
      g1[c * PL + p] = ok ? v : 0.f;
    }
    __syncthreads();
    // t[j][p] = sum_c U[c][j] g1[c][p];  R_h = h (.) t;  g2 = R_h / stab(h)
#pragma unroll
    for (int i = 0; i < QW; ++i) {
      const int jb = i, pb = w;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int k0 = 0; k0 < d4; k0 += 4) {
        const int c = k0 + (lane >> 4);
        acc = mfma16(Us[c * LD + jb * 16 + (lane & 15)], g1[c * PL + pb * 16 + (lane & 15)], acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = jb * 16 + (lane >> 4) * 4 + r, p = pb * 16 + (lane & 15);
        float hx;
        if constexpr (PF) {
          hx = hv[i * 4 + r];
        } else {
          const float hh = h[((size_t)b * d + (j < d ? j : 0)) * HW + pixl];
          hx = j < d ? hh : 0.f;
        }
        const float Rh = hx * acc[r];
        g2[j * PL + p] = Rh / stab(hx, eps_proj);
      }
    }
    __syncthreads();
#ifndef DRSA_PROJ_DBG
#define DRSA_PROJ_DBG 0
#endif
    for (int qi = 0; qi < ((DRSA_PROJ_DBG & 2) ? 0 : nq); ++qi) {   // ablation bit 2: no clone stage
      const int q = fanout == 1 ? qi : fanout == 2 ? qi + 1 : b % (K + 1);
      const int j0 = q == 0 ? 0 : (q - 1) * dk, j1 = q == 0 ? d : q * dk;
      const size_t orow = fanout ? (size_t)b * nq + qi : (size_t)b;
#pragma unroll
      for (int i = 0; i < QW; ++i) {
        const int cb = i, pb = w;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll PROJ_CLONE_UNROLL
        for (int k0 = j0; k0 < j1; k0 += 4) {
          const int j = k0 + (lane >> 4);
          const bool ok = j < j1;
          const float ua = ok ? Us[(cb * 16 + (lane & 15)) * LD + j] : 0.f;
          const float gb = ok ? g2[j * PL + pb * 16 + (lane & 15)] : 0.f;
          acc = mfma16(ua, gb, acc);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = cb * 16 + (lane >> 4) * 4 + r;
          const bool cok = c < d;
          const size_t os = ((size_t)b * d + (cok ? c : 0)) * HW + pixl;
          float ax, dx;
          if constexpr (PF) { ax = av[i * 4 + r]; dx = dv[i * 4 + r]; }
          else { ax = a[os]; dx = has_den ? den[os] : 1.f; }
          const float Rv = ax * acc[r];
          float gq;
          if (has_den) {
            const float qd = div_nb(Rv, stab(dx, eps_den));   // every lane, then the select
            gq = (ax > 0.f) ? qd : 0.f;
          } else {
            gq = (ax > 0.f) ? Rv : 0.f;
          }
#if DRSA_PROJ_DBG & 1
          if (cok && gq == 12345.f) G[(orow * d + c) * HW + pixl] = gq;   // ablation: no G stores
#else
          if (cok) G[(orow * d + c) * HW + pixl] = gq;
#endif
        }
      }
    }
  }
}

// ===========================================================================
// projection backward with h and a' recomputed from a (no h / a' buffers in HBM: the forward
// then writes only the pooled a' and its argmax).  Same math and the same MFMA operand order
// as projection_fwd_kernel (h, a') and projection_bwd_kernel (t, clones), so every value is
// bit-identical to the stored-buffer path.  Each wave owns one 16-pixel block of the 64-pixel
// tile end to end, so after U is staged no workgroup barrier is needed:
//   region A [DP][16]: a, then g1;  region B [DP][16]: h, then g2   (wave-private LDS)
// ===========================================================================
#ifndef DRSA_PT_RC
#define DRSA_PT_RC 2
#endif
constexpr int PT_RC = DRSA_PT_RC;   // tiles per workgroup (U staged once)
#ifndef DRSA_PROJ_RC_WPE
#define DRSA_PROJ_RC_WPE 3
#endif

template <int DP, bool PAD, bool PLDS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DP <= 64 ? DRSA_PROJ_RC_WPE : 1))) void projection_bwd_rc_kernel(
    const float* __restrict__ gp, const uint8_t* __restrict__ amax, const float* __restrict__ a,
    const float* __restrict__ den, const float* __restrict__ U, const float* __restrict__ Pm, float* __restrict__ G,
    int d_in, int H, int W, int K, float eps_proj, float eps_den, int sparse, int has_den, int fanout) {
  const int d = PAD ? d_in : DP;
  constexpr int P = 64, LD = DP + 1, PW = 16, NB = DP / 16;
  constexpr bool PF = DP <= 64;   // keep a / den of the output rows in registers
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  float* Us = sm;                                   // [DP][LD]
  float* RA = Us + DP * LD + w * 2 * DP * PW;       // [DP][PW]
  float* RB = RA + DP * PW;                         // [DP][PW]
  float* Ps = Us + DP * LD + 4 * 2 * DP * PW;       // [DP][DP + 16] P (when PLDS)
  const int b = blockIdx.y;
  const int TW = W < 32 ? W : 32, RPT = P / TW;
  const int HW = H * W, xt = W / TW, H2 = H / 2, W2 = W / 2;
  // per-sample bases (uniform, 64-bit) + 32-bit per-lane offsets: saddr + voffset addressing
  // instead of a 64-bit multiply-add per element (the host keeps d * H * W < 2^31)
  const float* __restrict__ a_b = a + (size_t)b * d * HW;
  const float* __restrict__ den_b = has_den ? den + (size_t)b * d * HW : a_b;
  const float* __restrict__ gp_b = gp + (size_t)b * d * (sparse ? H2 * W2 : HW);
  const uint8_t* __restrict__ am_b = sparse ? amax + (size_t)b * d * H2 * W2 : nullptr;
  const int dk = d / K, d4 = (d + 3) & ~3;
  // fanout 1: K+1 clones (standard + K subspaces); 2: the K subspace clones only; 0: replicated rows
  const int nq = fanout == 1 ? (K + 1) : fanout == 2 ? K : 1;
  const int pc = lane & 15, rg = lane >> 4;         // pixel column / row group of the MFMA layouts
  stage_u_padded<DP>(Us, U, d, tid);
  if constexpr (PLDS) stage_p<DP>(Ps, Pm, d, tid);
  __syncthreads();
  for (int t = 0; t < PT_RC; ++t) {
    const int tile = blockIdx.x * PT_RC + t;
    if (tile >= (H / RPT) * xt) break;
    const int y0 = (tile / xt) * RPT, x0 = (tile % xt) * TW;
    const int pl = w * 16 + pc;
    const int py = y0 + pl / TW, px = x0 + pl % TW;
    const int pixl = py * W + px;
    const int cell = (py >> 1) * W2 + (px >> 1);
    // a (and den) at rows c = i*16 + 4 rg + r: the output layout of every GEMM below
    float av[NB * 4], dv[PF ? NB * 4 : 1];
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = i * 16 + rg * 4 + r;
        const bool ok = c < d;
        const int os = (ok ? c : 0) * HW + pixl;
        const float aa = a_b[os];
        av[i * 4 + r] = ok ? aa : 0.f;
        if constexpr (PF) dv[i * 4 + r] = has_den ? den_b[os] : 1.f;
      }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < NB * 4; ++i) RA[(((i >> 2) * 16) + rg * 4 + (i & 3)) * PW + pc] = av[i];
    __builtin_amdgcn_wave_barrier();
    // Every GEMM below runs its NB output blocks as independent MFMA chains that share the B
    // operand read (per element the k order is the single-chain order of the stored path).
    // h[j][p] = sum_c U[c][j] a[c][p]        (projection_fwd_kernel order)
    {
      f32x4 acc[NB];
#pragma unroll
      for (int jb = 0; jb < NB; ++jb) acc[jb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
      for (int k0 = 0; k0 < d4; k0 += 4) {
        const int c = k0 + rg;
        const float bv = RA[c * PW + pc];
#pragma unroll
        for (int jb = 0; jb < NB; ++jb) acc[jb] = mfma16(Us[c * LD + jb * 16 + pc], bv, acc[jb]);
      }
#pragma unroll
      for (int jb = 0; jb < NB; ++jb)
#pragma unroll
        for (int r = 0; r < 4; ++r) RB[(jb * 16 + rg * 4 + r) * PW + pc] = acc[jb][r];
    }
    __builtin_amdgcn_wave_barrier();
    // a'[c][p] = a[c][p] + sum_k P[c][k] a[k][p]   (projection_fwd_kernel order; a separate pass:
    // folded into the h GEMM above, the second accumulator set spills at 3 waves/SIMD);
    // g1 = R_a' / stab(a')  -> region A (in place of a; a stays in registers)
    {
      f32x4 acc[NB];
#pragma unroll
      for (int cb = 0; cb < NB; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
      for (int k0 = 0; k0 < d4; k0 += 4) {
        const int k = k0 + rg;
        const float bv = RA[k * PW + pc];
#pragma unroll
        for (int cb = 0; cb < NB; ++cb) acc[cb] = mfma16(p_op<DP, PLDS>(Ps, Pm, d, cb * 16 + pc, k), bv, acc[cb]);
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int cb = 0; cb < NB; ++cb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = cb * 16 + rg * 4 + r;
          const bool ok = c < d;
          const int cc = ok ? c : 0;
          float R;
          if (sparse) {
            const int q = cc * H2 * W2 + cell;
            const float gv = gp_b[q];   // unconditional load, then the argmax select
            R = (am_b[q] == (((py & 1) << 1) | (px & 1))) ? gv : 0.f;
          } else {
            R = gp_b[cc * HW + pixl];
          }
          const float apv = av[cb * 4 + r] + acc[cb][r];
          const float v = R / stab(apv, eps_proj);
          RA[c * PW + pc] = ok ? v : 0.f;
        }
    }
    __builtin_amdgcn_wave_barrier();
    // t[j][p] = sum_c U[c][j] g1[c][p];  g2 = h (.) t / stab(h)  -> region B (in place of h)
    {
      f32x4 acc[NB];
#pragma unroll
      for (int jb = 0; jb < NB; ++jb) acc[jb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
      for (int k0 = 0; k0 < d4; k0 += 4) {
        const int c = k0 + rg;
        const float bv = RA[c * PW + pc];
#pragma unroll
        for (int jb = 0; jb < NB; ++jb) acc[jb] = mfma16(Us[c * LD + jb * 16 + pc], bv, acc[jb]);
      }
#pragma unroll
      for (int jb = 0; jb < NB; ++jb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float* e = RB + (jb * 16 + rg * 4 + r) * PW + pc;   // this lane's own h element
          const float hx = *e;
          *e = (hx * acc[jb][r]) / stab(hx, eps_proj);
        }
    }
    __builtin_amdgcn_wave_barrier();
#ifndef DRSA_PROJ_DBG
#define DRSA_PROJ_DBG 0
#endif
    // the clones share a and den: stabilise the denominators once per tile (without den the
    // quotient is x / 1 = x exactly), so the clone epilogue below is branch-free
    if constexpr (PF) {
#pragma unroll
      for (int i = 0; i < NB * 4; ++i) dv[i] = has_den ? stab(dv[i], eps_den) : 1.f;
    }
    for (int qi = 0; qi < ((DRSA_PROJ_DBG & 2) ? 0 : nq); ++qi) {   // ablation bit 2: no clone stage
      const int q = fanout == 1 ? qi : fanout == 2 ? qi + 1 : b % (K + 1);
      const int j0 = q == 0 ? 0 : (q - 1) * dk, j1 = q == 0 ? d : q * dk;
      const size_t orow = fanout ? (size_t)b * nq + qi : (size_t)b;
      float* __restrict__ G_q = G + orow * d * HW;
      f32x4 acc[NB];
#pragma unroll
      for (int cb = 0; cb < NB; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
      // operands read unconditionally from an in-range row and zeroed afterwards: one LDS round
      // trip per k-step instead of an exec branch and a wait per read
      if (j1 - j0 == 16) {
        // d_k = 16 (GTZAN j = 7: d = 64, K = 4): all four k-steps' operands in one round trip
        float g0[4], u0[4][NB];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int j = j0 + 4 * s + rg;
          g0[s] = RB[j * PW + pc];
#pragma unroll
          for (int cb = 0; cb < NB; ++cb) u0[s][cb] = Us[(cb * 16 + pc) * LD + j];
        }
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int cb = 0; cb < NB; ++cb) acc[cb] = mfma16(u0[s][cb], g0[s], acc[cb]);
      } else
#pragma unroll 2
      for (int k0 = j0; k0 < j1; k0 += 4) {
        const int j = k0 + rg;
        const bool ok = j < j1;
        const int jc = ok ? j : j0;
        const float g0 = RB[jc * PW + pc];
        float u0[NB];
#pragma unroll
        for (int cb = 0; cb < NB; ++cb) u0[cb] = Us[(cb * 16 + pc) * LD + jc];
        const float gb = ok ? g0 : 0.f;
#pragma unroll
        for (int cb = 0; cb < NB; ++cb) acc[cb] = mfma16(ok ? u0[cb] : 0.f, gb, acc[cb]);
      }
#pragma unroll
      for (int cb = 0; cb < NB; ++cb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = cb * 16 + rg * 4 + r;
          const bool cok = c < d;
          const int os = (cok ? c : 0) * HW + pixl;
          const float ax = av[cb * 4 + r];
          float sd;
          if constexpr (PF) {
            sd = dv[cb * 4 + r];
          } else {
            const float dx = den_b[os];   // den_b is a valid row (a) without den
            sd = has_den ? stab(dx, eps_den) : 1.f;
          }
          const float qd = div_nb(ax * acc[cb][r], sd);   // every lane, then the select
          const float gq = (ax > 0.f) ? qd : 0.f;
#if DRSA_PROJ_DBG & 1
          if (cok && gq == 12345.f) G_q[c * HW + pixl] = gq;   // ablation: no G stores
#else
          if (cok) G_q[c * HW + pixl] = gq;
#endif
        }
    }
  }
}

// ===========================================================================
// first layer backward (WSquare / Flat, one input channel):
//   R[y][x] = sum_co sum_{dy,dx} G[co][y+dy][x+dx] * W2[co][1-dy][1-dx]
//   G from pool-sparse (gp, argmax) or dense; 16 x 64 output tile, 4 pixels per thread
// ===========================================================================
#ifndef DRSA_FL_TH
#define DRSA_FL_TH 16
#endif
#ifndef DRSA_FL_CC
#define DRSA_FL_CC 4
#endif
constexpr int FL_TH = DRSA_FL_TH, FL_TW = 64, FL_CC = DRSA_FL_CC;
constexpr int FL_HY = FL_TH + 2, FL_RS = FL_TW + 8;           // LDS row: halo col 3, interior 4..67, halo 68
constexpr int FL_ROWS = FL_CC * FL_HY;                        // staged rows per channel group
constexpr int FL_NV4 = FL_ROWS * (FL_TW / 4);                 // interior float4 per group
constexpr int FL_IV = (FL_NV4 + 255) / 256, FL_IH = (FL_ROWS * 2 + 255) / 256;

// Each thread owns 4 adjacent output pixels of one row.  A channel group's g tile (+1 halo) is
// loaded as coalesced float4 rows (all of a thread's loads issued back to back into registers, the
// next group's while the current one is consumed), then written to LDS; the chain per output pixel
// is (channel, dy, dx), the order of oracle/lrp_exact.c and of the pooled kernel below.
template <bool VEC>
__global__ __launch_bounds__(256) void first_layer_bwd_kernel(const float* __restrict__ g, const float* __restrict__ w2,
                                                              float* __restrict__ out, int C, int H, int W) {
  __shared__ __attribute__((aligned(16))) float hal[FL_CC][FL_HY][FL_RS];
  const int tid = threadIdx.x;
  const int tiles_x = (W + FL_TW - 1) / FL_TW;
  const int ty0 = (blockIdx.x / tiles_x) * FL_TH, tx0 = (blockIdx.x % tiles_x) * FL_TW;
  const int bq = blockIdx.y;
  const int ly = tid / 16, lx = (tid % 16) * 4;   // 16 rows x 16 threads, 4 px each
  const size_t plane = (size_t)H * W;
  const int iplane = H * W;   // 32-bit per-lane offsets from the per-sample base (C * H * W < 2^31)
  const float* gb = g + (size_t)bq * C * plane;
  float4 rv[FL_IV];
  float rh[FL_IH];
  // loads from clamped (always valid) addresses, masked afterwards
  auto fetch = [&](int c0) {
#pragma unroll
    for (int it = 0; it < FL_IV; ++it) {
      const int i = tid + it * 256;
      const int row = i / (FL_TW / 4), q = i % (FL_TW / 4);
      const int ci = row / FL_HY, hy = row % FL_HY;
      const int gy = ty0 - 1 + hy, gx = tx0 + 4 * q, c = c0 + ci;
      const bool rok = i < FL_NV4 && c < C && gy >= 0 && gy < H;
      if constexpr (VEC) {
        const bool ok = rok && gx < W;
        const float4 v = *reinterpret_cast<const float4*>(gb + (ok ? c * iplane + gy * W + gx : 0));
        rv[it] = ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        float e[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const bool ok = rok && gx + k < W;
          const float v = gb[ok ? c * iplane + gy * W + gx + k : 0];
          e[k] = ok ? v : 0.f;
        }
        rv[it] = make_float4(e[0], e[1], e[2], e[3]);
      }
    }
#pragma unroll
    for (int it = 0; it < FL_IH; ++it) {
      const int i = tid + it * 256;
      const int row = i >> 1, side = i & 1;
      const int ci = row / FL_HY, hy = row % FL_HY;
      const int gy = ty0 - 1 + hy, gx = side ? tx0 + FL_TW : tx0 - 1, c = c0 + ci;
      const bool ok = i < FL_ROWS * 2 && c < C && gy >= 0 && gy < H && gx >= 0 && gx < W;
      const float v = gb[ok ? c * iplane + gy * W + gx : 0];
      rh[it] = ok ? v : 0.f;
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int it = 0; it < FL_IV; ++it) {
      const int i = tid + it * 256;
      if (i < FL_NV4) {
        const int row = i / (FL_TW / 4), q = i % (FL_TW / 4);
        *reinterpret_cast<float4*>(&hal[row / FL_HY][row % FL_HY][4 + 4 * q]) = rv[it];
      }
    }
#pragma unroll
    for (int it = 0; it < FL_IH; ++it) {
      const int i = tid + it * 256;
      if (i < FL_ROWS * 2) {
        const int row = i >> 1, side = i & 1;
        hal[row / FL_HY][row % FL_HY][side ? 4 + FL_TW : 3] = rh[it];
      }
    }
  };
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  fetch(0);
  for (int c0 = 0; c0 < C; c0 += FL_CC) {
    __syncthreads();
    stage();
    __syncthreads();
    if (c0 + FL_CC < C) fetch(c0 + FL_CC);
#pragma unroll 2
    for (int ci = 0; ci < FL_CC; ++ci) {
      // channels past C were staged as zeros: fma(0, w, acc) == acc, so any finite weight will do
      const int c = min(c0 + ci, C - 1);
      float wv[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) wv[t] = w2[c * 9 + t];
#pragma unroll
      for (int dy = -1; dy <= 1; ++dy) {
        const float* r = &hal[ci][ly + 1 + dy][3 + lx];      // pixel tx0 + lx - 1 ..
        const float4 m = *reinterpret_cast<const float4*>(r + 1);
        const float row[6] = {r[0], m.x, m.y, m.z, m.w, r[5]};
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
          const float wt = wv[(1 - dy) * 3 + (1 - dx)];
#pragma unroll
          for (int p = 0; p < 4; ++p) acc[p] = fmaf(row[p + 1 + dx], wt, acc[p]);
        }
      }
    }
  }
  const int y = ty0 + ly;
  if (y < H) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int x = tx0 + lx + p;
      if (x < W) out[((size_t)bq * H + y) * W + x] = acc[p];
    }
  }
}

// Pool-sparse variant (the VGG case: conv0 -> ReLU -> MaxPool2d(2)).  A workgroup covers
// 16 x 64 pool cells (32 x 128 output pixels); each thread owns 2 x 2 cells = a 4 x 4 pixel
// block.  Per group of FQ_C channels the cells of the tile (+1 halo) are expanded to pixels
// while staging (value at the argmax position, zeros elsewhere) into an image with origin
// pixel (2qy0-2, 2qx0-2) at column 1 (so that even pixel pairs of a thread's patch are 8-byte
// aligned); the next group's cells are prefetched (branch-free, clamped addresses) into
// registers while the current group is consumed.  Every thread reads its 6 x 6 patch per
// channel as five pixel pairs per row and runs packed fmas (v_pk_fma_f32: two output pixels
// per instruction) in the dense chain order (channel, dy, dx) — the chain of the dense kernel
// above and of oracle/lrp_exact.c (the zero terms included: fma(0, w, acc) == acc).
#ifndef DRSA_FQ_C
#define DRSA_FQ_C 1
#endif
// 1: two channel groups of loads in flight (two register sets; 106 VGPRs, 4 waves/SIMD, or spills
// at 6: the single set at 8 waves/SIMD keeps as many bytes in flight)
#ifndef DRSA_FQ_DEPTH2
#define DRSA_FQ_DEPTH2 0
#endif
#define FQ_DEPTH2 DRSA_FQ_DEPTH2
#ifndef DRSA_FQ_WPE
#define DRSA_FQ_WPE 8
#endif
// 1: cells staged through range-checked buffer loads into a pixel image that keeps its zeros
#ifndef DRSA_FQ_INC
#define DRSA_FQ_INC 1
#endif
// 1: the 6 x 6 patch streamed row by row (one row of pairs live: fewer VGPRs, more waves)
#ifndef DRSA_FQ_STREAM
#define DRSA_FQ_STREAM 1
#endif
constexpr int FQ_Y = 16, FQ_X = 64, FQ_C = DRSA_FQ_C;
constexpr int FQ_RY = FQ_Y + 2, FQ_RX = FQ_X + 2;            // cells incl. halo
constexpr int FQ_PY = 2 * FQ_RY, FQ_PX = 2 * FQ_RX + 4;      // pixel image (row pad 4)
constexpr int FQ_KR = (FQ_RY + 3) / 4;                       // row passes of 4 waves
// image column of the halo origin: 3 puts every thread's 6-pixel window (starting at 4tx + 4) on
// a 16-byte boundary, so a row of it is one ds_read_b128 + one ds_read_b64 over consecutive lanes
// (bank-conflict free; the former origin 1 gave 8-byte reads at a 16-byte lane stride)
constexpr int FQ_C0 = 3;
constexpr int FQ_NS = FQ_C * FQ_KR + 1;                      // staged cells per thread

typedef float fq2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void fq_put(float* img, int ci, int ry, int rx, float v, int sb) {
  float* d = img + (ci * FQ_PY + 2 * ry) * FQ_PX + 2 * rx + FQ_C0;
  d[0] = sb == 0 ? v : 0.f;
  d[1] = sb == 1 ? v : 0.f;
  d[FQ_PX] = sb == 2 ? v : 0.f;
  d[FQ_PX + 1] = sb == 3 ? v : 0.f;
}

// W2C > 0: the pooled width as a compile-time constant (GTZAN: 64), so the per-k row offsets of the
// staging loads are instruction immediates instead of adds
template <int W2C>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DRSA_FQ_WPE))) void first_layer_bwd_pooled_kernel(const float* __restrict__ g,
                                                                     const uint8_t* __restrict__ amax,
                                                                     const float* __restrict__ w2,
                                                                     float* __restrict__ out, int C, int H, int W,
                                                                     int clones) {
  extern __shared__ __attribute__((aligned(16))) float img[];    // [FQ_C][FQ_PY][FQ_PX]
  const int tid = threadIdx.x, lane = tid & 63, wv4 = tid >> 6;
  const int H2 = H / 2, W2 = W2C > 0 ? W2C : W / 2;
  const int tiles_x = (W2 + FQ_X - 1) / FQ_X;
  const int qy0 = (blockIdx.x / tiles_x) * FQ_Y, qx0 = (blockIdx.x % tiles_x) * FQ_X;
  const int bq = blockIdx.y, bs = bq / clones;
  const int ty = tid / (FQ_X / 2), tx = tid % (FQ_X / 2);      // 8 x 32 threads, 2x2 cells each
  const size_t plane = (size_t)H2 * W2;
  const int iplane = H2 * W2;
  const float* gb = g + (size_t)bq * C * plane;
  const uint8_t* ab = amax + (size_t)bs * C * plane;
  // staging map: interior columns rx = 1 + lane, rows ry = wave + 4k; the two halo columns
  // (rx = 0, 65) of all rows and channels by threads tid < 2 * FQ_RY * FQ_C
  const int hci = tid / (2 * FQ_RY), hr = tid % (2 * FQ_RY);
  const int hry = hr >> 1, hrx = (hr & 1) ? FQ_RX - 1 : 0;
  const bool hact = tid < 2 * FQ_RY * FQ_C;
  float v[FQ_NS], v2[FQ_DEPTH2 ? FQ_NS : 1];
  int sb[FQ_NS], sb2[FQ_DEPTH2 ? FQ_NS : 1];
  // loads are unconditional from a clamped (always valid) address and masked afterwards
  auto fetch = [&](int c0, auto& v, auto& sb) {
    const int cx = qx0 + lane;
#pragma unroll
    for (int ci = 0; ci < FQ_C; ++ci)
#pragma unroll
      for (int k = 0; k < FQ_KR; ++k) {
        const int ry = wv4 + 4 * k, cy = qy0 - 1 + ry, c = c0 + ci;
        const bool ok = ry < FQ_RY && c < C && cy >= 0 && cy < H2 && cx < W2;
        const unsigned o = ok ? c * iplane + cy * W2 + cx : 0;   // unsigned 32-bit offsets: saddr + voffset loads
        v[ci * FQ_KR + k] = gb[o];
        sb[ci * FQ_KR + k] = (int)ab[o];
      }
    {
      const int c = c0 + hci, cy = qy0 - 1 + hry, cxh = qx0 - 1 + hrx;
      const bool ok = hact && c < C && cy >= 0 && cy < H2 && cxh >= 0 && cxh < W2;
      const unsigned o = ok ? c * iplane + cy * W2 + cxh : 0;
      v[FQ_NS - 1] = gb[o];
      sb[FQ_NS - 1] = (int)ab[o];
    }
  };
  // the masks are re-evaluated here rather than kept live from the loads: a cell outside the
  // image / channel range gets argmax 4, i.e. zeros at all four pixels
  auto stage = [&](int c0, auto& v, auto& sb) {
    const int cx = qx0 + lane;
#pragma unroll
    for (int ci = 0; ci < FQ_C; ++ci)
#pragma unroll
      for (int k = 0; k < FQ_KR; ++k) {
        const int ry = wv4 + 4 * k, cy = qy0 - 1 + ry, c = c0 + ci;
        const bool ok = ry < FQ_RY && c < C && cy >= 0 && cy < H2 && cx < W2;
        if (ry < FQ_RY) fq_put(img, ci, ry, 1 + lane, v[ci * FQ_KR + k], ok ? sb[ci * FQ_KR + k] : 4);
      }
    {
      const int c = c0 + hci, cy = qy0 - 1 + hry, cxh = qx0 - 1 + hrx;
      const bool ok = hact && c < C && cy >= 0 && cy < H2 && cxh >= 0 && cxh < W2;
      if (hact) fq_put(img, hci, hry, hrx, v[FQ_NS - 1], ok ? sb[FQ_NS - 1] : 4);
    }
  };
  fq2 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = fq2{0.f, 0.f};
  auto compute = [&](int c0) {
#pragma unroll
    for (int ci = 0; ci < FQ_C; ++ci) {
      const int c = c0 + ci;
      float wv[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) wv[t] = (c < C) ? w2[c * 9 + t] : 0.f;
      // patch P[i][j] = pixel (2qy0 + 4ty - 1 + i, 2qx0 + 4tx - 1 + j) = img[4ty + 1 + i][4tx + FQ_C0 + 1 + j];
      // pair q (q = 0..4) = (P[i][q], P[i][q + 1])
      const float* base = img + (ci * FQ_PY + 4 * ty + 1) * FQ_PX + 4 * tx + FQ_C0 + 1;
#if DRSA_FQ_STREAM
      // patch rows streamed: row i feeds output rows py = i - 1 - dy, i.e. each output row takes
      // its taps in dy order (then dx) -- the chain order -- with only one patch row live
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const float* r = base + i * FQ_PX;
        const float4 q4 = *reinterpret_cast<const float4*>(r);
        const fq2 q2 = *reinterpret_cast<const fq2*>(r + 4);
        const fq2 rp[5] = {fq2{q4.x, q4.y}, fq2{q4.y, q4.z}, fq2{q4.z, q4.w}, fq2{q4.w, q2.x}, q2};
#pragma unroll
        for (int py = 0; py < 4; ++py) {
          const int dy = i - py - 1;
          if (dy < -1 || dy > 1) continue;
#pragma unroll
          for (int dx = -1; dx <= 1; ++dx) {
            const float w = wv[(1 - dy) * 3 + (1 - dx)];
            const fq2 ww = fq2{w, w};
            acc[py][0] = __builtin_elementwise_fma(rp[1 + dx], ww, acc[py][0]);
            acc[py][1] = __builtin_elementwise_fma(rp[3 + dx], ww, acc[py][1]);
          }
        }
      }
#else
      fq2 pr[6][5];
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const float* r = base + i * FQ_PX;
        const float4 q4 = *reinterpret_cast<const float4*>(r);
        const fq2 q2 = *reinterpret_cast<const fq2*>(r + 4);
        pr[i][0] = fq2{q4.x, q4.y};
        pr[i][1] = fq2{q4.y, q4.z};
        pr[i][2] = fq2{q4.z, q4.w};
        pr[i][3] = fq2{q4.w, q2.x};
        pr[i][4] = q2;
      }
#pragma unroll
      for (int py = 0; py < 4; ++py)
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
          for (int dx = -1; dx <= 1; ++dx) {
            const float w = wv[(1 - dy) * 3 + (1 - dx)];
            const fq2 ww = fq2{w, w};
            acc[py][0] = __builtin_elementwise_fma(pr[py + 1 + dy][1 + dx], ww, acc[py][0]);
            acc[py][1] = __builtin_elementwise_fma(pr[py + 1 + dy][3 + dx], ww, acc[py][1]);
          }
#endif
    }
  };
#if FQ_DEPTH2
  // two register sets: channel group c + 2 is in flight while c is computed (c + 1 already landed)
  fetch(0, v, sb);
  if (FQ_C < C) fetch(FQ_C, v2, sb2);
  for (int c0 = 0; c0 < C; c0 += 2 * FQ_C) {
    __syncthreads();
    stage(c0, v, sb);
    __syncthreads();
    if (c0 + 2 * FQ_C < C) fetch(c0 + 2 * FQ_C, v, sb);
    compute(c0);
    if (c0 + FQ_C >= C) break;
    __syncthreads();
    stage(c0 + FQ_C, v2, sb2);
    __syncthreads();
    if (c0 + 3 * FQ_C < C) fetch(c0 + 3 * FQ_C, v2, sb2);
    compute(c0 + FQ_C);
  }
#elif DRSA_FQ_INC
  static_assert(FQ_C == 1, "incremental staging: one channel per group");
  // Cells through buffer loads: a per-channel descriptor (uniform) over the channel's plane, so a
  // cell above / below the image reads 0 (value and argmax byte) by the hardware range check, and
  // a cell left / right of it is pushed out of range by its lane offset; the per-k lane offsets
  // are one base + k rows.  The pixel image keeps its zeros between channels: each staged cell
  // clears the one pixel it set for the previous channel and sets the argmax pixel of this one
  // (LDS writes of a lane land in order), 3 VALU per cell instead of 4 compares + 4 selects.
  const int cxl = qx0 + lane;
  const unsigned OOR = 0x80000000u;   // >= any plane's byte size: the range check returns 0
  const unsigned lane_off = cxl < W2 ? (unsigned)(((qy0 - 1 + wv4) * W2 + cxl) * 4) : OOR;
  const int cxh = qx0 - 1 + hrx;
  const unsigned halo_off =
      (hact && cxh >= 0 && cxh < W2) ? (unsigned)(((qy0 - 1 + hry) * W2 + cxh) * 4) : OOR;
  const unsigned row4 = (unsigned)(4 * 4 * W2);   // 4 cell rows in bytes
  const unsigned pbytes = (unsigned)(iplane * 4);
  float vi[FQ_NS];
  unsigned si[FQ_NS];
  auto fetch_b = [&](int c) {
    // re-derive the per-k offsets every channel (5 adds) instead of holding 10 of them live
    unsigned lo = lane_off, ho = halo_off;
    asm volatile("" : "+v"(lo), "+v"(ho));
    // row k = 0 may lie above the image (a negative offset, out of range as unsigned); rows k >= 1
    // hang off a base that is never negative, so their offsets add as instruction immediates (the
    // hardware sums voffset + immediate without a 32-bit wrap)
    const unsigned lo1 = lo + row4;
    const unsigned la0 = lo >> 2, la1 = lo1 >> 2;   // the argmax plane's (byte) offsets are the cell indices
    const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(gb + (size_t)c * plane), 0, (int)pbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(ab + (size_t)c * plane), 0, (int)(pbytes / 4), 0x00020000);
#pragma unroll
    for (int k = 0; k < FQ_KR; ++k) {
      // stays >= 2^31 (2^29 for the argmax plane) when lane_off is OOR
      const unsigned og = k == 0 ? lo : lo1 + (unsigned)(k - 1) * row4;
      const unsigned oa = k == 0 ? la0 : la1 + (unsigned)(k - 1) * (row4 / 4);
      vi[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rg, og, 0, 0));
      si[k] = __builtin_amdgcn_raw_buffer_load_b8(ra, oa, 0, 0);
    }
    vi[FQ_NS - 1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rg, ho, 0, 0));
    si[FQ_NS - 1] = __builtin_amdgcn_raw_buffer_load_b8(ra, ho >> 2, 0, 0);
  };
  // LDS byte address of each staged cell's top-left pixel and of the pixel set last channel
  typedef __attribute__((address_space(3))) char lds_char;
  typedef __attribute__((address_space(3))) float lds_float;
  lds_char* const imgb = (lds_char*)img;
  int cell0[FQ_NS];
  lds_float* prev[FQ_NS];
#pragma unroll
  for (int k = 0; k < FQ_KR; ++k) cell0[k] = 4 * (2 * (wv4 + 4 * k) * FQ_PX + 2 * (1 + lane) + FQ_C0);
  cell0[FQ_NS - 1] = 4 * (2 * hry * FQ_PX + 2 * hrx + FQ_C0);
#pragma unroll
  for (int k = 0; k < FQ_NS; ++k) prev[k] = (lds_float*)(imgb + cell0[k]);
  auto act = [&](int k) { return k == FQ_NS - 1 ? hact : (wv4 + 4 * k < FQ_RY); };
  for (int i = tid; i < FQ_PY * FQ_PX; i += 256) img[i] = 0.f;
  fetch_b(0);
  for (int c0 = 0; c0 < C; ++c0) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < FQ_NS; ++k) {
      if (act(k)) {
        // argmax b = 2 row + col -> byte offset 4 col + 4 FQ_PX row = 4 b + (4 FQ_PX - 8) (b & 2)
        const int b = (int)(si[k] & 3u);
        lds_float* const nw = (lds_float*)(imgb + (cell0[k] + 4 * b + (4 * FQ_PX - 8) / 2 * (b & 2)));
        *prev[k] = 0.f;
        *nw = vi[k];
        prev[k] = nw;
      }
    }
    __syncthreads();
    if (c0 + 1 < C) fetch_b(c0 + 1);
    compute(c0);
  }
#else
  fetch(0, v, sb);
  for (int c0 = 0; c0 < C; c0 += FQ_C) {
    __syncthreads();
    stage(c0, v, sb);
    __syncthreads();
    if (c0 + FQ_C < C) fetch(c0 + FQ_C, v, sb);
    compute(c0);
  }
#endif
  const int oy = 2 * qy0 + 4 * ty, ox = 2 * qx0 + 4 * tx;
  if (2 * (qx0 + 2 * tx) < W && ox < W) {
#pragma unroll
    for (int py = 0; py < 4; ++py) {
      if (oy + py < H)
        *reinterpret_cast<float4*>(out + ((size_t)bq * H + oy + py) * W + ox) =
            make_float4(acc[py][0].x, acc[py][0].y, acc[py][1].x, acc[py][1].y);
    }
  }
}

// den[co][y][x] = sum_ci sum_{in-bounds taps} w2[co][ci][ky][kx] * 1 + b2[co]
__global__ void first_layer_den_kernel(const float* __restrict__ w2, const float* __restrict__ b2, float* __restrict__ den,
                                       int C, int CI, int H, int W) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)C * H * W) return;
  const int co = (int)(i / ((size_t)H * W));
  const int y = (int)((i / W) % H), x = (int)(i % W);
  float acc = 0.f;
  for (int ci = 0; ci < CI; ++ci)
    for (int ky = 0; ky < 3; ++ky)
      for (int kx = 0; kx < 3; ++kx) {
        const int yy = y + ky - 1, xx = x + kx - 1;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W) acc = fmaf(1.f, w2[((co * CI + ci) * 3 + ky) * 3 + kx], acc);
      }
  den[i] = acc + (b2 ? b2[co] : 0.f);
}

// ===========================================================================
// heatmap finalisation (per sample): hm [B][K+1][H*W]
//   std_out [B][HW], std_rel [B], sub_out [B][K][HW] sorted by descending relevance,
//   rel [B][K] sorted, mask [B][K] int64 (numpy argsort(...)[..., ::-1] semantics:
//   stable ascending order reversed, i.e. ties -> larger index first)
//
// The per-map relevance is the reference's numpy float32 sum over the last two axes
// (explainer.py:161, :120): chunks of 8192 elements folded left to right into 0, each chunk by
// numpy's pairwise summation -- n < 8: a plain left-to-right chain; n <= 128: eight strided
// accumulators r[j] = a[j] + a[8+j] + ... combined as ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then
// the n % 8 tail; n > 128: split at n2 = n/2 - (n/2 % 8) and add the two halves' sums.  For
// n = 128 * 2^m the leaves are the 128-element blocks and the tree over them is balanced (a
// butterfly); other n take a serial walk of the same recursion.  Bit-identical to numpy (pinned
// by tests/golden/lrp_pins_fixture.npz).
// ===========================================================================
__device__ float pw_leaf(const float* a, int n) {   // numpy pairwise_sum for n <= 128
  if (n < 8) {
    float r = 0.f;
    for (int i = 0; i < n; ++i) r = r + a[i];
    return r;
  }
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = r[j] + a[i + j];
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res = res + a[i];
  return res;
}

__device__ float pw_serial(const float* a, int n) {   // the full recursion, one thread
  struct Fr { int lo, n, state; float left; };
  Fr st[32];
  int sp = 0;
  float ret = 0.f;
  st[0] = {0, n, 0, 0.f};
  while (sp >= 0) {
    Fr& f = st[sp];
    if (f.n <= 128) { ret = pw_leaf(a + f.lo, f.n); --sp; continue; }
    int n2 = f.n / 2;
    n2 -= n2 % 8;
    if (f.state == 0) { f.state = 1; st[sp + 1] = {f.lo, n2, 0, 0.f}; ++sp; continue; }
    if (f.state == 1) { f.state = 2; f.left = ret; st[sp + 1] = {f.lo + n2, f.n - n2, 0, 0.f}; ++sp; continue; }
    ret = f.left + ret;
    --sp;
  }
  return ret;
}

// half-leaf partial of the balanced case: thread (leaf L, half h) owns accumulators 4h..4h+3 of
// leaf L; returns ((r_4h + r_4h+1) + (r_4h+2 + r_4h+3)) -- the leaf is the two halves' sum
__device__ __forceinline__ float pw_half(const float4* leaf, int h) {
  float4 r = leaf[h];
#pragma unroll
  for (int i = 1; i < 16; ++i) {
    const float4 v = leaf[2 * i + h];
    r.x = r.x + v.x; r.y = r.y + v.y; r.z = r.z + v.z; r.w = r.w + v.w;
  }
  return (r.x + r.y) + (r.z + r.w);
}

// numpy pairwise sum of one run of n <= 8192 by the whole workgroup (256 threads); part: >= 128
// floats of LDS.  Result valid in every thread.  Contains barriers: call uniformly.
__device__ float pw_chunk_wg(const float* __restrict__ src, int n, float* part, float* bc) {
  const int tid = threadIdx.x;
  const int leaves = n / 128;
  if (n > 128 && n % 128 == 0 && (leaves & (leaves - 1)) == 0) {     // balanced: <= 64 leaves
    if (tid < 2 * leaves) part[tid] = pw_half(reinterpret_cast<const float4*>(src) + (size_t)(tid >> 1) * 32, tid & 1);
    __syncthreads();
    for (int w = 2 * leaves; w > 1; w >>= 1) {      // halves -> leaves -> balanced tree, adjacent pairs
      const float v = tid < w / 2 ? part[2 * tid] + part[2 * tid + 1] : 0.f;
      __syncthreads();
      if (tid < w / 2) part[tid] = v;
      __syncthreads();
    }
    const float r = part[0];
    __syncthreads();
    return r;
  }
  if (tid == 0) *bc = pw_serial(src, n);
  __syncthreads();
  const float r = *bc;
  __syncthreads();
  return r;
}

// numpy's float32 sum of a contiguous run: the reduction iterator feeds the inner loop chunks of
// 8192 elements (its buffer size), folded left to right into the identity 0, each chunk summed
// pairwise (oracle/lrp_ref.py numpy_pairwise_sum).
__device__ float pw_sum_wg(const float* __restrict__ src, int n, float* part, float* bc) {
  float acc = 0.f;
  for (int lo = 0; lo < n; lo += 8192) acc = acc + pw_chunk_wg(src + lo, n - lo < 8192 ? n - lo : 8192, part, bc);
  return acc;
}

__device__ void sort_desc(const float* sums, int K, int* order) {   // descending; ties: larger index first
  for (int k = 0; k < K; ++k) order[k] = k;
  for (int i = 1; i < K; ++i) {
    const int cur = order[i];
    int j = i - 1;
    while (j >= 0) {
      const float a = sums[1 + order[j]], c = sums[1 + cur];
      const bool before = (c > a) || (c == a && cur > order[j]);
      if (!before) break;
      order[j + 1] = order[j];
      --j;
    }
    order[j + 1] = cur;
  }
}

__global__ __launch_bounds__(256) void heatmap_sort_kernel(const float* __restrict__ hm, int K, int HW, int std_sum,
                                                           float* __restrict__ std_out, float* __restrict__ std_rel,
                                                           float* __restrict__ sub_out, float* __restrict__ rel,
                                                           int64_t* __restrict__ mask) {
  __shared__ float part[128];
  __shared__ float bc;
  __shared__ float sums[65];
  __shared__ int order[64];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int NM = std_sum ? K : K + 1;              // maps per sample in hm
  const float* base = hm + (size_t)b * NM * HW;
  const float* sub0 = base + (std_sum ? 0 : (size_t)HW);
  float* so = std_out + (size_t)b * HW;
  // the standard map: clone 0, or (std_sum) the sum of the K concept maps, k ascending
  for (int i = tid * 4; i < HW; i += 256 * 4) {
    float4 v = *reinterpret_cast<const float4*>(std_sum ? sub0 + i : base + i);
    for (int k = 1; std_sum && k < K; ++k) {
      const float4 u = *reinterpret_cast<const float4*>(sub0 + (size_t)k * HW + i);
      v.x = v.x + u.x; v.y = v.y + u.y; v.z = v.z + u.z; v.w = v.w + u.w;
    }
    *reinterpret_cast<float4*>(so + i) = v;
  }
  __syncthreads();                                  // std_out complete and visible to the block
  {
    const float s0 = pw_sum_wg(so, HW, part, &bc);
    if (tid == 0) sums[0] = s0;
  }
  for (int q = 0; q < K; ++q) {
    const float sq = pw_sum_wg(sub0 + (size_t)q * HW, HW, part, &bc);
    if (tid == 0) sums[1 + q] = sq;
  }
  __syncthreads();
  if (tid == 0) {
    sort_desc(sums, K, order);
    std_rel[b] = sums[0];
    for (int k = 0; k < K; ++k) {
      rel[(size_t)b * K + k] = sums[1 + order[k]];
      mask[(size_t)b * K + k] = order[k];
    }
  }
  __syncthreads();
  for (int k = 0; k < K; ++k) {
    const float* src = sub0 + (size_t)order[k] * HW;
    float* dst = sub_out + ((size_t)b * K + k) * HW;
    for (int i = tid * 4; i < HW; i += 256 * 4)
      *reinterpret_cast<float4*>(dst + i) = *reinterpret_cast<const float4*>(src + i);
  }
}

// The same split / sums / sort with every map read ONCE: at K = 4 and H*W = 16384 (GTZAN-128, the
// headline) each thread keeps its 16 float4 of the K subspace maps in registers (one workgroup per
// CU; the kernel is HBM-bound) and copies the standard map while loading it, so the sorted writes
// need no second read.  The numpy pairwise sums need each accumulator chain (stride-8 elements of
// one 128-element leaf) in one thread, so thread t = (leaf t/2, half t%2) loads the float4s
// 32 leaf + 2 i + half, i = 0..15: its four chains in order (a wave's load covers 32 B of each of
// 32 leaves; the four loads i..i+3 complete each 128-B line).  Outputs equal heatmap_sort_kernel's.
template <int KC, int NV4, bool SSUM>
__global__ __launch_bounds__(256) void heatmap_sort_cached_kernel(const float* __restrict__ hm, float* __restrict__ std_out,
                                                                  float* __restrict__ std_rel,
                                                                  float* __restrict__ sub_out, float* __restrict__ rel,
                                                                  int64_t* __restrict__ mask) {
  constexpr int HW = NV4 * 1024;
  static_assert(HW / 128 * 2 == 256 && NV4 == 16, "cached sort: one (leaf, half) per thread, 16 float4 each");
  __shared__ float red[KC + 1][4];
  __shared__ float sums[KC + 1];
  __shared__ int order[KC];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int L = tid >> 1, hh = tid & 1;
  constexpr int NM = SSUM ? KC : KC + 1;            // maps per sample in hm
  const float4* base = reinterpret_cast<const float4*>(hm + (size_t)b * NM * HW) + 32 * L + hh;
  const float4* sub0 = base + (SSUM ? 0 : HW / 4);
  float4* so = reinterpret_cast<float4*>(std_out + (size_t)b * HW) + 32 * L + hh;
  float4 v[KC][NV4];
  float s[KC + 1];
  auto chain = [&](const float4* x) -> float {   // pw_half on registers, then the leaf
    float4 r = x[0];
#pragma unroll
    for (int i = 1; i < NV4; ++i) {
      r.x = r.x + x[i].x; r.y = r.y + x[i].y; r.z = r.z + x[i].z; r.w = r.w + x[i].w;
    }
    const float p = (r.x + r.y) + (r.z + r.w);
    return p + shfl_xor(p, 1);
  };
  {
    float4 w[NV4];
    if constexpr (!SSUM) {
#pragma unroll
      for (int i = 0; i < NV4; ++i) w[i] = base[2 * i];
    }
#pragma unroll
    for (int q = 0; q < KC; ++q)
#pragma unroll
      for (int i = 0; i < NV4; ++i) v[q][i] = sub0[(size_t)q * (HW / 4) + 2 * i];
    if constexpr (SSUM) {   // the standard map = the concept maps summed, k ascending
#pragma unroll
      for (int i = 0; i < NV4; ++i) {
        float4 t = v[0][i];
#pragma unroll
        for (int q = 1; q < KC; ++q) {
          t.x = t.x + v[q][i].x; t.y = t.y + v[q][i].y; t.z = t.z + v[q][i].z; t.w = t.w + v[q][i].w;
        }
        w[i] = t;
      }
    }
#pragma unroll
    for (int i = 0; i < NV4; ++i) so[2 * i] = w[i];
    s[0] = chain(w);
  }
#pragma unroll
  for (int q = 0; q < KC; ++q) s[1 + q] = chain(v[q]);
  // balanced tree over the leaves: lanes 2L, 2L+1 hold leaf L; in-wave butterfly over L; waves
  // 0-1 hold the first 8192-element chunk, 2-3 the second: (0 + (w0 + w1)) + (w2 + w3)
#pragma unroll
  for (int q = 0; q <= KC; ++q) {
    float a = s[q];
    for (int m = 2; m <= 32; m <<= 1) a = a + shfl_xor(a, m);
    if (lane_id() == 0) red[q][wave_id()] = a;
  }
  __syncthreads();
  if (tid == 0) {
    for (int q = 0; q <= KC; ++q) sums[q] = (0.f + (red[q][0] + red[q][1])) + (red[q][2] + red[q][3]);
    sort_desc(sums, KC, order);
    std_rel[b] = sums[0];
    for (int k = 0; k < KC; ++k) {
      rel[(size_t)b * KC + k] = sums[1 + order[k]];
      mask[(size_t)b * KC + k] = order[k];
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const int src = order[k];   // uniform: the branch below is a scalar one
    float4* dst = reinterpret_cast<float4*>(sub_out + ((size_t)b * KC + k) * HW) + 32 * L + hh;
#pragma unroll
    for (int q = 0; q < KC; ++q)
      if (src == q) {
#pragma unroll
        for (int i = 0; i < NV4; ++i) dst[2 * i] = v[q][i];
      }
  }
}

// ===========================================================================
// AlphaBeta (zennit 0.5.1 AlphaBeta, reference pf.py:289) on a conv with non-negative input,
// around two plain backward convs (the x- terms vanish):
//   split:   gp = R / stab(den_p), gn = R / stab(den_n)          (per element of the conv output;
//            den per sample, R rows are sample*clones + clone)
//   combine: R_in = alpha * (x J^T_{W+} gp) - beta * (x J^T_{W-} gn)   (two roundings each, no fma)
//            then the post step of the layer below, as the conv epilogue: x > 0 ? R / stab(den) : 0
//            (POST_DIV), x > 0 ? R : 0 (POST_MASK) or R.
// ===========================================================================
__global__ __launch_bounds__(256) void ab_split_kernel(const float* __restrict__ g, const float* __restrict__ dp,
                                                       const float* __restrict__ dn, float* __restrict__ gp,
                                                       float* __restrict__ gn, int64_t n, int clones, int64_t total,
                                                       float eps) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t bq = i / n, j = i - bq * n;
    const int64_t o = (bq / clones) * n + j;
    const float r = g[i];
    gp[i] = div_nb(r, stab(dp[o], eps));
    gn[i] = div_nb(r, stab(dn[o], eps));
  }
}

__global__ __launch_bounds__(256) void ab_combine_kernel(const float* __restrict__ pos, const float* __restrict__ neg,
                                                         float alpha, float beta, const float* __restrict__ x,
                                                         const float* __restrict__ den, float* __restrict__ out,
                                                         int64_t n, int clones, int64_t total, int post, float eps) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t bq = i / n, j = i - bq * n;
    const int64_t o = (bq / clones) * n + j;
    const float a = alpha * pos[i];
    const float b = beta * neg[i];
    float R = a - b;
    if (post != POST_NONE) {
      const float xv = x[o];
      if (post == POST_DIV) R = div_nb(R, stab(den[o], eps));
      R = (xv > 0.f) ? R : 0.f;
    }
    out[i] = R;
  }
}

unsigned ew_grid(int64_t total) {
  const int64_t g = (total + 255) / 256;
  return (unsigned)(g < 65536 ? (g > 0 ? g : 1) : 65536);
}

template <typename F>
int with_lds(F* fn, size_t lds) {
  return drsa::ensure_smem((const void*)fn, lds);   // per device, thread-safe
}

// padded projection width: the smallest instantiated DP >= d (0 = unsupported)
int proj_dp(int d) { return d < 1 ? 0 : d <= 16 ? 16 : d <= 32 ? 32 : d <= 64 ? 64 : d <= 128 ? 128 : 0; }

template <int D, bool PL>
size_t proj_fwd_lds(bool hout) {
  return ((hout ? (size_t)D * (D + 1) : 0) + (size_t)D * 68 + p_lds_floats<D, PL>()) * sizeof(float);
}
template <int D>
size_t proj_bwd_lds() { return ((size_t)D * (D + 1) + 2 * (size_t)D * 68) * sizeof(float); }
template <int D, bool PL>
size_t proj_bwd_rc_lds() { return ((size_t)D * (D + 1) + 4 * 2 * (size_t)D * 16 + p_lds_floats<D, PL>()) * sizeof(float); }

// Where the projection kernels keep the residual P: the forward holds its MFMA operands in
// registers (unpadded DP <= 64; 0.139 ms at B = 512, d = 64, vs 0.161 with P in LDS, which costs a
// workgroup per CU) and the backward reads them through L1 (0.524 vs 0.537 ms from LDS; registers
// would cost it a wave per SIMD).  The LDS form stays compiled for padded problems' fallbacks.
bool proj_p_lds_fwd() { return false; }

bool proj_p_lds_bwd() { return false; }

}  // namespace

extern "C" {

int drsa_amd_linear_fwd(const float* x, const float* Wt, const float* bias, float* z_out, float* relu_out, int M,
                        int N, int K, void* stream) {
  DRSA_REQUIRE(M > 0 && N > 0 && K > 0, "linear_fwd: bad shape");
  LinArgs a{};
  a.A = x; a.W = Wt; a.bias = bias; a.out = z_out; a.out_relu = relu_out; a.M = M; a.N = N; a.K = K; a.bwd = 0;
  // int64_t K (float4-aligned rows): the prefetching kernel; same chain order, same results
  if (K % 4 == 0 && K >= L1K)
    hipLaunchKernelGGL(linear_fwd_w1_kernel, dim3((M + 15) / 16, (N + 15) / 16), dim3(64), 0, (hipStream_t)stream, a);
  else if (K % 4 == 0 && K >= LFK)
    hipLaunchKernelGGL(linear_fwd_kernel, dim3((M + LT - 1) / LT, (N + LT - 1) / LT), dim3(256), 0, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(linear_kernel, dim3((M + LT - 1) / LT, (N + LT - 1) / LT), dim3(256), 0, (hipStream_t)stream, a);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

// out[M][Kin] = epi( g[M][Nout] W[Nout][Kin] ),  g = prologue(R or seed, z)
int drsa_amd_linear_bwd(const float* R, const int* seed_cls, int one_hot, const float* z, int relu_mask, int rule_eps,
                        float eps, const float* Wt, const float* x, int xmode, const float* den, int post,
                        float eps_post, float* out, int M, int Nout, int Kin, void* stream) {
  DRSA_REQUIRE(M > 0 && Nout > 0 && Kin > 0, "linear_bwd: bad shape");
  DRSA_REQUIRE(R || seed_cls, "linear_bwd: need R or a seed");
  DRSA_REQUIRE(xmode == XM_NONE || x, "linear_bwd: xmode needs x");
  DRSA_REQUIRE(post == POST_NONE || (x && (den || post == POST_MASK)), "linear_bwd: POST_DIV needs x and den");
  LinArgs a{};
  a.A = R; a.cls = seed_cls; a.one_hot = one_hot; a.z = z; a.relu_mask = relu_mask; a.rule_eps = rule_eps;
  a.eps = eps; a.W = Wt; a.x = x; a.xmode = xmode; a.den = den; a.post = post; a.eps_post = eps_post; a.out = out;
  a.M = M; a.N = Kin; a.K = Nout; a.bwd = 1;
  hipLaunchKernelGGL(linear_kernel, dim3((M + LT - 1) / LT, (Kin + LT - 1) / LT), dim3(256), 0, (hipStream_t)stream, a);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

int drsa_amd_projection_residual(const float* U, int D, float* P, void* stream) {
  DRSA_REQUIRE(U && P && D >= 1 && D <= 128, "projection_residual: need U, P and 1 <= d <= 128");
  hipLaunchKernelGGL(projection_residual_kernel, dim3((D * D + 255) / 256), dim3(256), 0, (hipStream_t)stream, U, D, P);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

int drsa_amd_projection_fwd(const float* a, const float* U, const float* P, float* h, float* ap, float* pooled,
                            uint8_t* amax, int B, int D, int H, int W, int pool, void* stream) {
  const int TW = W < 32 ? W : 32;
  DRSA_REQUIRE(a && U && P, "projection_fwd: a, U and P (drsa_amd_projection_residual) are required");
  DRSA_REQUIRE((W == 8 || W == 16 || W % 32 == 0) && H % (64 / TW) == 0,
               "projection_fwd: W must be 8, 16 or a multiple of 32 and H a multiple of 64/min(W,32) (got %dx%d)", H, W);
  DRSA_REQUIRE(!pool || (pooled && amax), "projection_fwd: pool needs outputs");
  DRSA_REQUIRE((int64_t)D * H * W < ((int64_t)1 << 31), "projection_fwd: one sample's d x H x W must stay below 2^31");
  DRSA_REQUIRE(pool || ap, "projection_fwd: without pool a' (ap) is the output");
  hipStream_t s = (hipStream_t)stream;
  const int tiles = (H / (64 / TW)) * (W / TW);
  const dim3 grid((tiles + PT - 1) / PT, B);
  switch (proj_dp(D)) {
#define PF(DD)                                                                                        \
  case DD: {                                                                                          \
    constexpr bool PLC = DD <= 64;                                                                  \
    const bool pl = PLC && proj_p_lds_fwd();                                                        \
    auto kf = h ? (D == DD ? (pl ? projection_fwd_kernel<DD, false, PLC, true> : projection_fwd_kernel<DD, false, false, true>)   \
                           : (pl ? projection_fwd_kernel<DD, true, PLC, true> : projection_fwd_kernel<DD, true, false, true>))   \
                : (D == DD ? (pl ? projection_fwd_kernel<DD, false, PLC, false> : projection_fwd_kernel<DD, false, false, false>) \
                           : (pl ? projection_fwd_kernel<DD, true, PLC, false> : projection_fwd_kernel<DD, true, false, false>)); \
    const size_t lds = pl ? proj_fwd_lds<DD, PLC>(h != nullptr) : proj_fwd_lds<DD, false>(h != nullptr);  \
    { int rc = with_lds(kf, lds); if (rc) return rc; }                                              \
    hipLaunchKernelGGL(kf, grid, dim3(256), lds, s, a, U, P, h, ap, pooled, amax,                    \
                       D, H, W, pool);                                                                \
    break;                                                                                            \
  }
    PF(16) PF(32) PF(64) PF(128)
#undef PF
    default:
      drsa::set_error("projection_fwd: unsupported d=%d", D);
      return DRSA_EUNSUPPORTED;
  }
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

int drsa_amd_projection_bwd(const float* gp, const uint8_t* amax, const float* ap, const float* h, const float* a,
                            const float* den, const float* U, const float* P, float* G, int B, int D, int H, int W,
                            int K, float eps_proj, float eps_den, int fanout, void* stream) {
  const int TW = W < 32 ? W : 32;
  DRSA_REQUIRE(fanout >= 0 && fanout <= 2, "projection_bwd: fanout must be 0, 1 or 2");
  DRSA_REQUIRE((int64_t)D * H * W < ((int64_t)1 << 31), "projection_bwd: one sample's d x H x W must stay below 2^31");
  DRSA_REQUIRE(gp && a && U && G && ((ap && h) || P),
               "projection_bwd: gp, a, U, G and P (when h / a' are recomputed) are required");
  DRSA_REQUIRE((W == 8 || W == 16 || W % 32 == 0) && H % (64 / TW) == 0,
               "projection_bwd: W must be 8, 16 or a multiple of 32 and H a multiple of 64/min(W,32) (got %dx%d)", H, W);
  DRSA_REQUIRE(K > 0 && D % K == 0, "projection_bwd: K must divide d");
  hipStream_t s = (hipStream_t)stream;
  const int tiles = (H / (64 / TW)) * (W / TW);
  const int sparse = amax != nullptr, has_den = den != nullptr;
  if (!ap || !h) {   // recompute h and a' from a
    const dim3 grid((tiles + PT_RC - 1) / PT_RC, B);
    switch (proj_dp(D)) {
#define PR(DD)                                                                                        \
  case DD: {                                                                                          \
    constexpr bool PLC = DD <= 64;                                                                  \
    const bool pl = PLC && proj_p_lds_bwd();                                                        \
    auto kr = D == DD ? (pl ? projection_bwd_rc_kernel<DD, false, PLC> : projection_bwd_rc_kernel<DD, false, false>) \
                      : (pl ? projection_bwd_rc_kernel<DD, true, PLC> : projection_bwd_rc_kernel<DD, true, false>);  \
    const size_t lds = pl ? proj_bwd_rc_lds<DD, PLC>() : proj_bwd_rc_lds<DD, false>();              \
    { int rc = with_lds(kr, lds); if (rc) return rc; }                                              \
    hipLaunchKernelGGL(kr, grid, dim3(256), lds, s, gp, amax, a, den, U, P, G,                       \
                       D, H, W, K, eps_proj, eps_den, sparse, has_den, fanout);                      \
    break;                                                                                            \
  }
      PR(16) PR(32) PR(64) PR(128)
#undef PR
      default:
        drsa::set_error("projection_bwd: unsupported d=%d", D);
        return DRSA_EUNSUPPORTED;
    }
    DRSA_LAUNCH_CHECK();
    return DRSA_OK;
  }
  const dim3 grid((tiles + PT_BWD - 1) / PT_BWD, B);
  switch (proj_dp(D)) {
#define PB(DD)                                                                                        \
  case DD: {                                                                                          \
    auto kb = D == DD ? projection_bwd_kernel<DD, false> : projection_bwd_kernel<DD, true>;        \
    { int rc = with_lds(kb, proj_bwd_lds<DD>()); if (rc) return rc; }                               \
    hipLaunchKernelGGL(kb, grid, dim3(256), proj_bwd_lds<DD>(), s, gp, amax, ap, h, a, den, U,      \
                       G, D, H, W, K, eps_proj, eps_den, sparse, has_den, fanout);                            \
    break;                                                                                            \
  }
    PB(16) PB(32) PB(64) PB(128)
#undef PB
    default:
      drsa::set_error("projection_bwd: unsupported d=%d", D);
      return DRSA_EUNSUPPORTED;
  }
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

int drsa_amd_first_layer_bwd(const float* g, const uint8_t* amax, const float* w2f, float* out, int Bq, int clones,
                             int C, int H, int W, void* stream) {
  DRSA_REQUIRE(Bq > 0 && clones > 0 && Bq % clones == 0, "first_layer_bwd: bad batch");
  DRSA_REQUIRE((int64_t)C * H * W < ((int64_t)1 << 31), "first_layer_bwd: one sample's C x H x W must stay below 2^31");
  if (amax) {
    DRSA_REQUIRE(H % 2 == 0 && W % 4 == 0, "first_layer_bwd: pooled path needs even H and W % 4 == 0");
    const int H2 = H / 2, W2 = W / 2;
    const dim3 grid(((H2 + FQ_Y - 1) / FQ_Y) * ((W2 + FQ_X - 1) / FQ_X), Bq);
    constexpr size_t lds = sizeof(float) * FQ_C * FQ_PY * FQ_PX;
#ifndef DRSA_FL_W2C_OFF
#define DRSA_FL_W2C_OFF 0
#endif
    auto kf = W == 128 && !DRSA_FL_W2C_OFF ? first_layer_bwd_pooled_kernel<64> : first_layer_bwd_pooled_kernel<0>;
    DRSA_SMEM(kf, lds);
    hipLaunchKernelGGL(kf, grid, dim3(256), lds, (hipStream_t)stream, g, amax, w2f, out, C, H, W, clones);
  } else {
    const dim3 grid(((H + FL_TH - 1) / FL_TH) * ((W + FL_TW - 1) / FL_TW), Bq);
    if (W % 4 == 0)
      hipLaunchKernelGGL(first_layer_bwd_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, g, w2f, out, C, H, W);
    else
      hipLaunchKernelGGL(first_layer_bwd_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, g, w2f, out, C, H, W);
  }
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

int drsa_amd_first_layer_den(const float* w2, const float* b2, float* den, int C, int CI, int H, int W, void* stream) {
  const size_t n = (size_t)C * H * W;
  hipLaunchKernelGGL(first_layer_den_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, w2,
                     b2, den, C, CI, H, W);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

int drsa_amd_heatmap_sort(const float* hm, int B, int K, int HW, int std_from_sum, float* std_out, float* std_rel,
                          float* sub_out, float* rel, int64_t* mask, void* stream) {
  DRSA_REQUIRE(K >= 1 && K <= 64, "heatmap_sort: K must be in [1, 64]");
  DRSA_REQUIRE(HW % 4 == 0, "heatmap_sort: H*W must be a multiple of 4");
  if (K == 4 && HW == 16384) {
    auto kern = std_from_sum ? heatmap_sort_cached_kernel<4, 16, true> : heatmap_sort_cached_kernel<4, 16, false>;
    hipLaunchKernelGGL(kern, dim3(B), dim3(256), 0, (hipStream_t)stream, hm, std_out, std_rel, sub_out, rel, mask);
  } else {
    hipLaunchKernelGGL(heatmap_sort_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, hm, K, HW, std_from_sum ? 1 : 0,
                       std_out, std_rel, sub_out, rel, mask);
  }
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

int drsa_amd_ab_split(const float* g, const float* den_p, const float* den_n, float* gp, float* gn, int Bq,
                      int clones, int64_t n, float eps, void* stream) {
  DRSA_REQUIRE(g && den_p && den_n && gp && gn, "ab_split: null pointer");
  DRSA_REQUIRE(Bq > 0 && clones > 0 && Bq % clones == 0 && n > 0, "ab_split: bad shape");
  const int64_t total = (int64_t)Bq * n;
  hipLaunchKernelGGL(ab_split_kernel, dim3(ew_grid(total)), dim3(256), 0, (hipStream_t)stream, g, den_p, den_n, gp, gn,
                     n, clones, total, eps);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

int drsa_amd_ab_combine(const float* pos, const float* neg, float alpha, float beta, const float* x, const float* den,
                        float* out, int Bq, int clones, int64_t n, int post, float eps, void* stream) {
  DRSA_REQUIRE(pos && neg && out, "ab_combine: null pointer");
  DRSA_REQUIRE(Bq > 0 && clones > 0 && Bq % clones == 0 && n > 0, "ab_combine: bad shape");
  DRSA_REQUIRE(post == POST_NONE || (x && (den || post == POST_MASK)), "ab_combine: post needs x (and den)");
  const int64_t total = (int64_t)Bq * n;
  hipLaunchKernelGGL(ab_combine_kernel, dim3(ew_grid(total)), dim3(256), 0, (hipStream_t)stream, pos, neg, alpha,
                     beta, x, den, out, n, clones, total, post, eps);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

}  // extern "C"
