// DRSA optimiser on gfx950: one Stiefel gradient-ascent step + polar retraction.
//
// Reference semantics (cxai/xai/drsa/drsa.py):
//   obj_val        drsa.py:122-155   s = relu(sum_{j in k} (AU)_nj (CU)_nj)   [N, K]
//   objective_fn   drsa.py:224-238   f = (mean_k sqrt( sqrt(mean_n s_nk^2) ))^2
//   run            drsa.py:84-106    U <- orthogonalize(U + grad f(U)), log f(U)
//   orthogonalize  drsa.py:201-221   U (U^T U)^{-1/2}  (reference: fp64 eigh on the host)
//
// Device design (no host round trip per step):
//   drsa_partial_kernel  one pass over row tiles of A, C (fp32 MFMA 16x16x4):
//                        XA = A_t U, XC = C_t U, s, r = relu(s), S_k += r^2,
//                        Gt += A_t^T (R (.) XC) + C_t^T (R (.) XA)   (R = r broadcast over block k)
//                        -> one [D*D + K] fp32 partial slab per workgroup
//   drsa_reduce_kernel   fixed-order sum of the slabs (deterministic, no atomics)
//   drsa_finish_kernel   M_k = sqrt(S_k/N), f, c_k = sqrt(f)/(K N M_k^1.5), V = U + Gt diag(c),
//                        polar(V) by Newton-Schulz on fp32 MFMA in one workgroup; writes f, U_new
// The closed-form gradient equals autograd's (checked in float64 in tests/test_oracle_drsa.py).
#include "common.h"
#include "drsa_amd.h"

#include <stdarg.h>
#include <vector>

namespace drsa {
static thread_local char g_err[512];
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
const char* last_error() { return g_err; }
}  // namespace drsa

namespace {

constexpr int kThreads = 256;   // 4 waves

// ---------------------------------------------------------------------------
// partial kernel
//   D in {16, 32, 64, 128}; DK = D / K in {1,2,4,8,16} or a multiple of 16.
//   RT rows per tile: 64 (D <= 64) or 32 (D = 128, LDS budget).
//   LDS: Us[D][D], As/Cs/Ps/Qs[RT][D+1]  (D+1: conflict-free column reads)
//   GEMM1 wave w: row block rb = w % WR (16 rows), column group cg = w / WR (NBW column blocks)
//   GEMM2 wave w: Gt row blocks {w, w+4, ...} (16 rows each), all D/16 column blocks
// ---------------------------------------------------------------------------
template <int D>
struct PartialCfg {
  static constexpr int RT = (D <= 64) ? 64 : 32;
  static constexpr int NB = D / 16;             // 16-wide column blocks
  static constexpr int WR = RT / 16;            // row blocks per tile (waves along rows)
  static constexpr int WC = 4 / WR;             // column groups
  static constexpr int NBW = NB / WC;           // column blocks per wave in GEMM1
  static constexpr int LDA = D + 1;
  static constexpr int IB = (NB + 3) / 4;       // Gt row blocks per wave
  static constexpr size_t lds_floats = (size_t)D * D + 4 * (size_t)RT * LDA;
};

// BF: A and C are bf16 in HBM (C5: "bf16 MFMA projection with fp32 accumulate"); GEMM1
// (XA = A U, XC = C U) runs on v_mfma_f32_16x16x32_bf16 with U rounded to bf16 (RNE) once per
// step; everything after it (relu, S, P/Q, GEMM2 on the exactly widened A/C, slab) is fp32.
template <int D, int DK, bool BF>
__global__ __launch_bounds__(kThreads) void drsa_partial_kernel(
    const void* __restrict__ A_, const void* __restrict__ C_, int64_t N,
    const float* __restrict__ U, float* __restrict__ partials, int64_t tiles_per_wg) {
  using Cfg = PartialCfg<D>;
  constexpr int RT = Cfg::RT, NB = Cfg::NB, WR = Cfg::WR, NBW = Cfg::NBW, LDA = Cfg::LDA, IB = Cfg::IB;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const float* A = reinterpret_cast<const float*>(A_);
  const float* C = reinterpret_cast<const float*>(C_);
  const uint16_t* Ab = reinterpret_cast<const uint16_t*>(A_);
  const uint16_t* Cb = reinterpret_cast<const uint16_t*>(C_);
  float* Us = smem;                                            // fp32 U [D][D]  (BF: bf16 U^T [D][D])
  uint16_t* Ubt = reinterpret_cast<uint16_t*>(smem);
  float* As = Us + (BF ? D * D / 2 : D * D);
  float* Cs = As + RT * LDA;
  float* Ps = Cs + RT * LDA;
  float* Qs = Ps + RT * LDA;

  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  const int rb = w % WR, cg = w / WR;
  constexpr int K = D / DK;

  if constexpr (BF) {
    for (int i = tid; i < D * D; i += kThreads) {     // Ubt[c][k] = bf16_rne(U[k][c])
      const int c = i / D, k = i % D;
      const uint32_t u = __float_as_uint(U[k * D + c]);
      Ubt[i] = (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
    }
  } else {
    for (int i = tid; i < D * D; i += kThreads) Us[i] = U[i];
  }

  f32x4 g[IB][NB];
#pragma unroll
  for (int ib = 0; ib < IB; ++ib)
#pragma unroll
    for (int cb = 0; cb < NB; ++cb) g[ib][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  // S partial: per lane, per GEMM1 column block it owns (summed over its rows and tiles)
  float s_cb[NBW];
#pragma unroll
  for (int q = 0; q < NBW; ++q) s_cb[q] = 0.f;

  const int64_t n_tiles = (N + RT - 1) / RT;
  const int64_t t0 = (int64_t)blockIdx.x * tiles_per_wg;
  const int64_t t1 = min(n_tiles, t0 + tiles_per_wg);

  for (int64_t t = t0; t < t1; ++t) {
    const int64_t r0 = t * RT;
    __syncthreads();
    // ---- stage A, C tile (rows >= N zero-filled: they contribute nothing) ----
    for (int i = tid; i < RT * D / 4; i += kThreads) {
      const int row = (i * 4) / D, col = (i * 4) % D;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), c = a;
      if (r0 + row < N) {
        if constexpr (BF) {   // 4 bf16 -> 4 fp32 (exact)
          const uint2 ua = *reinterpret_cast<const uint2*>(Ab + (r0 + row) * D + col);
          const uint2 uc = *reinterpret_cast<const uint2*>(Cb + (r0 + row) * D + col);
          a = make_float4(__uint_as_float(ua.x << 16), __uint_as_float(ua.x & 0xffff0000u),
                          __uint_as_float(ua.y << 16), __uint_as_float(ua.y & 0xffff0000u));
          c = make_float4(__uint_as_float(uc.x << 16), __uint_as_float(uc.x & 0xffff0000u),
                          __uint_as_float(uc.y << 16), __uint_as_float(uc.y & 0xffff0000u));
        } else {
          a = *reinterpret_cast<const float4*>(A + (r0 + row) * D + col);
          c = *reinterpret_cast<const float4*>(C + (r0 + row) * D + col);
        }
      }
      float* pa = As + row * LDA + col;
      float* pc = Cs + row * LDA + col;
      pa[0] = a.x; pa[1] = a.y; pa[2] = a.z; pa[3] = a.w;
      pc[0] = c.x; pc[1] = c.y; pc[2] = c.z; pc[3] = c.w;
    }
    __syncthreads();
    // ---- GEMM1: XA, XC for rows [16 rb, 16 rb + 16), column blocks cg*NBW + q ----
    f32x4 xa[NBW], xc[NBW];
#pragma unroll
    for (int q = 0; q < NBW; ++q) { xa[q] = f32x4{0.f, 0.f, 0.f, 0.f}; xc[q] = xa[q]; }
    const int arow = 16 * rb + (lane & 15);
    if constexpr (BF) {
      // lane: A[row][k0 + 8(lane>>4) + j], U^T[col][k0 + 8(lane>>4) + j], j < 8
#pragma unroll
      for (int k0 = 0; k0 < D; k0 += 32) {
        const int kb = k0 + 8 * (lane >> 4);
        u16x8 ab, cb;
#pragma unroll
        for (int j = 0; j < 8; ++j) {   // widened bf16 values: the top 16 bits are exact
          ab[j] = (uint16_t)(__float_as_uint(As[arow * LDA + kb + j]) >> 16);
          cb[j] = (uint16_t)(__float_as_uint(Cs[arow * LDA + kb + j]) >> 16);
        }
#pragma unroll
        for (int q = 0; q < NBW; ++q) {
          const u16x8 ub = *reinterpret_cast<const u16x8*>(Ubt + (16 * (cg * NBW + q) + (lane & 15)) * D + kb);
          xa[q] = mfma16_bf16(ab, ub, xa[q]);
          xc[q] = mfma16_bf16(cb, ub, xc[q]);
        }
      }
    } else {
#pragma unroll 4
      for (int k0 = 0; k0 < D; k0 += 4) {
        const int kk = k0 + (lane >> 4);
        const float av = As[arow * LDA + kk];
        const float cv = Cs[arow * LDA + kk];
#pragma unroll
        for (int q = 0; q < NBW; ++q) {
          const float bv = Us[kk * D + 16 * (cg * NBW + q) + (lane & 15)];
          xa[q] = mfma16(av, bv, xa[q]);
          xc[q] = mfma16(cv, bv, xc[q]);
        }
      }
    }
    // ---- s = sum over the concept block of XA (.) XC, r = relu(s) ----
    // lane holds rows 16 rb + (lane>>4)*4 + r, column 16 (cg*NBW + q) + (lane&15)
    float rr[NBW][4];
    if constexpr (DK >= 16) {
      constexpr int cbk = DK / 16;   // column blocks per concept (divides NBW: host-checked)
#pragma unroll
      for (int q = 0; q < NBW; ++q) {
        if (q % cbk != 0) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = 0.f;
          for (int u = 0; u < cbk; ++u) v += xa[q + u][r] * xc[q + u][r];
          v += shfl_xor(v, 1); v += shfl_xor(v, 2); v += shfl_xor(v, 4); v += shfl_xor(v, 8);
          const float rv = v > 0.f ? v : 0.f;
          for (int u = 0; u < cbk; ++u) rr[q + u][r] = rv;
        }
      }
    } else {
#pragma unroll
      for (int q = 0; q < NBW; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = xa[q][r] * xc[q][r];
          if constexpr (DK >= 2) v += shfl_xor(v, 1);
          if constexpr (DK >= 4) v += shfl_xor(v, 2);
          if constexpr (DK >= 8) v += shfl_xor(v, 4);
          rr[q][r] = v > 0.f ? v : 0.f;
        }
    }
    // S partial: the first lane/column block of each concept records r^2 (4 rows)
    const bool owner = ((lane & 15) % (DK < 16 ? DK : 16)) == 0;
#pragma unroll
    for (int q = 0; q < NBW; ++q) {
      if (owner && (DK < 16 || (q % (DK / 16)) == 0)) {
        float acc = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc += rr[q][r] * rr[q][r];
        s_cb[q] += acc;
      }
    }
    // P = R (.) XC, Q = R (.) XA -> LDS
#pragma unroll
    for (int q = 0; q < NBW; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * rb + (lane >> 4) * 4 + r, col = 16 * (cg * NBW + q) + (lane & 15);
        Ps[row * LDA + col] = rr[q][r] * xc[q][r];
        Qs[row * LDA + col] = rr[q][r] * xa[q][r];
      }
    __syncthreads();
    // ---- GEMM2: Gt[i][j] += sum_n A[n][i] P[n][j] + C[n][i] Q[n][j] ----
#pragma unroll 2
    for (int n0 = 0; n0 < RT; n0 += 4) {
      const int nn = n0 + (lane >> 4);
#pragma unroll
      for (int ib = 0; ib < IB; ++ib) {
        const int iblk = w + 4 * ib;
        if (iblk >= NB) break;
        const float av = As[nn * LDA + 16 * iblk + (lane & 15)];
        const float cv = Cs[nn * LDA + 16 * iblk + (lane & 15)];
#pragma unroll
        for (int cb = 0; cb < NB; ++cb) {
          const float pv = Ps[nn * LDA + 16 * cb + (lane & 15)];
          const float qv = Qs[nn * LDA + 16 * cb + (lane & 15)];
          g[ib][cb] = mfma16(av, pv, g[ib][cb]);
          g[ib][cb] = mfma16(cv, qv, g[ib][cb]);
        }
      }
    }
  }
  // ---- write the slab: Gt (D*D, row-major [i][j]) then S[K] ----
  float* slab = partials + (size_t)blockIdx.x * (D * D + K);
#pragma unroll
  for (int ib = 0; ib < IB; ++ib) {
    const int iblk = w + 4 * ib;
    if (iblk >= NB) break;
#pragma unroll
    for (int cb = 0; cb < NB; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * iblk + (lane >> 4) * 4 + r, j = 16 * cb + (lane & 15);
        slab[i * D + j] = g[ib][cb][r];
      }
  }
  // S: owners' s_cb through LDS (reuse Ps), fixed summation order
  __syncthreads();
  float* red = Ps;   // [4 waves][64 lanes][NBW]
#pragma unroll
  for (int q = 0; q < NBW; ++q) red[(w * 64 + lane) * NBW + q] = s_cb[q];
  __syncthreads();
  if (tid < K) {
    const int k = tid;
    const int j0 = k * DK, cb = j0 / 16, l15 = j0 % 16;
    const int cgk = cb / NBW, q = cb % NBW;
    float acc = 0.f;
    for (int rbb = 0; rbb < WR; ++rbb) {
      const int ww = cgk * WR + rbb;
      for (int lg = 0; lg < 4; ++lg) acc += red[(ww * 64 + lg * 16 + l15) * NBW + q];
    }
    slab[D * D + k] = acc;
  }
}

// ---------------------------------------------------------------------------
// reduce: out[e] = sum_p partials[p][e]   (fixed order p = 0..P-1)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void drsa_reduce_kernel(const float* __restrict__ partials,
                                                          int P, int E, float* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  float acc = 0.f;
  int p = 0;
  for (; p + 4 <= P; p += 4) {
    const float v0 = partials[(size_t)(p + 0) * E + e];
    const float v1 = partials[(size_t)(p + 1) * E + e];
    const float v2 = partials[(size_t)(p + 2) * E + e];
    const float v3 = partials[(size_t)(p + 3) * E + e];
    acc += v0; acc += v1; acc += v2; acc += v3;
  }
  for (; p < P; ++p) acc += partials[(size_t)p * E + e];
  out[e] = acc;
}

// ---------------------------------------------------------------------------
// finish: objective, scaled gradient, V = U + G, polar(V) via Newton-Schulz
//   X0 = a V; X <- X (1.5 I - 0.5 X^T X) until max|X^T X - I| < tol.
//   One workgroup of polar_waves<D>() waves (enough to keep every SIMD's MFMA pipe fed from
//   LDS); matrices in LDS [D][D+1].
// ---------------------------------------------------------------------------
template <int D>
constexpr int polar_waves() { return D >= 128 ? 16 : (D >= 64 ? 8 : 4); }

template <int D>
__device__ void lds_matmul_tn(const float* X, const float* Y, float* Z, int ld) {
  // Z = X^T Y  (all D x D, row-major with leading dim ld), fp32 MFMA 16x16x4
  constexpr int NB = D / 16, NW = polar_waves<D>();
  const int lane = lane_id(), w = wave_id();
  for (int t = w; t < NB * NB; t += NW) {
    const int ib = t / NB, jb = t % NB;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int k0 = 0; k0 < D; k0 += 4) {
      const int kk = k0 + (lane >> 4);
      acc = mfma16(X[kk * ld + 16 * ib + (lane & 15)], Y[kk * ld + 16 * jb + (lane & 15)], acc);
    }
    for (int r = 0; r < 4; ++r) Z[(16 * ib + (lane >> 4) * 4 + r) * ld + 16 * jb + (lane & 15)] = acc[r];
  }
}

template <int D>
__device__ void lds_matmul_nn_inplace(float* X, const float* Y, int ld) {
  // X <- X Y.  Each wave keeps its output tiles in registers until every wave has
  // finished reading X, then overwrites X (saves a third D x D LDS matrix).
  constexpr int NB = D / 16, NW = polar_waves<D>();
  constexpr int NT = (NB * NB + NW - 1) / NW;
  const int lane = lane_id(), w = wave_id();
  f32x4 acc[NT];
#pragma unroll
  for (int q = 0; q < NT; ++q) {
    acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int t = w + NW * q;
    if (t >= NB * NB) break;
    const int ib = t / NB, jb = t % NB;
#pragma unroll 8
    for (int k0 = 0; k0 < D; k0 += 4) {
      const int kk = k0 + (lane >> 4);
      acc[q] = mfma16(X[(16 * ib + (lane & 15)) * ld + kk], Y[kk * ld + 16 * jb + (lane & 15)], acc[q]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NT; ++q) {
    const int t = w + NW * q;
    if (t >= NB * NB) break;
    const int ib = t / NB, jb = t % NB;
    for (int r = 0; r < 4; ++r) X[(16 * ib + (lane >> 4) * 4 + r) * ld + 16 * jb + (lane & 15)] = acc[q][r];
  }
}

__device__ float block_max(float v, float* scratch) {
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, shfl_xor(v, m));
  __syncthreads();
  if (lane_id() == 0) scratch[wave_id()] = v;
  __syncthreads();
  float r = scratch[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r = fmaxf(r, scratch[i]);
  return r;
}

__device__ float block_sum(float v, float* scratch) {
  for (int m = 32; m >= 1; m >>= 1) v += shfl_xor(v, m);
  __syncthreads();
  if (lane_id() == 0) scratch[wave_id()] = v;
  __syncthreads();
  float r = scratch[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r += scratch[i];
  return r;
}

template <int D>
__device__ void polar_ns(float* X, float* P, float* scratch, float tol, int max_iter, int* iters_out) {
  // in: X = V (LDS, ld D+1); out: X = polar factor.  X <- X (1.5 I - 0.5 X^T X).
  constexpr int ld = D + 1;
  const int tid = threadIdx.x;
  __syncthreads();
  lds_matmul_tn<D>(X, X, P, ld);
  __syncthreads();
  // scaling: a = sqrt(D / tr(P)) if a^2 * ||P||_inf < 2.9 else 1/sqrt(||P||_inf)
  float tr = 0.f, rowmax = 0.f;
  for (int i = tid; i < D; i += blockDim.x) {
    tr += P[i * ld + i];
    float rs = 0.f;
    for (int j = 0; j < D; ++j) rs += fabsf(P[i * ld + j]);
    rowmax = fmaxf(rowmax, rs);
  }
  tr = block_sum(tr, scratch);
  rowmax = block_max(rowmax, scratch + 16);
  float a2 = (float)D / tr;
  if (a2 * rowmax >= 2.9f) a2 = 1.f / rowmax;
  const float a = sqrtf(a2);
  for (int i = tid; i < D * D; i += blockDim.x) {
    const int r = i / D, c = i % D;
    X[r * ld + c] *= a;
  }
  int it = 0;
  for (; it < max_iter; ++it) {
    __syncthreads();
    lds_matmul_tn<D>(X, X, P, ld);
    __syncthreads();
    float err = 0.f;
    for (int i = tid; i < D * D; i += blockDim.x) {
      const int r = i / D, c = i % D;
      const float pv = P[r * ld + c];
      err = fmaxf(err, fabsf(pv - (r == c ? 1.f : 0.f)));
      P[r * ld + c] = (r == c ? 1.5f : 0.f) - 0.5f * pv;   // T, in place
    }
    err = block_max(err, scratch + 32);
    if (err < tol) break;
    lds_matmul_nn_inplace<D>(X, P, ld);
  }
  if (iters_out && tid == 0) *iters_out = it;
  __syncthreads();
}

// mode 0: full step (f, U_out = polar(U + G)); mode 1: objective only
template <int D>
__global__ __launch_bounds__(polar_waves<D>() * 64) void drsa_finish_kernel(
    const float* __restrict__ gs, double n_total, int K, const float* __restrict__ U,
    float* __restrict__ U_out, float* __restrict__ f_out, int* __restrict__ step_counter,
    int f_stride_by_counter, int mode, float tol, int max_iter, int* __restrict__ iters_out) {
  constexpr int ld = D + 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* X = smem;
  float* P = X + D * ld;
  float* scratch = P + D * ld;   // 64 floats
  __shared__ float cvec[128];
  __shared__ float fsh;
  const int tid = threadIdx.x;
  const int DK = D / K;
  if (tid == 0) {
    // f = (mean_k sqrt(M_k))^2, M_k = sqrt(S_k / N)  (evaluated in double from fp32 sums)
    double sum = 0.0;
    for (int k = 0; k < K; ++k) sum += sqrt(sqrt((double)gs[D * D + k] / n_total));
    const double mean = sum / K;
    const double f = mean * mean;
    fsh = (float)f;
    for (int k = 0; k < K; ++k) {
      const double Mk = sqrt((double)gs[D * D + k] / n_total);
      const double ck = (Mk > 0.0) ? sqrt(f) / (K * n_total * Mk * sqrt(Mk)) : 0.0;
      cvec[k] = (float)ck;
    }
  }
  __syncthreads();
  int slot = 0;
  if (f_stride_by_counter) slot = *step_counter;
  if (tid == 0) f_out[slot] = fsh;
  if (mode == 1) return;
  for (int i = tid; i < D * D; i += blockDim.x) {
    const int r = i / D, c = i % D;
    X[r * ld + c] = U[i] + gs[i] * cvec[c / DK];
  }
  polar_ns<D>(X, P, scratch, tol, max_iter, iters_out);
  for (int i = tid; i < D * D; i += blockDim.x) {
    const int r = i / D, c = i % D;
    U_out[i] = X[r * ld + c];
  }
  if (f_stride_by_counter && tid == 0) *step_counter = slot + 1;
}

// polar only (orthogonalize API)
template <int D>
__global__ __launch_bounds__(polar_waves<D>() * 64) void polar_kernel(const float* __restrict__ V, float* __restrict__ U_out,
                                                    float tol, int max_iter, int* iters_out) {
  constexpr int ld = D + 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* X = smem;
  float* P = X + D * ld;
  float* scratch = P + D * ld;
  for (int i = threadIdx.x; i < D * D; i += blockDim.x) X[(i / D) * ld + i % D] = V[i];
  polar_ns<D>(X, P, scratch, tol, max_iter, iters_out);
  for (int i = threadIdx.x; i < D * D; i += blockDim.x) U_out[i] = X[(i / D) * ld + i % D];
}

// ---------------------------------------------------------------------------
// compute_subspace_relevances (explainer.py:206-242):
//   r[b][k] = sum_n sum_{j in block k} (a_n U)_j (c_n U)_j   (no ReLU)
// One workgroup per instance b; thread t owns rows t, t+256, ...; fixed-order reduction.
// ---------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256) void subspace_relevance_kernel(const float* __restrict__ act,
                                                                 const float* __restrict__ ctx, int64_t N, int K,
                                                                 const float* __restrict__ U, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Us = sm;              // [D][D]
  float* red = Us + D * D;     // [256][K]
  const int b = blockIdx.x, tid = threadIdx.x;
  const int dk = D / K;
  for (int i = tid; i < D * D; i += 256) Us[i] = U[i];
  for (int k = 0; k < K; ++k) red[tid * K + k] = 0.f;
  __syncthreads();
  const float* A = act + (size_t)b * N * D;
  const float* C = ctx + (size_t)b * N * D;
  for (int64_t n = tid; n < N; n += 256) {
    float av[D], cv[D];
#pragma unroll
    for (int c = 0; c < D; ++c) { av[c] = A[n * D + c]; cv[c] = C[n * D + c]; }
    for (int j = 0; j < D; ++j) {
      float xa = 0.f, xc = 0.f;
#pragma unroll
      for (int c = 0; c < D; ++c) {
        xa = fmaf(av[c], Us[c * D + j], xa);
        xc = fmaf(cv[c], Us[c * D + j], xc);
      }
      red[tid * K + j / dk] += xa * xc;
    }
  }
  __syncthreads();
  if (tid < K) {
    float acc = 0.f;
    for (int t = 0; t < 256; ++t) acc += red[t * K + tid];
    out[(size_t)b * K + tid] = acc;
  }
}

// ---------------------------------------------------------------------------
// host-side dispatch
// ---------------------------------------------------------------------------
inline bool supported_dims(int d, int K) {
  if (!(d == 16 || d == 32 || d == 64 || d == 128)) return false;
  if (K <= 0 || d % K != 0 || K > 128) return false;
  const int dk = d / K;
  if (!(dk == 1 || dk == 2 || dk == 4 || dk == 8 || dk == 16 || dk == 32 || dk == 64)) return false;
  // at D = 128 a wave's GEMM1 columns span D/2: a concept block must fit in it
  if (d == 128 && dk > 64) return false;
  return true;
}

inline int rows_per_tile(int d) { return d <= 64 ? 64 : 32; }

int cu_count() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  return cus;
}

struct PartialPlan {
  int grid;
  int64_t tiles_per_wg;
};

PartialPlan plan_partial(int64_t N, int d) {
  const int rt = rows_per_tile(d);
  const int64_t n_tiles = (N + rt - 1) / rt;
  const int64_t cap = (int64_t)cu_count();   // one 4-wave workgroup per CU (LDS-bound at D=64)
  int64_t per = (n_tiles + cap - 1) / cap;
  if (per < 1) per = 1;
  int grid = (int)((n_tiles + per - 1) / per);
  if (grid < 1) grid = 1;
  return {grid, per};
}

template <int D, int DK, bool BF>
int launch_partial(const void* A, const void* C, int64_t N, const float* U, float* partials,
                   const PartialPlan& pl, hipStream_t s) {
  const size_t lds = (PartialCfg<D>::lds_floats - (BF ? (size_t)D * D / 2 : 0)) * sizeof(float);
  static bool attr_set = false;
  if (!attr_set) {
    DRSA_HIP(hipFuncSetAttribute((const void*)drsa_partial_kernel<D, DK, BF>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr_set = true;
  }
  hipLaunchKernelGGL((drsa_partial_kernel<D, DK, BF>), dim3(pl.grid), dim3(kThreads), lds, s, A, C, N, U,
                     partials, pl.tiles_per_wg);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

template <int D, bool BF>
int dispatch_partial_d(const void* A, const void* C, int64_t N, int K, const float* U, float* partials,
                       const PartialPlan& pl, hipStream_t s) {
  switch (D / K) {
    case 1: if constexpr (D / 1 <= 128) return launch_partial<D, 1, BF>(A, C, N, U, partials, pl, s); break;
    case 2: return launch_partial<D, 2, BF>(A, C, N, U, partials, pl, s);
    case 4: return launch_partial<D, 4, BF>(A, C, N, U, partials, pl, s);
    case 8: return launch_partial<D, 8, BF>(A, C, N, U, partials, pl, s);
    case 16: return launch_partial<D, 16, BF>(A, C, N, U, partials, pl, s);
    case 32: if constexpr (D >= 32) return launch_partial<D, 32, BF>(A, C, N, U, partials, pl, s); break;
    case 64: if constexpr (D >= 64) return launch_partial<D, 64, BF>(A, C, N, U, partials, pl, s); break;
    default: break;
  }
  drsa::set_error("drsa_partial: unsupported d=%d K=%d", D, K);
  return DRSA_EUNSUPPORTED;
}

int dispatch_partial(const void* A, const void* C, int64_t N, int d, int K, const float* U,
                     float* partials, const PartialPlan& pl, hipStream_t s, bool bf = false) {
  switch (d) {
    case 16: return bf ? DRSA_EUNSUPPORTED : dispatch_partial_d<16, false>(A, C, N, K, U, partials, pl, s);
    case 32: return bf ? dispatch_partial_d<32, true>(A, C, N, K, U, partials, pl, s)
                       : dispatch_partial_d<32, false>(A, C, N, K, U, partials, pl, s);
    case 64: return bf ? dispatch_partial_d<64, true>(A, C, N, K, U, partials, pl, s)
                       : dispatch_partial_d<64, false>(A, C, N, K, U, partials, pl, s);
    case 128: return bf ? dispatch_partial_d<128, true>(A, C, N, K, U, partials, pl, s)
                        : dispatch_partial_d<128, false>(A, C, N, K, U, partials, pl, s);
  }
  return DRSA_EUNSUPPORTED;
}

template <int D>
size_t finish_lds() { return (2 * (size_t)D * (D + 1) + 64) * sizeof(float); }

template <int D>
int launch_finish(const float* gs, double n_total, int K, const float* U, float* U_out, float* f_out,
                  int* counter, int by_counter, int mode, float tol, int max_iter, int* iters,
                  hipStream_t s) {
  const size_t lds = finish_lds<D>();
  static bool attr_set = false;
  if (!attr_set) {
    DRSA_HIP(hipFuncSetAttribute((const void*)drsa_finish_kernel<D>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr_set = true;
  }
  hipLaunchKernelGGL(drsa_finish_kernel<D>, dim3(1), dim3(polar_waves<D>() * 64), lds, s, gs, n_total, K, U, U_out, f_out,
                     counter, by_counter, mode, tol, max_iter, iters);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

int dispatch_finish(const float* gs, double n_total, int d, int K, const float* U, float* U_out,
                    float* f_out, int* counter, int by_counter, int mode, float tol, int max_iter,
                    int* iters, hipStream_t s) {
  switch (d) {
    case 16: return launch_finish<16>(gs, n_total, K, U, U_out, f_out, counter, by_counter, mode, tol, max_iter, iters, s);
    case 32: return launch_finish<32>(gs, n_total, K, U, U_out, f_out, counter, by_counter, mode, tol, max_iter, iters, s);
    case 64: return launch_finish<64>(gs, n_total, K, U, U_out, f_out, counter, by_counter, mode, tol, max_iter, iters, s);
    case 128: return launch_finish<128>(gs, n_total, K, U, U_out, f_out, counter, by_counter, mode, tol, max_iter, iters, s);
  }
  return DRSA_EUNSUPPORTED;
}

constexpr float kPolarTol = 4e-7f;
constexpr int kPolarMaxIter = 40;

// workspace layout: [partials P*(d*d+K)] [gs (d*d+K)] [counter int (padded 16B)] [iters int]
size_t ws_bytes(int64_t N, int d, int K) {
  const PartialPlan pl = plan_partial(N, d);
  const size_t E = (size_t)d * d + K;
  return ((size_t)pl.grid * E + E) * sizeof(float) + 64;
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

const char* drsa_amd_last_error(void) { return drsa::last_error(); }

int drsa_amd_version(void) { return 1; }

size_t drsa_amd_drsa_workspace_bytes(int64_t N, int d, int K) {
  if (!supported_dims(d, K) || N <= 0) return 0;
  return ws_bytes(N, d, K);
}

static int partial_impl(const void* A, const void* C, int64_t N, int d, int K, const float* U, float* gs_out,
                        void* ws, size_t ws_size, void* stream, int dtype) {
  DRSA_REQUIRE(supported_dims(d, K), "drsa_partial: unsupported d=%d K=%d", d, K);
  DRSA_REQUIRE(N >= 0, "drsa_partial: N < 0");
  DRSA_REQUIRE(dtype == 0 || (dtype == 1 && d >= 32), "drsa_partial: bf16 needs d >= 32");
  hipStream_t s = (hipStream_t)stream;
  const size_t E = (size_t)d * d + K;
  if (N == 0) {
    DRSA_HIP(hipMemsetAsync(gs_out, 0, E * sizeof(float), s));
    return DRSA_OK;
  }
  DRSA_REQUIRE(ws_size >= ws_bytes(N, d, K), "drsa_partial: workspace too small");
  DRSA_REQUIRE(((uintptr_t)A % 16) == 0 && ((uintptr_t)C % 16) == 0, "drsa_partial: A/C must be 16B aligned");
  const PartialPlan pl = plan_partial(N, d);
  float* partials = (float*)ws;
  int rc = dispatch_partial(A, C, N, d, K, U, partials, pl, s, dtype == 1);
  if (rc) return rc;
  hipLaunchKernelGGL(drsa_reduce_kernel, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, s, partials,
                     pl.grid, (int)E, gs_out);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

int drsa_amd_drsa_partial(const float* A, const float* C, int64_t N, int d, int K, const float* U,
                          float* gs_out, void* ws, size_t ws_size, void* stream) {
  return partial_impl(A, C, N, d, K, U, gs_out, ws, ws_size, stream, 0);
}

int drsa_amd_drsa_partial_bf16(const uint16_t* A, const uint16_t* C, int64_t N, int d, int K, const float* U,
                               float* gs_out, void* ws, size_t ws_size, void* stream) {
  return partial_impl(A, C, N, d, K, U, gs_out, ws, ws_size, stream, 1);
}

int drsa_amd_drsa_finish(const float* gs, int64_t N_total, int d, int K, const float* U, float* U_out,
                         float* f_out, int objective_only, int* iters_out, void* stream) {
  DRSA_REQUIRE(supported_dims(d, K), "drsa_finish: unsupported d=%d K=%d", d, K);
  DRSA_REQUIRE(N_total > 0, "drsa_finish: N_total must be > 0");
  return dispatch_finish(gs, (double)N_total, d, K, U, U_out, f_out, nullptr, 0, objective_only ? 1 : 0,
                         kPolarTol, kPolarMaxIter, iters_out, (hipStream_t)stream);
}

int drsa_amd_drsa_step(const float* A, const float* C, int64_t N, int d, int K, const float* U,
                       float* U_out, float* f_out, void* ws, size_t ws_size, void* stream) {
  DRSA_REQUIRE(supported_dims(d, K), "drsa_step: unsupported d=%d K=%d", d, K);
  DRSA_REQUIRE(N > 0, "drsa_step: N must be > 0");
  DRSA_REQUIRE(U != U_out, "drsa_step: U and U_out must not alias");
  const PartialPlan pl = plan_partial(N, d);
  const size_t E = (size_t)d * d + K;
  DRSA_REQUIRE(ws_size >= ws_bytes(N, d, K), "drsa_step: workspace too small");
  float* gs = (float*)ws + (size_t)pl.grid * E;
  int rc = drsa_amd_drsa_partial(A, C, N, d, K, U, gs, ws, ws_size, stream);
  if (rc) return rc;
  return drsa_amd_drsa_finish(gs, N, d, K, U, U_out, f_out, 0, nullptr, stream);
}

int drsa_amd_drsa_objective(const float* A, const float* C, int64_t N, int d, int K, const float* U,
                            float* f_out, void* ws, size_t ws_size, void* stream) {
  DRSA_REQUIRE(supported_dims(d, K), "drsa_objective: unsupported d=%d K=%d", d, K);
  DRSA_REQUIRE(N > 0, "drsa_objective: N must be > 0");
  const PartialPlan pl = plan_partial(N, d);
  const size_t E = (size_t)d * d + K;
  DRSA_REQUIRE(ws_size >= ws_bytes(N, d, K), "drsa_objective: workspace too small");
  float* gs = (float*)ws + (size_t)pl.grid * E;
  int rc = drsa_amd_drsa_partial(A, C, N, d, K, U, gs, ws, ws_size, stream);
  if (rc) return rc;
  return drsa_amd_drsa_finish(gs, N, d, K, U, nullptr, f_out, 1, nullptr, stream);
}

// S steps in one call: f_traj[0..steps] receives f(U_t) before each update and f(U_S) after
// the loop (SubspaceOptimizer.run's trajectory, drsa.py:82-117).  U_io holds U_0 on entry and
// U_S on exit; U_tmp is a d*d scratch.  With use_graph != 0 the two-step body is captured
// once into a hipGraph and replayed (launch-bound loop).
int drsa_amd_drsa_run(const float* A, const float* C, int64_t N, int d, int K, float* U_io, float* U_tmp,
                      int steps, float* f_traj, int* counter, void* ws, size_t ws_size, int use_graph,
                      void* stream) {
  DRSA_REQUIRE(supported_dims(d, K), "drsa_run: unsupported d=%d K=%d", d, K);
  DRSA_REQUIRE(N > 0 && steps >= 0, "drsa_run: bad N/steps");
  DRSA_REQUIRE(ws_size >= ws_bytes(N, d, K), "drsa_run: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const PartialPlan pl = plan_partial(N, d);
  const size_t E = (size_t)d * d + K;
  float* gs = (float*)ws + (size_t)pl.grid * E;
  DRSA_HIP(hipMemsetAsync(counter, 0, sizeof(int), s));
  auto one = [&](const float* Uin, float* Uout) -> int {
    int rc = drsa_amd_drsa_partial(A, C, N, d, K, Uin, gs, ws, ws_size, stream);
    if (rc) return rc;
    return dispatch_finish(gs, (double)N, d, K, Uin, Uout, f_traj, counter, 1, 0, kPolarTol,
                           kPolarMaxIter, nullptr, s);
  };
  int done = 0;
  if (use_graph && steps >= 2) {
    // capture U_io -> U_tmp -> U_io
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    DRSA_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    int rc1 = one(U_io, U_tmp);
    int rc2 = rc1 ? rc1 : one(U_tmp, U_io);
    hipError_t ce = hipStreamEndCapture(s, &graph);
    if (rc2) { if (graph) (void)hipGraphDestroy(graph); return rc2; }
    DRSA_HIP(ce);
    DRSA_HIP(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    for (; done + 2 <= steps; done += 2) {
      hipError_t le = hipGraphLaunch(exec, s);
      if (le != hipSuccess) { (void)hipGraphExecDestroy(exec); (void)hipGraphDestroy(graph); DRSA_HIP(le); }
    }
    (void)hipGraphExecDestroy(exec);
    (void)hipGraphDestroy(graph);
  }
  for (; done + 2 <= steps; done += 2) {
    int rc = one(U_io, U_tmp);
    if (rc) return rc;
    rc = one(U_tmp, U_io);
    if (rc) return rc;
  }
  if (done < steps) {
    int rc = one(U_io, U_tmp);
    if (rc) return rc;
    DRSA_HIP(hipMemcpyAsync(U_io, U_tmp, (size_t)d * d * sizeof(float), hipMemcpyDeviceToDevice, s));
    ++done;
  }
  // final objective -> f_traj[steps]
  int rc = drsa_amd_drsa_partial(A, C, N, d, K, U_io, gs, ws, ws_size, stream);
  if (rc) return rc;
  return dispatch_finish(gs, (double)N, d, K, U_io, nullptr, f_traj, counter, 1, 1, kPolarTol,
                         kPolarMaxIter, nullptr, s);
}

// P independent problems (e.g. the C5 joint optimisation of two layers, optsubspaces.py:18-23
// run one after the other in the reference) advanced together: per step every problem's
// partial/reduce/finish chain runs on its own forked stream inside ONE captured hipGraph, so
// the latency-bound single-workgroup finish kernels of different problems overlap and the
// whole S-step joint loop is one graph launch per two steps.
int drsa_amd_drsa_run_multi(int P, const drsa_amd_problem_t* probs, int steps, int use_graph, void* stream) {
  DRSA_REQUIRE(P >= 1 && P <= 64 && probs, "drsa_run_multi: P must be in [1, 64]");
  DRSA_REQUIRE(steps >= 0, "drsa_run_multi: steps < 0");
  for (int p = 0; p < P; ++p) {
    const drsa_amd_problem_t& q = probs[p];
    DRSA_REQUIRE(supported_dims(q.d, q.K), "drsa_run_multi: problem %d unsupported d=%d K=%d", p, q.d, q.K);
    DRSA_REQUIRE(q.N > 0 && q.A && q.C && q.U_io && q.U_tmp && q.f_traj && q.counter && q.ws,
                 "drsa_run_multi: problem %d has null pointers or N <= 0", p);
    DRSA_REQUIRE(q.ws_size >= ws_bytes(q.N, q.d, q.K), "drsa_run_multi: problem %d workspace too small", p);
    DRSA_REQUIRE(q.dtype == 0 || (q.dtype == 1 && q.d >= 32), "drsa_run_multi: problem %d: dtype must be 0 (fp32) "
                 "or 1 (bf16, d >= 32)", p);
  }
  bool all_f32 = true;
  for (int p = 0; p < P; ++p) all_f32 = all_f32 && probs[p].dtype == 0;
  if (all_f32 && (P == 1 || !use_graph || steps < 2)) {
    for (int p = 0; p < P; ++p) {
      const drsa_amd_problem_t& q = probs[p];
      int rc = drsa_amd_drsa_run(q.A, q.C, q.N, q.d, q.K, q.U_io, q.U_tmp, steps, q.f_traj, q.counter, q.ws,
                                 q.ws_size, use_graph, stream);
      if (rc) return rc;
    }
    return DRSA_OK;
  }
  hipStream_t s = (hipStream_t)stream;
  hipStream_t side[64] = {nullptr};
  hipEvent_t ev_fork = nullptr, ev_join[64] = {nullptr};
  int rc = DRSA_OK;
  auto cleanup = [&]() {
    for (int p = 0; p < P; ++p) {
      if (side[p]) (void)hipStreamDestroy(side[p]);
      if (ev_join[p]) (void)hipEventDestroy(ev_join[p]);
    }
    if (ev_fork) (void)hipEventDestroy(ev_fork);
  };
  auto hip_ok = [&](hipError_t e, const char* what) -> bool {
    if (e == hipSuccess) return true;
    drsa::set_error("drsa_run_multi: %s: %s", what, hipGetErrorString(e));
    rc = (int)e;
    return false;
  };
  if (!hip_ok(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming), "event")) { cleanup(); return rc; }
  for (int p = 0; p < P; ++p) {
    if (!hip_ok(hipStreamCreateWithFlags(&side[p], hipStreamNonBlocking), "stream") ||
        !hip_ok(hipEventCreateWithFlags(&ev_join[p], hipEventDisableTiming), "event")) {
      cleanup();
      return rc;
    }
    const drsa_amd_problem_t& q = probs[p];
    if (!hip_ok(hipMemsetAsync(q.counter, 0, sizeof(int), s), "memset")) { cleanup(); return rc; }
  }
  // one step of problem p on stream st: U_in -> U_out, f -> f_traj[counter++]
  auto one = [&](int p, hipStream_t st, const float* Uin, float* Uout) -> int {
    const drsa_amd_problem_t& q = probs[p];
    const PartialPlan pl = plan_partial(q.N, q.d);
    float* gs = (float*)q.ws + (size_t)pl.grid * ((size_t)q.d * q.d + q.K);
    int r = partial_impl(q.A, q.C, q.N, q.d, q.K, Uin, gs, q.ws, q.ws_size, st, q.dtype);
    if (r) return r;
    return dispatch_finish(gs, (double)q.N, q.d, q.K, Uin, Uout, q.f_traj, q.counter, 1, Uout ? 0 : 1, kPolarTol,
                           kPolarMaxIter, nullptr, st);
  };
  // fork -> per-problem body -> join, captured from stream s
  auto forked = [&](int nsteps_body, bool final_objective) -> int {
    if (!hip_ok(hipEventRecord(ev_fork, s), "record")) return rc;
    for (int p = 0; p < P; ++p) {
      if (!hip_ok(hipStreamWaitEvent(side[p], ev_fork, 0), "wait")) return rc;
      const drsa_amd_problem_t& q = probs[p];
      for (int k = 0; k < nsteps_body; ++k) {
        int r = (k % 2 == 0) ? one(p, side[p], q.U_io, q.U_tmp) : one(p, side[p], q.U_tmp, q.U_io);
        if (r) return r;
      }
      if (final_objective) {
        int r = one(p, side[p], q.U_io, nullptr);
        if (r) return r;
      }
      if (!hip_ok(hipEventRecord(ev_join[p], side[p]), "record")) return rc;
      if (!hip_ok(hipStreamWaitEvent(s, ev_join[p], 0), "wait")) return rc;
    }
    return DRSA_OK;
  };
  int done = 0;
  if (use_graph && steps >= 2) {
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    if (!hip_ok(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal), "capture")) { cleanup(); return rc; }
    int rbody = forked(2, false);
    hipError_t ce = hipStreamEndCapture(s, &graph);
    if (rbody || !hip_ok(ce, "end capture") ||
        !hip_ok(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0), "instantiate")) {
      if (graph) (void)hipGraphDestroy(graph);
      cleanup();
      return rbody ? rbody : rc;
    }
    for (; done + 2 <= steps; done += 2)
      if (!hip_ok(hipGraphLaunch(exec, s), "graph launch")) break;
    (void)hipGraphExecDestroy(exec);
    (void)hipGraphDestroy(graph);
    if (rc) { cleanup(); return rc; }
  } else {
    for (; done + 2 <= steps; done += 2) {
      int r = forked(2, false);
      if (r) { cleanup(); return r; }
    }
  }
  // odd tail step + final objective, eager on the forked streams
  if (done < steps) {
    if (!hip_ok(hipEventRecord(ev_fork, s), "record")) { cleanup(); return rc; }
    for (int p = 0; p < P; ++p) {
      const drsa_amd_problem_t& q = probs[p];
      if (!hip_ok(hipStreamWaitEvent(side[p], ev_fork, 0), "wait")) { cleanup(); return rc; }
      int r = one(p, side[p], q.U_io, q.U_tmp);
      if (r) { cleanup(); return r; }
      if (!hip_ok(hipMemcpyAsync(q.U_io, q.U_tmp, (size_t)q.d * q.d * sizeof(float), hipMemcpyDeviceToDevice,
                                 side[p]), "copy")) { cleanup(); return rc; }
      if (!hip_ok(hipEventRecord(ev_join[p], side[p]), "record") || !hip_ok(hipStreamWaitEvent(s, ev_join[p], 0), "wait")) {
        cleanup();
        return rc;
      }
    }
  }
  int r = forked(0, true);
  if (r) { cleanup(); return r; }
  // make sure nothing is pending on the side streams before they are destroyed
  for (int p = 0; p < P; ++p) (void)hipStreamSynchronize(side[p]);
  cleanup();
  return DRSA_OK;
}

int drsa_amd_polar(const float* V, int d, float* U_out, int* iters_out, void* stream) {
  DRSA_REQUIRE(d == 16 || d == 32 || d == 64 || d == 128, "polar: unsupported d=%d", d);
  hipStream_t s = (hipStream_t)stream;
  auto go = [&](auto tag) -> int {
    constexpr int D = decltype(tag)::value;
    const size_t lds = finish_lds<D>();
    static bool set = false;
    if (!set) {
      DRSA_HIP(hipFuncSetAttribute((const void*)polar_kernel<D>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)lds));
      set = true;
    }
    hipLaunchKernelGGL(polar_kernel<D>, dim3(1), dim3(polar_waves<D>() * 64), lds, s, V, U_out, kPolarTol, kPolarMaxIter,
                       iters_out);
    DRSA_LAUNCH_CHECK();
    return DRSA_OK;
  };
  switch (d) {
    case 16: return go(std::integral_constant<int, 16>{});
    case 32: return go(std::integral_constant<int, 32>{});
    case 64: return go(std::integral_constant<int, 64>{});
    default: return go(std::integral_constant<int, 128>{});
  }
}

int drsa_amd_subspace_relevances(const float* act, const float* ctx, int64_t B, int64_t N, int d, int K,
                                 const float* U, float* out, void* stream) {
  DRSA_REQUIRE(d == 16 || d == 32 || d == 64 || d == 128, "subspace_relevances: unsupported d=%d", d);
  DRSA_REQUIRE(K > 0 && K <= 128 && d % K == 0, "subspace_relevances: K must divide d");
  hipStream_t s = (hipStream_t)stream;
  auto go = [&](auto tag) -> int {
    constexpr int D = decltype(tag)::value;
    const size_t lds = ((size_t)D * D + 256 * (size_t)K) * sizeof(float);
    DRSA_HIP(hipFuncSetAttribute((const void*)subspace_relevance_kernel<D>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(subspace_relevance_kernel<D>, dim3((unsigned)B), dim3(256), lds, s, act, ctx, N, K, U, out);
    DRSA_LAUNCH_CHECK();
    return DRSA_OK;
  };
  switch (d) {
    case 16: return go(std::integral_constant<int, 16>{});
    case 32: return go(std::integral_constant<int, 32>{});
    case 64: return go(std::integral_constant<int, 64>{});
    default: return go(std::integral_constant<int, 128>{});
  }
}

}  // extern "C"

