// compute_subspace_relevances (cxai/xai/explain/explainer.py:206-242) on gfx950:
//   r[b][k] = sum_n sum_{j in block k} (a_n U)_j (c_n U)_j      (no ReLU; blocks of width d/K)
// The reference forms x = (act U) (.) (ctx U), transposes it to [b, d, N] and sums the view
// [b, K, N, d/K] over its last two axes: every (n, j) of concept k's columns, in any order.
//
// Kernel: grid (chunks of kRows rows, instances b); 4 waves, each owning 16-row blocks.  XA, XC
// on fp32 MFMA (16x16x4) with U staged once per workgroup in LDS (zero-padded to DP columns), the
// per-column products accumulated in registers, then a fixed-order combine over waves, lane groups
// and the columns of each concept -> partial[b][chunk][k]; a second kernel sums the chunks in order.
// Any d <= 128 (d = 100: VGGish layer 19) with K | d.
#include "common.h"
#include "drsa_amd.h"

#include <type_traits>

namespace {

constexpr int kRows = 256;   // rows per workgroup (chunk)

template <int DP>
struct SCfg {
  static constexpr int NB = DP / 16;
  static constexpr int LDU = DP + 4;
  static constexpr int LDA = DP + 4;
  static constexpr int STAGE = 2 * 16 * LDA;
  static constexpr size_t lds_floats = (size_t)DP * LDU + 4 * (size_t)STAGE;
  static constexpr size_t lds_bytes = lds_floats * sizeof(float);
};

template <int DP>
__global__ __launch_bounds__(256) void subrel_kernel(const float* __restrict__ act, const float* __restrict__ ctx,
                                                     int64_t N, int d, int K, const float* __restrict__ U,
                                                     float* __restrict__ partial) {
  using Cfg = SCfg<DP>;
  constexpr int NB = Cfg::NB, LDU = Cfg::LDU, LDA = Cfg::LDA, NQ = DP / 16;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Us = smem;                                           // [DP][LDU] (rows, cols >= d zero)
  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  const int l15 = lane & 15, lg = lane >> 4;
  const int chunk = blockIdx.x, b = blockIdx.y, chunks = gridDim.x;
  for (int e = tid; e < DP * DP; e += 256) {
    const int i = e / DP, j = e % DP;
    Us[i * LDU + j] = (i < d && j < d) ? U[(size_t)i * d + j] : 0.f;
  }
  __syncthreads();
  float* As = smem + (size_t)DP * LDU + (size_t)w * Cfg::STAGE;
  float* Cs = As + 16 * LDA;
  const float* A = act + (size_t)b * N * d;
  const float* Cx = ctx + (size_t)b * N * d;
  const int nq_live = (d + 15) / 16;
  float colacc[NB];
#pragma unroll
  for (int cb = 0; cb < NB; ++cb) colacc[cb] = 0.f;

  const int64_t row_lo = (int64_t)chunk * kRows;
  for (int64_t r0 = row_lo + 16 * w; r0 < row_lo + kRows && r0 < N; r0 += 64) {
    for (int i = lane; i < 16 * DP; i += 64) {
      const int row = i / DP, col = i % DP;
      float a = 0.f, c = 0.f;
      if (r0 + row < N && col < d) {
        a = A[(size_t)(r0 + row) * d + col];
        c = Cx[(size_t)(r0 + row) * d + col];
      }
      As[row * LDA + col] = a;
      Cs[row * LDA + col] = c;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    f32x4 xa[NB], xc[NB];
#pragma unroll
    for (int cb = 0; cb < NB; ++cb) { xa[cb] = f32x4{0.f, 0.f, 0.f, 0.f}; xc[cb] = xa[cb]; }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (q >= nq_live) break;
      const float4 a4 = *reinterpret_cast<const float4*>(As + l15 * LDA + 16 * q + 4 * lg);
      const float4 c4 = *reinterpret_cast<const float4*>(Cs + l15 * LDA + 16 * q + 4 * lg);
      const float av[4] = {a4.x, a4.y, a4.z, a4.w}, cv[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int k = 16 * q + 4 * lg + t;
#pragma unroll
        for (int cb = 0; cb < NB; ++cb) {
          const float u = Us[k * LDU + 16 * cb + l15];
          xa[cb] = mfma16(av[t], u, xa[cb]);
          xc[cb] = mfma16(cv[t], u, xc[cb]);
        }
      }
    }
#pragma unroll
    for (int cb = 0; cb < NB; ++cb) {
      float s = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) s += xa[cb][r] * xc[cb][r];
      colacc[cb] += s;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // fixed-order combine: waves, then lane groups (rows), then the columns of each concept
  __syncthreads();
  float* red = smem;                      // [4 waves][64 lanes][NB]
  float* col = smem + 4 * 64 * NB;        // [DP]
#pragma unroll
  for (int cb = 0; cb < NB; ++cb) red[(w * 64 + lane) * NB + cb] = colacc[cb];
  __syncthreads();
  if (tid < DP) {
    const int cb = tid / 16, c15 = tid % 16;
    float acc = 0.f;
    for (int ww = 0; ww < 4; ++ww)
      for (int q = 0; q < 4; ++q) acc += red[(ww * 64 + 16 * q + c15) * NB + cb];
    col[tid] = acc;
  }
  __syncthreads();
  const int dk = d / K;
  for (int k = tid; k < K; k += 256) {
    float acc = 0.f;
    for (int j = k * dk; j < (k + 1) * dk; ++j) acc += col[j];
    partial[((size_t)b * chunks + chunk) * K + k] = acc;
  }
}

__global__ __launch_bounds__(256) void subrel_reduce_kernel(const float* __restrict__ partial, int64_t B, int chunks,
                                                            int K, float* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= B * K) return;
  const int64_t b = e / K, k = e % K;
  float acc = 0.f;
  for (int c = 0; c < chunks; ++c) acc += partial[((size_t)b * chunks + c) * K + k];
  out[e] = acc;
}

int chunks_of(int64_t N) { return (int)((N + kRows - 1) / kRows); }

}  // namespace

extern "C" {

size_t drsa_amd_subspace_relevances_workspace_bytes(int64_t B, int64_t N, int d, int K) {
  if (B <= 0 || N <= 0 || d <= 0 || d > 128 || K <= 0 || d % K) return 0;
  return (size_t)B * chunks_of(N) * K * sizeof(float) + 64;
}

int drsa_amd_subspace_relevances(const float* act, const float* ctx, int64_t B, int64_t N, int d, int K,
                                 const float* U, float* out, void* ws, size_t ws_size, void* stream) {
  DRSA_REQUIRE(d >= 1 && d <= 128, "subspace_relevances: unsupported d=%d (1..128)", d);
  DRSA_REQUIRE(K > 0 && d % K == 0, "subspace_relevances: n_concepts=%d must divide d=%d", K, d);
  DRSA_REQUIRE(B > 0 && N > 0, "subspace_relevances: empty input (B=%lld, N=%lld)", (long long)B, (long long)N);
  DRSA_REQUIRE(B <= 65535, "subspace_relevances: B=%lld exceeds the grid limit 65535", (long long)B);
  DRSA_REQUIRE(act && ctx && U && out && ws, "subspace_relevances: null pointer");
  DRSA_REQUIRE(ws_size >= drsa_amd_subspace_relevances_workspace_bytes(B, N, d, K),
               "subspace_relevances: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int chunks = chunks_of(N);
  float* partial = (float*)ws;
  auto go = [&](auto tag) -> int {
    constexpr int DP = decltype(tag)::value;
    using Cfg = SCfg<DP>;
    DRSA_SMEM(subrel_kernel<DP>, Cfg::lds_bytes);
    hipLaunchKernelGGL(subrel_kernel<DP>, dim3((unsigned)chunks, (unsigned)B), dim3(256), Cfg::lds_bytes, s, act, ctx,
                       N, d, K, U, partial);
    DRSA_LAUNCH_CHECK();
    return DRSA_OK;
  };
  int rc;
  if (d <= 16) rc = go(std::integral_constant<int, 16>{});
  else if (d <= 32) rc = go(std::integral_constant<int, 32>{});
  else if (d <= 64) rc = go(std::integral_constant<int, 64>{});
  else rc = go(std::integral_constant<int, 128>{});
  if (rc) return rc;
  const int64_t E = B * K;
  hipLaunchKernelGGL(subrel_reduce_kernel, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, s, partial, B, chunks, K,
                     out);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

}  // extern "C"
