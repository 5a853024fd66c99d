// DRSA training-data extraction (SURVEY.md §8 row R16, rank 1 of §8f): activation and relevance
// capture at layer j, location sampling, context vectors and normalisation, on device.
//
// Reference: cxai/xai/drsa/preprocessing.py:18-89 (preprocess_data), :106-176 (get_intermediate:
// activation = layer output, relevance = layer.output.grad under the LRP hooks), :179-193
// (compute_context_vectors), :196-216 (sample_spatial_locations), :219-231 (normalize_vectors),
// :234-256 (get_vectors_from_maps); cxai/xai/drsa/cluster/getdrsadata.py:47-59
// (load_and_normalize_data).
//
// The LRP backward stops at layer j and hands over the relevance at the layer's output in the
// engine's native form: at pool resolution plus the pool argmax byte when a 2x2 max-pool
// follows the ReLU (relevance reaches a pooled ReLU output only at the argmax).  The
// extraction kernel reads the activation and that sparse relevance only at the sampled
// locations, so the [B, d, H, W] relevance map of the reference is never materialised.
#include "common.h"
#include "drsa_amd.h"

namespace {

// relevance at flat location p of channel map (b, c) from a full map or a pooled map + argmax
// (ph x pw max-pool; argmax byte = dy * pw + dx, the first maximum in row-major window order)
__device__ __forceinline__ float rel_at(const float* __restrict__ rel, const uint8_t* __restrict__ amax, size_t bc,
                                        size_t bc_amax, int p, int H, int W, int ph, int pw) {
  if (!amax) return rel[bc * (size_t)(H * W) + p];
  const int y = p / W, x = p % W;
  const int W2 = W / pw, H2 = H / ph;
  const size_t cell = (size_t)(y / ph) * W2 + (x / pw);
  return ((int)amax[bc_amax * (size_t)(H2 * W2) + cell] == (y % ph) * pw + (x % pw)) ? rel[bc * (size_t)(H2 * W2) + cell]
                                                                                     : 0.f;
}

// layout 0: get_vectors_from_maps exactly as the reference (preprocessing.py:251-255): the
//   [b, L, d] gather is transposed to [b, d, L] and re-read as rows of d (channel and location
//   interleave; DESIGN.md defect D12);  layout 1: row (b, l) = the d-vector at location l;
//   idx == NULL: every location, [b, H*W, d] (preprocessing.py:80-85, inference branch).
__global__ __launch_bounds__(256) void drsa_vectors_kernel(const float* __restrict__ act, const float* __restrict__ rel,
                                                           const uint8_t* __restrict__ amax,
                                                           const int* __restrict__ idx, int B, int C, int H, int W,
                                                           int ph, int pw, int L, int layout, float* __restrict__ A_out,
                                                           float* __restrict__ C_out) {
  const int64_t total = (int64_t)B * L * C;
  for (int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x; o < total; o += (int64_t)gridDim.x * 256) {
    const int b = (int)(o / ((int64_t)L * C));
    const int rem = (int)(o % ((int64_t)L * C));
    int ch, l;
    if (layout == 0) {
      ch = rem / L;
      l = rem % L;
    } else {
      l = rem / C;
      ch = rem % C;
    }
    const int p = idx ? idx[(size_t)b * L + l] : l;
    const size_t bc = (size_t)b * C + ch;
    const float a = act[bc * (size_t)(H * W) + p];
    const float r = rel_at(rel, amax, bc, bc, p, H, W, ph, pw);
    A_out[o] = a;
    C_out[o] = r / (a + 1e-7f);      // compute_context_vectors
  }
}

// relevance (or rule-divided g) at full resolution from the pooled form: get_intermediate's
// layer.output.grad, and the engine's max-pool backward for pools other than 2x2.  Rows of rel
// are sample*clones + clone; amax is per sample.
__global__ __launch_bounds__(256) void unpool_kernel(const float* __restrict__ rel, const uint8_t* __restrict__ amax,
                                                     int64_t BC, int C, int clones, int H, int W, int ph, int pw,
                                                     float* __restrict__ out) {
  const int64_t total = BC * H * W;
  for (int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x; o < total; o += (int64_t)gridDim.x * 256) {
    const size_t bc = (size_t)(o / (H * W));
    const size_t bca = (bc / C) / clones * C + bc % C;
    out[o] = rel_at(rel, amax, bc, bca, (int)(o % (H * W)), H, W, ph, pw);
  }
}

// ph x pw max-pool (stride = kernel) of a full-resolution activation with the engine's argmax
// byte (first maximum in row-major window order, NaN wins: torch max_pool2d) and the rule
// denominator gathered at the argmax — the tensors the fused conv+2x2-pool epilogue writes.
__global__ __launch_bounds__(256) void maxpool_capture_kernel(const float* __restrict__ a, const float* __restrict__ den,
                                                              int64_t BC, int H, int W, int ph, int pw,
                                                              float* __restrict__ y, uint8_t* __restrict__ amax,
                                                              float* __restrict__ den_p) {
  const int H2 = H / ph, W2 = W / pw;
  const int64_t total = BC * H2 * W2;
  for (int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x; o < total; o += (int64_t)gridDim.x * 256) {
    const size_t bc = (size_t)(o / (H2 * W2));
    const int rem = (int)(o % (H2 * W2));
    const int qy = rem / W2, qx = rem % W2;
    const size_t base = bc * (size_t)(H * W) + (size_t)(ph * qy) * W + pw * qx;
    int am = 0;
    size_t amoff = 0;
    float m = a[base];
    for (int s = 1; s < ph * pw; ++s) {
      const size_t off = (size_t)(s / pw) * W + (s % pw);
      const float v = a[base + off];
      if (v > m || (v != v && m == m)) {
        m = v;
        am = s;
        amoff = off;
      }
    }
    y[o] = m;
    amax[o] = (uint8_t)am;
    if (den) den_p[o] = den[base + amoff];
  }
}

// normalize_vectors: v / sqrt(mean(v^2)) / d^(1/4) over ALL elements.  Deterministic: fixed
// per-block fp64 partial sums, re-reduced in block order by every block of the scale pass.
constexpr int NV_BLOCKS = 512;
__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ v, int64_t n, double* __restrict__ part) {
  __shared__ double red[4];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double x = v[i];
    s += x * x;
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane_id() == 0) red[wave_id()] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// the block partials re-reduced in a fixed order (wave 0: stride-64 chains, then a shuffle tree)
__device__ double reduce_parts(const double* __restrict__ part, int nblk) {
  double s = 0.0;
  for (int i = threadIdx.x; i < nblk; i += 64) s += part[i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  return s;
}

// one fp64 sum of squares per call (the sharded normalisation's local term)
__global__ __launch_bounds__(64) void sumsq_finish_kernel(const double* __restrict__ part, int nblk,
                                                          double* __restrict__ sum_out) {
  const double s = reduce_parts(part, nblk);
  if (threadIdx.x == 0) sum_out[0] = s;
}

// E = sqrt((sums[0] + sums[1] + ... in rank order) / n_total); the scale over this call's elements.
// nsums == 0: the sum is this call's own block partials (single-process normalize_vectors).
__global__ __launch_bounds__(256) void scale_kernel(const float* __restrict__ v, int64_t n, float d4, int nblk,
                                                    const double* __restrict__ part, const double* __restrict__ sums,
                                                    int nsums, double n_total, float* __restrict__ out) {
  __shared__ float sc;
  if (threadIdx.x < 64) {
    double s;
    if (nsums == 0) {
      s = reduce_parts(part, nblk);
    } else {
      s = 0.0;
      for (int r = 0; r < nsums; ++r) s += sums[r];
    }
    if (threadIdx.x == 0) sc = (float)sqrt(s / n_total);
  }
  __syncthreads();
  const float E = sc;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    out[i] = v[i] / E / d4;         // preprocessing.py:231: vectors / E / d**0.25
}

int grid_for(int64_t total) {
  int64_t g = (total + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace

extern "C" int drsa_amd_maxpool_capture(const float* a, const float* den, float* y, uint8_t* amax, float* den_pooled,
                                        int B, int C, int H, int W, int ph, int pw, void* stream) {
  DRSA_REQUIRE(a && y && amax, "maxpool_capture: null pointer");
  DRSA_REQUIRE(!den || den_pooled, "maxpool_capture: den needs den_pooled");
  DRSA_REQUIRE(ph >= 1 && pw >= 1 && ph * pw <= 256, "maxpool_capture: bad pool kernel %dx%d", ph, pw);
  DRSA_REQUIRE(B >= 0 && C > 0 && H > 0 && W > 0 && H % ph == 0 && W % pw == 0, "maxpool_capture: bad shape");
  if (B == 0) return DRSA_OK;
  const int64_t BC = (int64_t)B * C;
  hipLaunchKernelGGL(maxpool_capture_kernel, dim3(grid_for(BC * (H / ph) * (W / pw))), dim3(256), 0,
                     (hipStream_t)stream, a, den, BC, H, W, ph, pw, y, amax, den_pooled);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

extern "C" int drsa_amd_relevance_unpool(const float* rel, const uint8_t* amax, int Bq, int clones, int C, int H, int W,
                                         int ph, int pw, float* out, void* stream) {
  DRSA_REQUIRE(rel && amax && out, "relevance_unpool: null pointer");
  DRSA_REQUIRE(clones >= 1 && Bq % clones == 0, "relevance_unpool: bad clones");
  DRSA_REQUIRE(ph >= 1 && pw >= 1 && ph * pw <= 256, "relevance_unpool: bad pool kernel");
  DRSA_REQUIRE(Bq >= 0 && C > 0 && H % ph == 0 && W % pw == 0, "relevance_unpool: bad shape");
  if (Bq == 0) return DRSA_OK;
  const int64_t BC = (int64_t)Bq * C;
  hipLaunchKernelGGL(unpool_kernel, dim3(grid_for(BC * H * W)), dim3(256), 0, (hipStream_t)stream, rel, amax, BC, C,
                     clones, H, W, ph, pw, out);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

extern "C" int drsa_amd_drsa_vectors(const float* act, const float* rel, const uint8_t* rel_amax, const int* idx,
                                     int B, int C, int H, int W, int ph, int pw, int L, int layout, float* A_out,
                                     float* C_out, void* stream) {
  DRSA_REQUIRE(act && rel && A_out && C_out, "drsa_vectors: null pointer");
  DRSA_REQUIRE(B >= 0 && C > 0 && H > 0 && W > 0, "drsa_vectors: bad shape");
  DRSA_REQUIRE(!rel_amax || (ph >= 1 && pw >= 1 && H % ph == 0 && W % pw == 0),
               "drsa_vectors: pooled relevance needs H, W divisible by the pool kernel");
  DRSA_REQUIRE(layout == 0 || layout == 1, "drsa_vectors: layout must be 0 (reference) or 1 (rows)");
  if (!idx) {
    DRSA_REQUIRE(L == H * W, "drsa_vectors: idx == NULL takes every location (L must be H*W)");
    layout = 1;
  } else {
    DRSA_REQUIRE(L >= 1 && L <= H * W, "drsa_vectors: L must be in [1, H*W]");
  }
  if (B == 0) return DRSA_OK;
  hipLaunchKernelGGL(drsa_vectors_kernel, dim3(grid_for((int64_t)B * L * C)), dim3(256), 0, (hipStream_t)stream, act,
                     rel, rel_amax, idx, B, C, H, W, ph, pw, L, layout, A_out, C_out);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

extern "C" size_t drsa_amd_normalize_workspace_bytes(void) { return NV_BLOCKS * sizeof(double); }

extern "C" int drsa_amd_normalize_vectors(const float* v, int64_t n, int d, float* out, void* ws, size_t ws_bytes,
                                          void* stream) {
  DRSA_REQUIRE(v && out && ws, "normalize_vectors: null pointer");
  DRSA_REQUIRE(n > 0 && d > 0, "normalize_vectors: empty input");
  DRSA_REQUIRE(ws_bytes >= NV_BLOCKS * sizeof(double), "normalize_vectors: workspace too small");
  const int64_t nb = (n + 255) / 256;
  const int nblk = (int)(nb < NV_BLOCKS ? nb : NV_BLOCKS);
  const float d4 = (float)pow((double)d, 0.25);
  hipLaunchKernelGGL(sumsq_kernel, dim3(nblk), dim3(256), 0, (hipStream_t)stream, v, n, (double*)ws);
  DRSA_LAUNCH_CHECK();
  hipLaunchKernelGGL(scale_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, v, n, d4, nblk,
                     (const double*)ws, (const double*)nullptr, 0, (double)n, out);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

extern "C" int drsa_amd_normalize_sumsq(const float* v, int64_t n, void* ws, size_t ws_bytes, double* sum_out,
                                        void* stream) {
  DRSA_REQUIRE(ws && sum_out, "normalize_sumsq: null pointer");
  DRSA_REQUIRE(n >= 0 && (n == 0 || v), "normalize_sumsq: bad input");
  DRSA_REQUIRE(ws_bytes >= NV_BLOCKS * sizeof(double), "normalize_sumsq: workspace too small");
  if (n == 0) {                     // a rank without rows contributes 0
    DRSA_HIP(hipMemsetAsync(sum_out, 0, sizeof(double), (hipStream_t)stream));
    return DRSA_OK;
  }
  const int64_t nb = (n + 255) / 256;
  const int nblk = (int)(nb < NV_BLOCKS ? nb : NV_BLOCKS);
  hipLaunchKernelGGL(sumsq_kernel, dim3(nblk), dim3(256), 0, (hipStream_t)stream, v, n, (double*)ws);
  DRSA_LAUNCH_CHECK();
  hipLaunchKernelGGL(sumsq_finish_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (const double*)ws, nblk,
                     sum_out);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

extern "C" int drsa_amd_normalize_scale(const float* v, int64_t n, int d, const double* sums, int nsums,
                                        int64_t n_total, float* out, void* stream) {
  DRSA_REQUIRE(sums && nsums >= 1, "normalize_scale: needs >= 1 partial sum");
  DRSA_REQUIRE(n >= 0 && d > 0 && n_total > 0 && n <= n_total, "normalize_scale: bad sizes");
  DRSA_REQUIRE(n == 0 || (v && out), "normalize_scale: null pointer");
  if (n == 0) return DRSA_OK;
  const float d4 = (float)pow((double)d, 0.25);
  hipLaunchKernelGGL(scale_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, v, n, d4, 0,
                     (const double*)nullptr, sums, nsums, (double)n_total, out);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}
