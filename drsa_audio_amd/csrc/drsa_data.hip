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
__device__ __forceinline__ float rel_at(const float* __restrict__ rel, const uint8_t* __restrict__ amax, size_t bc,
                                        int p, int H, int W) {
  if (!amax) return rel[bc * (size_t)(H * W) + p];
  const int y = p / W, x = p % W;
  const int W2 = W >> 1, H2 = H >> 1;
  const size_t q = bc * (size_t)(H2 * W2) + (size_t)(y >> 1) * W2 + (x >> 1);
  return ((int)amax[q] == ((y & 1) << 1 | (x & 1))) ? rel[q] : 0.f;
}

// layout 0: get_vectors_from_maps exactly as the reference (preprocessing.py:251-255): the
//   [b, L, d] gather is transposed to [b, d, L] and re-read as rows of d (channel and location
//   interleave; DESIGN.md defect D12);  layout 1: row (b, l) = the d-vector at location l;
//   idx == NULL: every location, [b, H*W, d] (preprocessing.py:80-85, inference branch).
__global__ __launch_bounds__(256) void drsa_vectors_kernel(const float* __restrict__ act, const float* __restrict__ rel,
                                                           const uint8_t* __restrict__ amax,
                                                           const int* __restrict__ idx, int B, int C, int H, int W,
                                                           int L, int layout, float* __restrict__ A_out,
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
    const float r = rel_at(rel, amax, bc, p, H, W);
    A_out[o] = a;
    C_out[o] = r / (a + 1e-7f);      // compute_context_vectors
  }
}

// relevance map at full resolution from the pooled form (get_intermediate's layer.output.grad)
__global__ __launch_bounds__(256) void unpool_kernel(const float* __restrict__ rel, const uint8_t* __restrict__ amax,
                                                     int64_t BC, int H, int W, float* __restrict__ out) {
  const int64_t total = BC * H * W;
  for (int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x; o < total; o += (int64_t)gridDim.x * 256) {
    const size_t bc = (size_t)(o / (H * W));
    out[o] = rel_at(rel, amax, bc, (int)(o % (H * W)), H, W);
  }
}

// 2x2 max-pool of a full-resolution activation with the engine's argmax byte (first maximum in
// row-major window order, NaN wins: torch max_pool2d) and the rule denominator gathered at the
// argmax — the same tensors the fused conv+pool forward epilogue writes.
__global__ __launch_bounds__(256) void maxpool_capture_kernel(const float* __restrict__ a, const float* __restrict__ den,
                                                              int64_t BC, int H, int W, float* __restrict__ y,
                                                              uint8_t* __restrict__ amax, float* __restrict__ den_p) {
  const int H2 = H >> 1, W2 = W >> 1;
  const int64_t total = BC * H2 * W2;
  for (int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x; o < total; o += (int64_t)gridDim.x * 256) {
    const size_t bc = (size_t)(o / (H2 * W2));
    const int rem = (int)(o % (H2 * W2));
    const int qy = rem / W2, qx = rem % W2;
    const size_t base = bc * (size_t)(H * W) + (size_t)(2 * qy) * W + 2 * qx;
    const size_t off[4] = {0, 1, (size_t)W, (size_t)W + 1};
    int am = 0;
    float m = a[base];
#pragma unroll
    for (int s = 1; s < 4; ++s) {
      const float v = a[base + off[s]];
      if (v > m || (v != v && m == m)) {
        m = v;
        am = s;
      }
    }
    y[o] = m;
    amax[o] = (uint8_t)am;
    if (den) den_p[o] = den[base + off[am]];
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

__global__ __launch_bounds__(256) void scale_kernel(const float* __restrict__ v, int64_t n, float d4, int nblk,
                                                    const double* __restrict__ part, float* __restrict__ out) {
  __shared__ float sc;
  if (threadIdx.x < 64) {           // wave 0 re-reduces the partials in a fixed order
    double s = 0.0;
    for (int i = threadIdx.x; i < nblk; i += 64) s += part[i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (threadIdx.x == 0) sc = (float)sqrt(s / (double)n);
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
                                        int B, int C, int H, int W, void* stream) {
  DRSA_REQUIRE(a && y && amax, "maxpool_capture: null pointer");
  DRSA_REQUIRE(!den || den_pooled, "maxpool_capture: den needs den_pooled");
  DRSA_REQUIRE(B >= 0 && C > 0 && H % 2 == 0 && W % 2 == 0 && H > 0 && W > 0, "maxpool_capture: bad shape");
  if (B == 0) return DRSA_OK;
  const int64_t BC = (int64_t)B * C;
  hipLaunchKernelGGL(maxpool_capture_kernel, dim3(grid_for(BC * (H / 2) * (W / 2))), dim3(256), 0,
                     (hipStream_t)stream, a, den, BC, H, W, y, amax, den_pooled);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

extern "C" int drsa_amd_relevance_unpool(const float* rel, const uint8_t* amax, int B, int C, int H, int W, float* out,
                                         void* stream) {
  DRSA_REQUIRE(rel && amax && out, "relevance_unpool: null pointer");
  DRSA_REQUIRE(B >= 0 && C > 0 && H % 2 == 0 && W % 2 == 0, "relevance_unpool: bad shape");
  if (B == 0) return DRSA_OK;
  const int64_t BC = (int64_t)B * C;
  hipLaunchKernelGGL(unpool_kernel, dim3(grid_for(BC * H * W)), dim3(256), 0, (hipStream_t)stream, rel, amax, BC, H,
                     W, out);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

extern "C" int drsa_amd_drsa_vectors(const float* act, const float* rel, const uint8_t* rel_amax, const int* idx,
                                     int B, int C, int H, int W, int L, int layout, float* A_out, float* C_out,
                                     void* stream) {
  DRSA_REQUIRE(act && rel && A_out && C_out, "drsa_vectors: null pointer");
  DRSA_REQUIRE(B >= 0 && C > 0 && H > 0 && W > 0, "drsa_vectors: bad shape");
  DRSA_REQUIRE(!rel_amax || (H % 2 == 0 && W % 2 == 0), "drsa_vectors: pooled relevance needs even H, W");
  DRSA_REQUIRE(layout == 0 || layout == 1, "drsa_vectors: layout must be 0 (reference) or 1 (rows)");
  if (!idx) {
    DRSA_REQUIRE(L == H * W, "drsa_vectors: idx == NULL takes every location (L must be H*W)");
    layout = 1;
  } else {
    DRSA_REQUIRE(L >= 1 && L <= H * W, "drsa_vectors: L must be in [1, H*W]");
  }
  if (B == 0) return DRSA_OK;
  hipLaunchKernelGGL(drsa_vectors_kernel, dim3(grid_for((int64_t)B * L * C)), dim3(256), 0, (hipStream_t)stream, act,
                     rel, rel_amax, idx, B, C, H, W, L, layout, A_out, C_out);
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
                     (const double*)ws, out);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}
