// Standalone probe: slab-reduce variants timed right after a real drsa_partial launch (so the
// slabs are dirty in the producers' L2s, as in the step).  C3 (N=20000, d=64, K=4) and d=128.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "runtime.hip"
#include "drsa_step.hip"

// (a) one thread per element, 4 chains over 256 threads (round-2 first version)
__global__ __launch_bounds__(256) void red_a(const float* __restrict__ partials, int P, int E, int ES, float* out) {
  __shared__ float part[4][64];
  const int l = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + l;
  float acc = 0.f;
  if (e < E) {
#pragma unroll 8
    for (int p = grp; p < P; p += 4) acc += partials[(size_t)p * ES + e];
  }
  part[grp][l] = acc;
  __syncthreads();
  if (grp == 0 && e < E) out[e] = ((part[0][l] + part[1][l]) + part[2][l]) + part[3][l];
}
// (b) slab-split grid: blockIdx.y = quarter; quarter sums written separately
template <int Q>
__global__ __launch_bounds__(256) void red_b(const float* __restrict__ partials, int P, int E, int ES, float* out) {
  __shared__ float part[4][64];
  const int l = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + l;
  const int per = P / Q, p0 = blockIdx.y * per;
  float acc = 0.f;
  if (e < E) {
#pragma unroll 16
    for (int p = p0 + grp; p < p0 + per; p += 4) acc += partials[(size_t)p * ES + e];
  }
  part[grp][l] = acc;
  __syncthreads();
  if (grp == 0 && e < E) out[(size_t)blockIdx.y * E + e] = ((part[0][l] + part[1][l]) + part[2][l]) + part[3][l];
}

static void run(int N, int d, int K) {
  float *A, *C, *U;
  hipMalloc(&A, (size_t)N * d * 4); hipMalloc(&C, (size_t)N * d * 4); hipMalloc(&U, d * d * 4);
  float* h = (float*)malloc((size_t)N * d * 4);
  for (size_t i = 0; i < (size_t)N * d; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f;
  hipMemcpy(A, h, (size_t)N * d * 4, hipMemcpyHostToDevice);
  hipMemcpy(C, h, (size_t)N * d * 4, hipMemcpyHostToDevice);
  for (int i = 0; i < d * d; ++i) h[i] = (i % (d + 1)) == 0 ? 1.f : 0.f;
  hipMemcpy(U, h, d * d * 4, hipMemcpyHostToDevice);
  const Geom g = geom(d, K);
  const PartialPlan pl = plan_partial(N);
  const int E = (int)slab_floats(g), ES = (int)slab_stride(g);
  size_t ws = drsa_amd_drsa_workspace_bytes(N, d, K);
  void* w; hipMalloc(&w, ws);
  float* out; hipMalloc(&out, (size_t)8 * E * 4);
  hipEvent_t e0, e1, e2; hipEventCreate(&e0); hipEventCreate(&e1); hipEventCreate(&e2);
  for (int variant = 0; variant < 5; ++variant) {
    float tp = 0, tr = 0;
    for (int rep = 0; rep < 6; ++rep) {
      hipEventRecord(e0);
      dispatch_partial(A, C, N, g, U, (float*)w, pl, 0, false);
      hipEventRecord(e1);
      if (variant == 0)
        hipLaunchKernelGGL(drsa_reduce_kernel, dim3((E + 63) / 64), dim3(256), 0, 0, (float*)w, pl.grid, E, ES, out);
      else if (variant == 1)
        hipLaunchKernelGGL(red_a, dim3((E + 63) / 64), dim3(256), 0, 0, (float*)w, pl.grid, E, ES, out);
      else if (variant == 2)
        hipLaunchKernelGGL(red_b<4>, dim3((E + 63) / 64, 4), dim3(256), 0, 0, (float*)w, pl.grid, E, ES, out);
      else if (variant == 3)
        hipLaunchKernelGGL(red_b<8>, dim3((E + 63) / 64, 8), dim3(256), 0, 0, (float*)w, pl.grid, E, ES, out);
      else
        hipLaunchKernelGGL(red_b<2>, dim3((E + 63) / 64, 2), dim3(256), 0, 0, (float*)w, pl.grid, E, ES, out);
      hipEventRecord(e2);
      hipDeviceSynchronize();
      float a, b; hipEventElapsedTime(&a, e0, e1); hipEventElapsedTime(&b, e1, e2);
      if (rep >= 2) { tp += a; tr += b; }
    }
    printf("N=%d d=%d K=%d grid=%d variant %d: partial %.2f us, reduce %.2f us\n", N, d, K, pl.grid, variant,
           tp / 4 * 1e3, tr / 4 * 1e3);
  }
}

int main() {
  run(20000, 64, 4);
  run(20000, 128, 16);
  return 0;
}
