// Standalone probe: phase timestamps (s_memtime) of the production Newton-Schulz polar
// (csrc/polar_ns.h) at d = 64 and 128 on a near-orthogonal V.  hipcc -O3 --offload-arch=gfx950
// -ffp-contract=off -I drsa_audio_amd/csrc -I include scripts/probe_ns.hip -o /tmp/probe_ns
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
__device__ unsigned long long* g_stamps;
#define DRSA_NS_STAMP(slot) do { if (threadIdx.x == 0 && (slot) < 200) g_stamps[(slot)] = wall_clock64(); } while (0)
#include "polar_ns.h"
namespace drsa { void set_error(const char*, ...) {} }

template <int DP>
__global__ __launch_bounds__(fin_threads<DP>()) void probe_kernel(const float* V, float* U, unsigned long long* st,
                                                                  int* iters) {
  constexpr int NT = fin_threads<DP>(), LD = ns_ld<DP>();
  extern __shared__ float smem[];
  if (threadIdx.x == 0) { g_stamps = st; st[199] = wall_clock64(); }
  __syncthreads();
  float* X = smem; float* T = X + DP * LD; float* red = T + DP * LD; float* scr = red + 64;
  for (int e = threadIdx.x; e < DP * DP; e += NT) X[(e / DP) * LD + e % DP] = V[e];
  int it = polar_run<DP>(X, T, red, scr, 4e-7f, 40);
  for (int e = threadIdx.x; e < DP * DP; e += NT) U[e] = X[(e / DP) * LD + e % DP];
  if (threadIdx.x == 0) { *iters = it; st[198] = wall_clock64(); }
}

template <int DP>
void run() {
  const size_t lds = (2 * (size_t)DP * ns_ld<DP>() + 64 + ns_scratch_floats<DP>()) * 4;
  float* hV = (float*)malloc(DP * DP * 4);
  srand(DP);
  for (int i = 0; i < DP; ++i)
    for (int j = 0; j < DP; ++j) hV[i * DP + j] = (i == j ? 1.1f : 0.f) + 0.1f * ((rand() / (float)RAND_MAX) - 0.5f);
  float *V, *U; unsigned long long* st; int* it;
  hipMalloc(&V, DP * DP * 4); hipMalloc(&U, DP * DP * 4); hipMalloc(&st, 200 * 8); hipMalloc(&it, 4);
  hipMemcpy(V, hV, DP * DP * 4, hipMemcpyHostToDevice);
  hipFuncSetAttribute((const void*)probe_kernel<DP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    hipMemset(st, 0, 200 * 8);
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe_kernel<DP>, dim3(1), dim3(fin_threads<DP>()), lds, 0, V, U, st, it);
    hipEventRecord(e1);
    hipDeviceSynchronize();
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[200]; int hit;
    hipMemcpy(h, st, 200 * 8, hipMemcpyDeviceToHost); hipMemcpy(&hit, it, 4, hipMemcpyDeviceToHost);
    float* hU = (float*)malloc(DP * DP * 4);
    hipMemcpy(hU, U, DP * DP * 4, hipMemcpyDeviceToHost);
    double orth = 0;
    for (int i = 0; i < DP; ++i)
      for (int j = 0; j < DP; ++j) {
        double acc = 0;
        for (int k = 0; k < DP; ++k) acc += (double)hU[k * DP + i] * hU[k * DP + j];
        orth = fmax(orth, fabs(acc - (i == j ? 1.0 : 0.0)));
      }
    free(hU);
    printf("DP=%d rep %d: event %.2f us, iters %d, kernel ticks %llu, max|U^T U - I| %.2e\n", DP, rep, ms * 1e3, hit,
           h[198] - h[199], orth);
    unsigned long long prev = h[199];
    for (int s = 0; s < 4 * (hit + 1) && s < 196; ++s) {
      if (!h[s]) continue;
      printf("  it %d phase %d: +%llu ticks\n", s / 4, s % 4, h[s] - prev);
      prev = h[s];
    }
  }
}

int main() {
  run<64>();
  run<128>();
  return 0;
}
