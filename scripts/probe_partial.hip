// Standalone probe: phase timestamps (wall_clock64, 10 ns) inside the production DRSA partial
// kernel (csrc/drsa_step.hip) for blocks 0 and 128, C3 shape (N=20000, d=64, K=4) and d=128/K=16.
// hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I drsa_audio_amd/csrc -I include
//       scripts/probe_partial.hip -o scripts/probe_partial
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
__device__ unsigned long long g_pst[32];
#define DRSA_PARTIAL_STAMP(slot)                                                              \
  do {                                                                                        \
    if (threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == 128))                           \
      g_pst[(blockIdx.x ? 16 : 0) + (slot)] = wall_clock64();                                 \
  } while (0)
#include "runtime.hip"
#include "drsa_step.hip"

static void run(int N, int d, int K) {
  float *A, *C, *U;
  hipMalloc(&A, (size_t)N * d * 4); hipMalloc(&C, (size_t)N * d * 4); hipMalloc(&U, d * d * 4);
  float* h = (float*)malloc((size_t)N * d * 4);
  for (size_t i = 0; i < (size_t)N * d; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f;
  hipMemcpy(A, h, (size_t)N * d * 4, hipMemcpyHostToDevice);
  hipMemcpy(C, h, (size_t)N * d * 4, hipMemcpyHostToDevice);
  for (int i = 0; i < d * d; ++i) h[i] = (i % (d + 1)) == 0 ? 1.f : 0.f;
  hipMemcpy(U, h, d * d * 4, hipMemcpyHostToDevice);
  size_t ws = drsa_amd_drsa_workspace_bytes(N, d, K);
  void* w; hipMalloc(&w, ws);
  float* gs; hipMalloc(&gs, drsa_amd_drsa_slab_floats(d, K) * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 4; ++rep) {
    unsigned long long z[32] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_pst), z, sizeof(z));
    hipEventRecord(e0);
    int rc = drsa_amd_drsa_partial(A, C, N, d, K, U, gs, w, ws, nullptr);
    hipEventRecord(e1);
    hipDeviceSynchronize();
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long t[32];
    hipMemcpyFromSymbol(t, HIP_SYMBOL(g_pst), sizeof(t));
    printf("N=%d d=%d K=%d rc=%d partial+reduce %.2f us |", N, d, K, rc, ms * 1e3);
    for (int b = 0; b < 2; ++b) {
      printf(" blk%d:", b ? 128 : 0);
      for (int s = 1; s < 7; ++s) printf(" %lld", (long long)(t[16 * b + s] - t[16 * b + s - 1]));
      printf(" (start %+lld)", (long long)(t[16 * b] - t[0]));
    }
    printf("\n");
  }
}

int main() {
  run(20000, 64, 4);
  run(20000, 128, 16);
  return 0;
}
