// Sustained fp32 MFMA rate on this box: v_mfma_f32_32x32x2_f32 back to back on random operands,
// every CU busy at 1..4 waves per SIMD, plus the in-kernel clock (s_memtime / s_memrealtime stamps
// into a buffer of their own).  The achievable ceiling for the fp32 conv kernels' roofline.frac.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/probe_mfma_peak scripts/probe_mfma_peak.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ __launch_bounds__(256) void mfma_loop(const float* __restrict__ seed, float* __restrict__ out,
                                                 unsigned long long* __restrict__ stamps, int iters) {
  const int lane = threadIdx.x & 63;
  float a = seed[(blockIdx.x * 256 + threadIdx.x) & 4095];
  float b = seed[(blockIdx.x * 256 + threadIdx.x + 1234) & 4095];
  f32x16 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = seed[(lane * 16 + r + i * 7) & 4095];
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
    asm volatile("" : "+v"(a), "+v"(b));
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NACC; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[i][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = t1 - t0;
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
}

int main() {
  const int blocks_per_cu_list[] = {1, 2, 3, 4};
  std::vector<float> h(4096);
  unsigned x = 12345;
  for (auto& v : h) { x = x * 1664525u + 1013904223u; v = (float)((x >> 8) & 0xffff) / 65536.f - 0.5f; }
  float *seed, *out;
  unsigned long long* stamps;
  hipMalloc(&seed, 4096 * 4);
  hipMemcpy(seed, h.data(), 4096 * 4, hipMemcpyHostToDevice);
  const int maxb = 256 * 4;
  hipMalloc(&out, (size_t)maxb * 256 * 4);
  hipMalloc(&stamps, (size_t)maxb * 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  for (int bpc : blocks_per_cu_list) {
    const int blocks = 256 * bpc;
    for (int rep = 0; rep < 3; ++rep) mfma_loop<4><<<blocks, 256>>>(seed, out, stamps, iters);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    const int reps = 10;
    for (int rep = 0; rep < reps; ++rep) mfma_loop<4><<<blocks, 256>>>(seed, out, stamps, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> st((size_t)blocks * 2);
    hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> clk;
    for (int i = 0; i < blocks; ++i) clk.push_back((double)st[2 * i] / (double)st[2 * i + 1] * 100.0);   // MHz
    std::sort(clk.begin(), clk.end());
    const double flop = 2.0 * 32 * 32 * 2 * 4.0 * iters * 4 /*waves*/ * blocks * reps;
    printf("{\"waves_per_simd\": %d, \"tflops\": %.1f, \"frac_of_157_3\": %.3f, \"clock_mhz_median\": %.0f}\n", bpc,
           flop / ms / 1e9, flop / ms / 1e9 / 157.3, clk[clk.size() / 2]);
  }
  return 0;
}
