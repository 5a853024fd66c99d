// Shared helpers for the drsa_amd HIP library (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------
// status / error reporting across the C ABI (never throws)
// ---------------------------------------------------------------------------
namespace drsa {
void set_error(const char* fmt, ...);
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (current device, kernel); thread-safe.
int ensure_smem(const void* fn, size_t bytes);
// multiprocessor count of the current device (cached per device); thread-safe.
int cu_count();
}  // namespace drsa

#define DRSA_SMEM(fn, bytes)                                           \
  do {                                                                 \
    int _rc = drsa::ensure_smem((const void*)(fn), (size_t)(bytes));   \
    if (_rc) return _rc;                                               \
  } while (0)

#define DRSA_OK 0
#define DRSA_EINVAL (-1)
#define DRSA_EWORKSPACE (-2)
#define DRSA_EUNSUPPORTED (-3)
#define DRSA_ETIMEOUT (-4)   /* a cooperative kernel's cross-workgroup hand-off timed out (results NaN) */

#define DRSA_REQUIRE(cond, ...)           \
  do {                                    \
    if (!(cond)) {                        \
      drsa::set_error(__VA_ARGS__);       \
      return DRSA_EINVAL;                 \
    }                                     \
  } while (0)

#define DRSA_HIP(call)                                                     \
  do {                                                                     \
    hipError_t _e = (call);                                                \
    if (_e != hipSuccess) {                                                \
      drsa::set_error("%s:%d %s: %s", __FILE__, __LINE__, #call,           \
                      hipGetErrorString(_e));                              \
      return (int)_e;                                                      \
    }                                                                      \
  } while (0)

#define DRSA_LAUNCH_CHECK() DRSA_HIP(hipGetLastError())

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
// fp32-input MFMA, 16x16x4 (exact f32 fma chain, k-ordered).
//   A operand: lane l holds A[i = l&15][k = l>>4]
//   B operand: lane l holds B[k = l>>4][j = l&15]
//   C/D:       lane l, reg r holds C[row = (l>>4)*4 + r][col = l&15]
__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// fp32-input MFMA, 32x32x2.
//   A operand: lane l holds A[i = l&31][k = l>>5]
//   B operand: lane l holds B[k = l>>5][j = l&31]
//   C/D:       lane l, reg r holds C[row = (r&3) + 8*(r>>2) + 4*(l>>5)][col = l&31]
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// bf16-input MFMA, 16x16x32 (gfx950), fp32 accumulate.
//   A operand: lane l holds A[i = l&15][k = 8(l>>4) + j], j < 8 (bf16 bit patterns)
//   B operand: lane l holds B[k = 8(l>>4) + j][col = l&15]
//   C/D:       as mfma16
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x4 mfma16_bf16(u16x8 a, u16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}
// bf16-input MFMA, 32x32x16 (gfx950), fp32 accumulate.
//   A operand: lane l holds A[i = l&31][k = 8(l>>5) + j], j < 8;  B: B[k = 8(l>>5) + j][col = l&31]
//   C/D:       as mfma32
__device__ __forceinline__ f32x16 mfma32_bf16(u16x8 a, u16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}
// two floats -> packed bf16x2 (round to nearest even; v_cvt_pk_bf16_f32)
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  const bf16x2_t p = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, p);
}
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
// the same layout on v_mfma_f32_16x16x32_f16 (fp16 bit patterns)
__device__ __forceinline__ f32x4 mfma16_f16(u16x8 a, u16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c,
                                                0, 0, 0);
}

// zennit Stabilizer: t + eps * (sign(t) + [t == 0]).  sign(t) + [t == 0] is exactly +1 for
// t >= 0 (including -0), -1 for t < 0, and 0 for NaN (where t + 0 = NaN = t - eps), so the
// select below is bit-identical with one compare instead of three.
__device__ __forceinline__ float stab(float t, float eps) {
  return t + ((t >= 0.f) ? eps : -eps);
}

// n / d (IEEE) computed unconditionally: the empty asm pins the quotient in a VGPR, so a
// following select does not get turned into an exec branch around the division sequence (which
// also drags the operand loads into the branch and serialises their latency).
__device__ __forceinline__ float div_nb(float n, float d) {
  float q = n / d;
  asm volatile("" : "+v"(q));
  return q;
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

// xor-shuffle within a wave (64 lanes) via ds_bpermute
__device__ __forceinline__ float shfl_xor(float v, int mask) {
  return __shfl_xor(v, mask, 64);
}
