// DRSA optimiser on gfx950: one Stiefel gradient-ascent step + polar retraction.
//
// Reference semantics (cxai/xai/drsa/drsa.py):
//   obj_val        drsa.py:122-155   s = relu(sum_{j in k} (AU)_nj (CU)_nj)   [N, K]
//   objective_fn   drsa.py:224-238   f = (mean_k sqrt( sqrt(mean_n s_nk^2) ))^2
//   run            drsa.py:84-106    U <- orthogonalize(U + grad f(U)), log f(U)
//   orthogonalize  drsa.py:201-221   U (U^T U)^{-1/2}  (reference: fp64 eigh on the host)
//
// One step = three launches (a dependent kernel boundary costs ~1.5 us on MI355X, less than a
// hand-rolled grid barrier, MI355X_MICROARCH.md "boundary" / "barrier-xcd"):
//   drsa_partial_kernel  row blocks of A, C spread over every CU.  Per 16-row block a wave runs
//                        XA = A_b U, XC = C_b U (fp32 MFMA, U held in registers), s, r = relu(s),
//                        S_k += r^2 and Gt += A_b^T (r (.) XC) + C_b^T (r (.) XA) straight from the
//                        MFMA output registers (no LDS round trip for P, Q); one [DP^2 + Kp] slab
//                        per workgroup, waves combined in a fixed order.
//   drsa_reduce_kernel   fixed-order sum of the slabs (deterministic, no atomics).
//   drsa_finish_kernel   M_k = sqrt(S_k/N), f, c_k = sqrt(f)/(K N M_k^1.5), V = U + Gt diag(c),
//                        polar(V) by Newton-Schulz on fp32 MFMA in one 16-wave workgroup (the Gram
//                        matrix from its upper block triangle, scaling from the first Gram).
// The closed-form gradient equals autograd's (checked in float64 in tests/test_oracle_drsa.py).
//
// Any d <= 128 with K | d runs through an exact embedding into a padded problem (DP, DKp):
// concept block k of width dk = d/K occupies padded columns [k DKp, k DKp + dk) with DKp the next
// power of two >= dk; padded columns and rows hold zeros in A, C, U, so every sum gets only exact
// +0 terms, and the polar step pairs the DP - d padded rows with the padded columns through an
// identity block (polar(diag(V, I)) = diag(polar(V), I)).  E.g. VGGish layer 19 (d = 100, K = 4,
// getdrsadata.py:119) runs as DP = 128, DKp = 32.  The gradient slab that crosses the ABI (and the
// all-reduce of the sharded path) is in padded coordinates: drsa_amd_drsa_slab_floats(d, K).
#include "common.h"
#include "drsa_amd.h"
#include "polar_ns.h"

#ifndef DRSA_PARTIAL_STAMP
#define DRSA_PARTIAL_STAMP(slot)
#endif

#include <stdlib.h>
#include <type_traits>

namespace {

inline int pow2ceil(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

struct Geom {
  int d, K, dk;     // real problem
  int DKp, DP, Kp;  // padded concept width, padded size, concept slots (K real + phantom)
  bool ok;
};

Geom geom(int d, int K) {
  Geom g{d, K, 0, 0, 0, 0, false};
  if (d <= 0 || d > 128 || K <= 0 || d % K) return g;
  g.dk = d / K;
  g.DKp = pow2ceil(g.dk);
  if (g.DKp > 64) return g;
  const int need = K * g.DKp;
  g.DP = pow2ceil(need < 16 ? 16 : need);
  if (g.DP > 128) return g;
  g.Kp = g.DP / g.DKp;
  g.ok = true;
  return g;
}

inline size_t slab_floats(const Geom& g) { return (size_t)g.DP * g.DP + g.Kp; }
// per-workgroup slab stride in the workspace: 16-B aligned rows for the float4 reduce
inline size_t slab_stride(const Geom& g) { return (slab_floats(g) + 3) / 4 * 4; }

// v if keep else +0.f, by bit mask: a use that is unconditional, so the compiler neither sinks the
// load that produced v into a branch nor has to wait for it before the use
__device__ __forceinline__ float keep_or_zero(float v, bool keep) {
  return __uint_as_float(__float_as_uint(v) & (keep ? 0xffffffffu : 0u));
}
__device__ __forceinline__ float4 keep_or_zero4(float4 v, bool keep) {
  return make_float4(keep_or_zero(v.x, keep), keep_or_zero(v.y, keep), keep_or_zero(v.z, keep),
                     keep_or_zero(v.w, keep));
}

// m-th padded column of the embedding (pairs with padded row d + m in the identity block)
__device__ __forceinline__ int pad_col(int m, int K, int dk, int DKp) {
  const int per = DKp - dk;
  if (per > 0 && m < K * per) return (m / per) * DKp + dk + m % per;
  return K * DKp + (m - K * per);
}

// ---------------------------------------------------------------------------
// partial kernel
// ---------------------------------------------------------------------------
template <int DP, int DKP>
struct PCfg {
  static constexpr int CW = DKP < 16 ? 16 : DKP;   // column-group width (a concept never straddles)
  static constexpr int CG = DP / CW;               // column groups
  static constexpr int NCB = CW / 16;              // 16-wide column blocks per group
  static constexpr int NIB = DP / 16;              // Gt row blocks
  // waves: 16 where the registers allow (4 per SIMD hide the staging latency), fewer for wide groups
  static constexpr int NW = (DP * CW > 4096) ? 4 : ((DP <= 64 && CW == 16) ? 16 : 8);
  static constexpr int NT = NW * 64;
  static constexpr int KP = DP / DKP;
  // rows per staged tile (one tile per leaf at N / kLeaves <= RT).  DP = 128: 80 rows, so the
  // grouped kernel's LDS accumulator (DP x SLD) fits beside the tiles in 160 KB
  static constexpr int RT = DP <= 64 ? 128 : 80;
  static constexpr int LDA = DP + 4;               // staging row stride (16-B aligned rows)
  static constexpr int NV = RT * DP / 4;           // float4 slots per matrix per tile
  static constexpr int PFN = (NV + NT - 1) / NT;   // prefetch registers (float4) per matrix per thread
  static constexpr size_t tile_floats = 2 * (size_t)RT * LDA;
  static constexpr size_t red_floats = (size_t)NW * DP * CW + (size_t)NW * 64 * NCB;
  static constexpr size_t lds_bytes = (tile_floats > red_floats ? tile_floats : red_floats) * sizeof(float);
  // grouped kernel (drsa_partial_grouped_kernel): only the waves w >= CG park their Gt in LDS (the
  // partners w % CG fold them), beside the S-partials; the leaf-group accumulator has its own area
  static constexpr int SLD = DP + 4;               // accumulator row stride: lanes 4 rows apart on other banks
  static constexpr size_t gred_floats = (size_t)(NW - CG) * DP * CW + (size_t)NW * 64 * NCB;
  static constexpr size_t gtile_floats = tile_floats > gred_floats ? tile_floats : gred_floats;
  static constexpr size_t gacc_floats = (size_t)DP * SLD + KP;
  static constexpr size_t glds_bytes = (gtile_floats + gacc_floats) * sizeof(float);
  static_assert(glds_bytes <= 160 * 1024, "grouped partial: LDS");
};

// The row partition of every fp32 gradient (drsa_run, drsa_partial, the fused and sharded steps,
// run_multi, the batched grid): L = min(kLeaves, ceil(N / 16)) LEAVES, leaf l = row blocks
// [l R / L, (l + 1) R / L) of the R 16-row blocks, each reduced by the partial's fixed wave order
// into a leaf slab; leaves form groups of kLeafGroup (ascending); the gradient is the left fold over
// groups of the left fold over each group's leaves.  drsa_partial_kernel runs one workgroup per
// leaf; drsa_partial_grouped_kernel (the batched grid) runs whole groups per workgroup and folds
// them on chip -- the same leaf slabs added in the same order, so the same bits for any number of
// workgroups per problem.  Fixed constants (not the CU count): results do not depend on the device.
constexpr int kLeaves = 256;
constexpr int kLeafGroup = 8;
constexpr int kMaxGroups = kLeaves / kLeafGroup;

// 16-bit A/C element (DT 1 bf16, DT 2 fp16 bit patterns) -> fp32 (exact), fp32 that came from
// such an element -> its bits (exact), and fp32 -> 16-bit with round-to-nearest-even (U)
template <int DT>
__device__ __forceinline__ float wid16(uint32_t b) {
  if constexpr (DT == 1) return __uint_as_float(b << 16);
  else return (float)__builtin_bit_cast(_Float16, (uint16_t)b);
}
template <int DT>
__device__ __forceinline__ uint16_t nar16(float v) {
  if constexpr (DT == 1) return (uint16_t)(__float_as_uint(v) >> 16);
  else return __builtin_bit_cast(uint16_t, (_Float16)v);
}
template <int DT>
__device__ __forceinline__ uint16_t rne16(float v) {
  if constexpr (DT == 1) {
    const uint32_t u = __float_as_uint(v);
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
  } else {
    return __builtin_bit_cast(uint16_t, (_Float16)v);   // v_cvt_f16_f32: RNE
  }
}

template <int DP, int DKP>
constexpr int partial_threads() { return PCfg<DP, DKP>::NT; }

// DT 1 / 2: A and C are bf16 / fp16 in HBM (C5: "bf16 CNN ... fp16 MFMA projection", fp32
// accumulate); GEMM1 (XA = A U, XC = C U) runs on v_mfma_f32_16x16x32_{bf16,f16} with U rounded
// to the 16-bit type (RNE) once per launch; everything after it (relu, S, the gradient GEMM on the
// exactly widened A/C, slab) is fp32.  DT 0: fp32 throughout.
//
// Workgroup g owns row blocks [rb0, rb1) (16 rows each), staged RT rows at a time into LDS by
// all threads (the next tile is prefetched into registers while the current one is computed);
// wave w owns column group w % CG and the tile's row blocks w / CG, w / CG + NW / CG, ...
// VEC (d % 4 == 0): float4 row loads.  A compile-time choice: a runtime branch per prefetch slot
// made the compiler wait for every outstanding load at each join, which serialised the slots and
// defeated the prefetch of the next tile.
//
// partial_core is the body; `pre()` runs after the first tile's loads are issued and before U is
// read (the fused step computes U there, see drsa_fused_step_kernel), `uval(k, j, jp)` returns
// U[k][j] (jp: its padded column), `mid()` runs after U is in registers and before the first LDS
// tile store.
// One 16-row block of a staged tile (rows Ar / Cr, LDA stride) for this wave's column group:
// GEMM1 (XA = A U, XC = C U), s = sum over the concept block of XA (.) XC, r = relu(s), the S
// partials (sacc) and GEMM2 (Gt += A^T (r XC) + C^T (r XA)) accumulated in g.  Shared by the
// per-leaf and the grouped partial kernels, so both add the same terms in the same order.
template <int DP, int DKP, int DT>
__device__ __forceinline__ void rowblock_step(const float* __restrict__ Ar, const float* __restrict__ Cr,
                                              const float (&ureg)[DT ? 1 : PCfg<DP, DKP>::NCB][DT ? 1 : DP / 16][4],
                                              const u16x8 (&ubf)[DT ? PCfg<DP, DKP>::NCB : 1][DT ? (DP / 32 > 0 ? DP / 32 : 1) : 1],
                                              f32x4 (&g)[DP / 16][PCfg<DP, DKP>::NCB], float (&sacc)[PCfg<DP, DKP>::NCB],
                                              int nq_live, int l15, int lg) {
  using Cfg = PCfg<DP, DKP>;
  constexpr bool BF = DT != 0;
  constexpr int NCB = Cfg::NCB, NIB = Cfg::NIB, LDA = Cfg::LDA;
  constexpr int NQ = DP / 16, NQ2 = DP / 32 > 0 ? DP / 32 : 1;
  // ---- GEMM1: XA, XC for the 16 rows and this wave's NCB column blocks ----
  f32x4 xa[NCB], xc[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) { xa[cb] = f32x4{0.f, 0.f, 0.f, 0.f}; xc[cb] = xa[cb]; }
  if constexpr (!BF) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (q >= nq_live) break;
      const float4 a4 = *reinterpret_cast<const float4*>(Ar + l15 * LDA + 16 * q + 4 * lg);
      const float4 c4 = *reinterpret_cast<const float4*>(Cr + l15 * LDA + 16 * q + 4 * lg);
      const float av[4] = {a4.x, a4.y, a4.z, a4.w}, cv[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
          xa[cb] = mfma16(av[tt], ureg[cb][q][tt], xa[cb]);
          xc[cb] = mfma16(cv[tt], ureg[cb][q][tt], xc[cb]);
        }
    }
  } else {
#pragma unroll
    for (int q2 = 0; q2 < NQ2; ++q2) {
      const float* pa8 = Ar + l15 * LDA + 32 * q2 + 8 * lg;
      const float* pc8 = Cr + l15 * LDA + 32 * q2 + 8 * lg;
      const float4 a0 = *reinterpret_cast<const float4*>(pa8), a1 = *reinterpret_cast<const float4*>(pa8 + 4);
      const float4 c0 = *reinterpret_cast<const float4*>(pc8), c1 = *reinterpret_cast<const float4*>(pc8 + 4);
      u16x8 ab, cbv;   // the widened 16-bit values narrow back exactly
      ab[0] = nar16<DT>(a0.x); ab[1] = nar16<DT>(a0.y); ab[2] = nar16<DT>(a0.z); ab[3] = nar16<DT>(a0.w);
      ab[4] = nar16<DT>(a1.x); ab[5] = nar16<DT>(a1.y); ab[6] = nar16<DT>(a1.z); ab[7] = nar16<DT>(a1.w);
      cbv[0] = nar16<DT>(c0.x); cbv[1] = nar16<DT>(c0.y); cbv[2] = nar16<DT>(c0.z); cbv[3] = nar16<DT>(c0.w);
      cbv[4] = nar16<DT>(c1.x); cbv[5] = nar16<DT>(c1.y); cbv[6] = nar16<DT>(c1.z); cbv[7] = nar16<DT>(c1.w);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        if constexpr (DT == 1) {
          xa[cb] = mfma16_bf16(ab, ubf[cb][q2], xa[cb]);
          xc[cb] = mfma16_bf16(cbv, ubf[cb][q2], xc[cb]);
        } else {
          xa[cb] = mfma16_f16(ab, ubf[cb][q2], xa[cb]);
          xc[cb] = mfma16_f16(cbv, ubf[cb][q2], xc[cb]);
        }
      }
    }
  }

  // ---- s = sum over the concept block of XA (.) XC, r = relu(s); S partial ----
  // lane holds rows 4 lg + r, column 16 (cg NCB + cb) + l15
  float rr[NCB][4];
  if constexpr (DKP >= 16) {   // the whole column group is one concept
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = 0.f;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) v += xa[cb][r] * xc[cb][r];
      v += shfl_xor(v, 1); v += shfl_xor(v, 2); v += shfl_xor(v, 4); v += shfl_xor(v, 8);
      const float rv = v > 0.f ? v : 0.f;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) rr[cb][r] = rv;
    }
    if (l15 == 0) {
      float acc = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) acc += rr[0][r] * rr[0][r];
      sacc[0] += acc;
    }
  } else {
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = xa[cb][r] * xc[cb][r];
        if constexpr (DKP >= 2) v += shfl_xor(v, 1);
        if constexpr (DKP >= 4) v += shfl_xor(v, 2);
        if constexpr (DKP >= 8) v += shfl_xor(v, 4);
        rr[cb][r] = v > 0.f ? v : 0.f;
      }
      if ((l15 % DKP) == 0) {
        float acc = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc += rr[cb][r] * rr[cb][r];
        sacc[cb] += acc;
      }
    }
  }

  // ---- GEMM2: Gt[i][j] += sum_n A[n][i] P[n][j] + C[n][i] Q[n][j]  (P = r XC, Q = r XA) ----
  // k-step tt covers rows n = 4 lg + tt: the B operand is this lane's own MFMA output register.
#pragma unroll
  for (int ib = 0; ib < NIB; ++ib) {
    if (ib >= nq_live) break;
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      const float av = Ar[(4 * lg + tt) * LDA + 16 * ib + l15];
      const float cv = Cr[(4 * lg + tt) * LDA + 16 * ib + l15];
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        g[ib][cb] = mfma16(av, rr[cb][tt] * xc[cb][tt], g[ib][cb]);
        g[ib][cb] = mfma16(cv, rr[cb][tt] * xa[cb][tt], g[ib][cb]);
      }
    }
  }
}

template <int DP, int DKP, int DT, bool VEC, class Pre, class UVal, class Mid>
__device__ __forceinline__ void partial_core(const void* __restrict__ A_, const void* __restrict__ C_, int64_t N,
                                             int d, int K, int dk, float* __restrict__ partials, int64_t rb_total,
                                             Pre pre, UVal uval, Mid mid, int nblk) {
  using Cfg = PCfg<DP, DKP>;
  constexpr bool BF = DT != 0;   // 16-bit A/C (bf16 or fp16)
  constexpr int CW = Cfg::CW, CG = Cfg::CG, NCB = Cfg::NCB, NIB = Cfg::NIB, NW = Cfg::NW, NT = Cfg::NT;
  constexpr int KP = Cfg::KP, RT = Cfg::RT, LDA = Cfg::LDA, NV = Cfg::NV, PFN = Cfg::PFN;
  constexpr int WPG = NW / CG, NQ = DP / 16, NQ2 = DP / 32 > 0 ? DP / 32 : 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  const int l15 = lane & 15, lg = lane >> 4;
  const int cg = w % CG;
  float* As = smem;                 // [RT][LDA]
  float* Cs = smem + RT * LDA;      // [RT][LDA]
  const float* A = reinterpret_cast<const float*>(A_);
  const float* C = reinterpret_cast<const float*>(C_);
  const uint16_t* Ab = reinterpret_cast<const uint16_t*>(A_);
  const uint16_t* Cb = reinterpret_cast<const uint16_t*>(C_);

  const int64_t rb0 = (int64_t)blockIdx.x * rb_total / nblk;       // nblk workgroups share the rows
  const int64_t rb1 = (int64_t)(blockIdx.x + 1) * rb_total / nblk;
  const int ntile = (int)((rb1 - rb0 + RT / 16 - 1) / (RT / 16));

  // ---- tile staging: global -> registers (prefetch) -> LDS; rows >= N and columns >= d are 0 ----
  float4 pa[PFN], pc[PFN];
  uint32_t okm = 0;
  static_assert(PFN <= 32, "prefetch mask");
  // Loads are unconditional from a clamped (always valid) address and masked afterwards, so they
  // issue back to back with no exec branches or per-load waits.
  auto load_tile = [&](int t) {
    const int64_t r0 = (rb0 + (int64_t)t * (RT / 16)) * 16;
    const int64_t rmax = rb1 * 16 < N ? rb1 * 16 : N;
    // the tile's first row as a uniform base, the lane's element as a 32-bit offset from it
    // (saddr + voffset loads); a masked lane reads the base itself
    const float* A = reinterpret_cast<const float*>(A_) + r0 * d;
    const float* C = reinterpret_cast<const float*>(C_) + r0 * d;
    const uint16_t* Ab = reinterpret_cast<const uint16_t*>(A_) + r0 * d;
    const uint16_t* Cb = reinterpret_cast<const uint16_t*>(C_) + r0 * d;
#pragma unroll
    for (int p = 0; p < PFN; ++p) {
      const int i = tid + p * NT;
      const int row = (i / (DP / 4)) % RT, col = 4 * (i % (DP / 4));
      const bool ok = i < NV && r0 + row < rmax && col < d;
      const unsigned off = ok ? (unsigned)(row * d + col) : 0u;
      float4 a, c;
      if constexpr (BF) {   // 4 x 16-bit -> 4 fp32 (exact)
        if constexpr (VEC) {
          const uint2 ua = *reinterpret_cast<const uint2*>(Ab + off);
          const uint2 uc = *reinterpret_cast<const uint2*>(Cb + off);
          a = make_float4(wid16<DT>(ua.x & 0xffffu), wid16<DT>(ua.x >> 16), wid16<DT>(ua.y & 0xffffu),
                          wid16<DT>(ua.y >> 16));
          c = make_float4(wid16<DT>(uc.x & 0xffffu), wid16<DT>(uc.x >> 16), wid16<DT>(uc.y & 0xffffu),
                          wid16<DT>(uc.y >> 16));
        } else {
          float va[4], vc[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const unsigned o = (ok && col + u < d) ? off + u : 0u;
            const uint32_t xa = Ab[o], xc = Cb[o];
            va[u] = keep_or_zero(wid16<DT>(xa), col + u < d);
            vc[u] = keep_or_zero(wid16<DT>(xc), col + u < d);
          }
          a = make_float4(va[0], va[1], va[2], va[3]);
          c = make_float4(vc[0], vc[1], vc[2], vc[3]);
        }
      } else {
        if constexpr (VEC) {
          a = *reinterpret_cast<const float4*>(A + off);
          c = *reinterpret_cast<const float4*>(C + off);
        } else {
          float va[4], vc[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const unsigned o = (ok && col + u < d) ? off + u : 0u;
            const float xa = A[o], xc = C[o];
            va[u] = keep_or_zero(xa, col + u < d);
            vc[u] = keep_or_zero(xc, col + u < d);
          }
          a = make_float4(va[0], va[1], va[2], va[3]);
          c = make_float4(vc[0], vc[1], vc[2], vc[3]);
        }
      }
      pa[p] = a;                       // masked at the store (no wait for the data here)
      pc[p] = c;
      okm = (okm & ~(1u << p)) | ((ok ? 1u : 0u) << p);
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int p = 0; p < PFN; ++p) {
      const int i = tid + p * NT;
      if (i < NV) {
        const int row = i / (DP / 4), col = 4 * (i % (DP / 4));
        const bool ok = (okm >> p) & 1u;
        *reinterpret_cast<float4*>(As + row * LDA + col) = keep_or_zero4(pa[p], ok);
        *reinterpret_cast<float4*>(Cs + row * LDA + col) = keep_or_zero4(pc[p], ok);
      }
    }
  };
  DRSA_PARTIAL_STAMP(0);
  if (ntile > 0) load_tile(0);
  DRSA_PARTIAL_STAMP(1);
  pre();

  // ---- embedded U for this wave's column group, in MFMA B-operand order (loads all independent,
  //      issued back to back, overlapping the tile loads above) ----
  //   fp32: ureg[cb][q][t] = Up[16q + 4lg + t][16(cg NCB + cb) + l15]
  //   bf16: ubf[cb][q2][j] = bf16(Up[32 q2 + 8 lg + j][...])
  float ureg[BF ? 1 : NCB][BF ? 1 : NQ][4];
  u16x8 ubf[BF ? NCB : 1][BF ? NQ2 : 1];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    const int jp = 16 * (cg * NCB + cb) + l15;
    const int kc = jp / DKP, l = jp % DKP;
    const bool real = kc < K && l < dk;
    const int j = real ? kc * dk + l : 0;
    if constexpr (!BF) {
#pragma unroll
      for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int k = 16 * q + 4 * lg + t;
          const float v = uval(k < d ? k : 0, j, jp);   // clamped address, masked after
          ureg[cb][q][t] = keep_or_zero(v, real && k < d);
        }
    } else {
#pragma unroll
      for (int q2 = 0; q2 < NQ2; ++q2)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          const int k = 32 * q2 + 8 * lg + jj;
          const float v = uval(k < d ? k : 0, j, jp);
          ubf[cb][q2][jj] = rne16<DT>(keep_or_zero(v, real && k < d));
        }
    }
  }

  f32x4 g[NIB][NCB];
#pragma unroll
  for (int ib = 0; ib < NIB; ++ib)
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) g[ib][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  float sacc[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) sacc[cb] = 0.f;
  const int nq_live = (d + 15) / 16;   // k chunks / Gt row blocks that can be nonzero

  DRSA_PARTIAL_STAMP(2);
  mid();
  if (ntile > 0) store_tile();
  __syncthreads();
  DRSA_PARTIAL_STAMP(3);
  for (int t = 0; t < ntile; ++t) {
    if (t + 1 < ntile) load_tile(t + 1);
    const int64_t rbt = rb0 + (int64_t)t * (RT / 16);
    const int nrb = (int)((rb1 - rbt) < (RT / 16) ? (rb1 - rbt) : (RT / 16));
    for (int rbl = w / CG; rbl < nrb; rbl += WPG) {
      rowblock_step<DP, DKP, DT>(As + 16 * rbl * LDA, Cs + 16 * rbl * LDA, ureg, ubf, g, sacc, nq_live, l15, lg);
    }
    if (t + 1 < ntile) {
      __syncthreads();
      store_tile();
      __syncthreads();
    }
  }

  // ---- combine the waves of each column group in a fixed order -> slab ----
  DRSA_PARTIAL_STAMP(4);
  __syncthreads();
  DRSA_PARTIAL_STAMP(5);
  float* red = smem;                                  // [NW][DP][CW]
  float* sred = smem + (size_t)NW * DP * CW;          // [NW][64][NCB]
#pragma unroll
  for (int ib = 0; ib < NIB; ++ib)
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[((size_t)w * DP + 16 * ib + 4 * lg + r) * CW + 16 * cb + l15] = g[ib][cb][r];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) sred[(w * 64 + lane) * NCB + cb] = sacc[cb];
  __syncthreads();
  float* slab = partials + (size_t)blockIdx.x * ((DP * DP + KP + 3) / 4 * 4);
  for (int e = tid; e < DP * DP; e += NT) {
    const int i = e / DP, j = e % DP, gcg = j / CW, jj = j % CW;
    float acc = 0.f;
    for (int ww = gcg; ww < NW; ww += CG) acc += red[((size_t)ww * DP + i) * CW + jj];
    slab[e] = acc;
  }
  for (int k = tid; k < KP; k += NT) {
    const int j0 = k * DKP, gcg = j0 / CW, cb = (j0 % CW) / 16, lo = DKP < 16 ? j0 % 16 : 0;
    float acc = 0.f;
    for (int ww = gcg; ww < NW; ww += CG)
      for (int q = 0; q < 4; ++q) acc += sred[(ww * 64 + 16 * q + lo) * NCB + cb];
    slab[DP * DP + k] = acc;
  }
  DRSA_PARTIAL_STAMP(6);
}

template <int DP, int DKP, int DT, bool VEC>
__global__ __launch_bounds__((partial_threads<DP, DKP>())) void drsa_partial_kernel(
    const void* __restrict__ A_, const void* __restrict__ C_, int64_t N, int d, int K, int dk,
    const float* __restrict__ U, float* __restrict__ partials, int64_t rb_total) {
  partial_core<DP, DKP, DT, VEC>(
      A_, C_, N, d, K, dk, partials, rb_total, [] {},
      [&](int k, int j, int) { return U[(size_t)k * d + j]; }, [] {}, (int)gridDim.x);
}

// ---------------------------------------------------------------------------
// batched problems: the descriptor of one problem (task-parallel DRSA grid, optsubspaces.py:17-23)
// ---------------------------------------------------------------------------
struct BatchDesc {
  const float* A;
  const float* C;
  int64_t N;
  int64_t rb_total;
  int d, K, dk, DKP;
  int G;                // partial workgroups of this problem (<= gridDim.x)
  int L;                // leaves (kLeaves partition)
  int m;                // leaf groups per workgroup (0: one leaf per workgroup, per-leaf slabs)
  float* U_io;
  float* U_tmp;
  float* f_traj;
  int* counter;
  float* partials;      // one slab per leaf group
  float* gs;
};

// Workgroup b of problem p owns leaf groups [b m, (b + 1) m) and computes their leaves one after
// another with the per-leaf kernel's arithmetic (rowblock_step, the same tile cut and wave order,
// Gt reset per leaf), folding each leaf slab -- combined in the per-leaf kernel's wave order -- into
// an LDS accumulator; a finished group's accumulator is its slab.  U is loaded once per workgroup
// and the next tile (possibly the next leaf's) is prefetched under the current one's MFMAs.
template <int DP, int DKP, bool VEC>
__global__ __launch_bounds__((partial_threads<DP, DKP>())) void drsa_partial_grouped_kernel(
    const BatchDesc* __restrict__ bd, int parity) {
  using Cfg = PCfg<DP, DKP>;
  constexpr int CW = Cfg::CW, CG = Cfg::CG, NCB = Cfg::NCB, NIB = Cfg::NIB, NW = Cfg::NW, NT = Cfg::NT;
  constexpr int KP = Cfg::KP, RT = Cfg::RT, LDA = Cfg::LDA, NV = Cfg::NV, PFN = Cfg::PFN, SLD = Cfg::SLD;
  constexpr int WPG = NW / CG, NQ = DP / 16, RB = RT / 16;
  constexpr size_t ES = (DP * DP + KP + 3) / 4 * 4;
  const BatchDesc& q = bd[blockIdx.y];
  if ((int)blockIdx.x >= q.G) return;    // uniform per workgroup: before any barrier
  extern __shared__ __attribute__((aligned(16))) float smem[];
  // w uniform (readfirstlane): the per-wave roles of the leaf fold are scalar branches
  const int tid = threadIdx.x, lane = lane_id(), w = __builtin_amdgcn_readfirstlane(wave_id());
  const int l15 = lane & 15, lg = lane >> 4;
  const int cg = w % CG;
  float* As = smem;                        // [RT][LDA]
  float* Cs = smem + RT * LDA;             // [RT][LDA]
  float* red = smem;                       // [(NW - CG) x NIB x NCB x 4][64]   (aliases the tiles)
  float* sred = smem + (size_t)(NW - CG) * DP * CW;   // [NW][64][NCB]
  float* S = smem + Cfg::gtile_floats;     // [DP][SLD] + [KP]: the group accumulator
  const float* U = parity ? q.U_tmp : q.U_io;
  const int d = q.d, K = q.K, dk = q.dk, L = q.L;
  const int64_t N = q.N, R = q.rb_total;
  const int ngrp = (L + kLeafGroup - 1) / kLeafGroup;
  const int gq0 = (int)blockIdx.x * q.m, gq1 = gq0 + q.m < ngrp ? gq0 + q.m : ngrp;
  const int lf0 = gq0 * kLeafGroup, lf1 = gq1 * kLeafGroup < L ? gq1 * kLeafGroup : L;
  const float* A = q.A;
  const float* C = q.C;
  // leaf bounds in row blocks (uniform), evaluated once per leaf
  auto leaf_rb0 = [&](int lf) -> int64_t { return (int64_t)lf * R / L; };

  float4 pa[PFN], pc[PFN];
  uint32_t okm = 0;
  auto load_tile = [&](int64_t rb0, int64_t rb1, int t) {   // = partial_core's load_tile (fp32)
    const int64_t r0 = (rb0 + (int64_t)t * RB) * 16;
    const int64_t rmax = rb1 * 16 < N ? rb1 * 16 : N;
    const float* Ab = A + r0 * d;
    const float* Cb = C + r0 * d;
#pragma unroll
    for (int p = 0; p < PFN; ++p) {
      const int i = tid + p * NT;
      const int row = (i / (DP / 4)) % RT, col = 4 * (i % (DP / 4));
      const bool ok = i < NV && r0 + row < rmax && col < d;
      const unsigned off = ok ? (unsigned)(row * d + col) : 0u;
      float4 a, c;
      if constexpr (VEC) {
        a = *reinterpret_cast<const float4*>(Ab + off);
        c = *reinterpret_cast<const float4*>(Cb + off);
      } else {
        float va[4], vc[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const unsigned o = (ok && col + u < d) ? off + u : 0u;
          const float xa = Ab[o], xc = Cb[o];
          va[u] = keep_or_zero(xa, col + u < d);
          vc[u] = keep_or_zero(xc, col + u < d);
        }
        a = make_float4(va[0], va[1], va[2], va[3]);
        c = make_float4(vc[0], vc[1], vc[2], vc[3]);
      }
      pa[p] = a;
      pc[p] = c;
      okm = (okm & ~(1u << p)) | ((ok ? 1u : 0u) << p);
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int p = 0; p < PFN; ++p) {
      const int i = tid + p * NT;
      if (i < NV) {
        const int row = i / (DP / 4), col = 4 * (i % (DP / 4));
        const bool ok = (okm >> p) & 1u;
        *reinterpret_cast<float4*>(As + row * LDA + col) = keep_or_zero4(pa[p], ok);
        *reinterpret_cast<float4*>(Cs + row * LDA + col) = keep_or_zero4(pc[p], ok);
      }
    }
  };
  if (lf0 >= lf1) return;                 // (no such workgroup: G = ceil(groups / m))
  int64_t c0 = leaf_rb0(lf0), c1 = leaf_rb0(lf0 + 1);           // current leaf
  int64_t n1 = lf0 + 1 < lf1 ? leaf_rb0(lf0 + 2) : c1;            // end of the next leaf
  load_tile(c0, c1, 0);
  // group accumulator = +0
  for (int e = tid; e < DP * SLD + KP; e += NT) S[e] = 0.f;

  float ureg[NCB][NQ][4];
  u16x8 ubf[1][1];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    const int jp = 16 * (cg * NCB + cb) + l15;
    const int kc = jp / DKP, l = jp % DKP;
    const bool real = kc < K && l < dk;
    const int j = real ? kc * dk + l : 0;
#pragma unroll
    for (int qq = 0; qq < NQ; ++qq)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int k = 16 * qq + 4 * lg + t;
        const float v = U[(size_t)(k < d ? k : 0) * d + j];
        ureg[cb][qq][t] = keep_or_zero(v, real && k < d);
      }
  }
  f32x4 g[NIB][NCB];
  float sacc[NCB];
  auto zero_acc = [&]() {
#pragma unroll
    for (int ib = 0; ib < NIB; ++ib)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) g[ib][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) sacc[cb] = 0.f;
  };
  zero_acc();
  const int nq_live = (d + 15) / 16;
  store_tile();
  __syncthreads();
  int lf = lf0, t = 0, nt = (int)((c1 - c0 + RB - 1) / RB);
  for (;;) {
    // the next tile: this leaf's next one, else the next leaf's first
    const bool more_in_leaf = t + 1 < nt;
    const bool has_next = more_in_leaf || lf + 1 < lf1;
    if (has_next) {
      const int64_t la = more_in_leaf ? c0 : c1, lb = more_in_leaf ? c1 : n1;
      load_tile(la, lb, more_in_leaf ? t + 1 : 0);
    }
    const int64_t rbt = c0 + (int64_t)t * RB;
    const int nrb = (int)((c1 - rbt) < RB ? (c1 - rbt) : RB);
    for (int rbl = w / CG; rbl < nrb; rbl += WPG)
      rowblock_step<DP, DKP, 0>(As + 16 * rbl * LDA, Cs + 16 * rbl * LDA, ureg, ubf, g, sacc, nq_live, l15, lg);
    __syncthreads();                      // tile reads done
    if (!more_in_leaf) {
      // leaf slab = ((0 + Gt_cg) + Gt_{cg + CG}) + ... (drsa_partial_kernel's wave order), S += slab.
      // LDS element offsets from one opaque per-lane base + compile-time constants (ds offset field):
      // otherwise the 64 loop-invariant addresses are hoisted out of the leaf loop and spill.
      constexpr int GE = NIB * NCB * 4;                  // Gt registers per lane
      if (w >= CG) {
        uint32_t ro = (uint32_t)((w - CG) * GE * 64 + lane);
        asm volatile("" : "+v"(ro));
#pragma unroll
        for (int ib = 0; ib < NIB; ++ib)
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
            for (int r = 0; r < 4; ++r) red[ro + ((ib * NCB + cb) * 4 + r) * 64] = g[ib][cb][r];
      }
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) sred[(w * 64 + lane) * NCB + cb] = sacc[cb];
      __syncthreads();
      if (w < CG) {
        uint32_t ro = (uint32_t)(w * GE * 64 + lane);    // partner w + CG's element (ib, cb, r) = 0
        uint32_t so = (uint32_t)(4 * lg * SLD + w * CW + l15);
        asm volatile("" : "+v"(ro), "+v"(so));
#pragma unroll
        for (int ib = 0; ib < NIB; ++ib)
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float acc = 0.f + g[ib][cb][r];
#pragma unroll
              for (int k = 1; k < WPG; ++k)      // partners w + CG, w + 2 CG, ... in order
                acc += red[ro + (k - 1) * CG * GE * 64 + ((ib * NCB + cb) * 4 + r) * 64];
              float* sp = S + so + (16 * ib + r) * SLD + 16 * cb;
              *sp = *sp + acc;
            }
      }
      for (int k = tid; k < KP; k += NT) {
        const int j0 = k * DKP, gcg = j0 / CW, cb = (j0 % CW) / 16, lo = DKP < 16 ? j0 % 16 : 0;
        float acc = 0.f;
        for (int ww = gcg; ww < NW; ww += CG)
          for (int qq = 0; qq < 4; ++qq) acc += sred[(ww * 64 + 16 * qq + lo) * NCB + cb];
        S[DP * SLD + k] = S[DP * SLD + k] + acc;
      }
      zero_acc();
      __syncthreads();                    // red / sred reads and the S updates done
      if ((lf + 1) % kLeafGroup == 0 || lf + 1 == lf1) {
        // the group is complete: its slab, then a fresh accumulator
        float* slab = q.partials + (size_t)(lf / kLeafGroup) * ES;
        for (int e = tid; e < DP * DP; e += NT) {
          const int i = e / DP, j = e % DP;
          slab[e] = S[i * SLD + j];
          S[i * SLD + j] = 0.f;
        }
        for (int k = tid; k < KP; k += NT) {
          slab[DP * DP + k] = S[DP * SLD + k];
          S[DP * SLD + k] = 0.f;
        }
        // (the next fold into S comes two barriers later)
      }
    }
    if (!has_next) break;
    if (more_in_leaf) {
      ++t;
    } else {
      ++lf;
      t = 0;
      c0 = c1;
      c1 = n1;
      n1 = lf + 1 < lf1 ? leaf_rb0(lf + 2) : c1;
      nt = (int)((c1 - c0 + RB - 1) / RB);
    }
    store_tile();
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// reduce: out[e] = the left fold over leaf groups q (ascending) of G_q[e], G_q[e] = the left fold
// over the group's slabs (at most LG of them, ascending), both from +0 -- the kLeaves partition's
// fixed order (deterministic, no atomics).  LG = kLeafGroup for per-leaf slabs (drsa_partial_kernel,
// the fused step), 1 for the grouped kernel's per-group slabs: the same additions either way.
// Thread group grp of a block computes G_q for q = grp, grp + 4, ... with every slab load of its
// groups issued before the adds (the slabs were just written by every CU: one memory round trip per
// batch of loads), then one thread per element folds the G_q in order.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void reduce_grouped(const float* __restrict__ partials, int P, int LG, int ES, int E,
                                               float* __restrict__ out) {
  __shared__ float part[kMaxGroups][64];
  const int l = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + l;
  const int ng = (P + LG - 1) / LG;
  const int ec = e < E ? e : 0;
#pragma unroll
  for (int q0 = 0; q0 < kMaxGroups; q0 += 4) {
    const int qq = q0 + grp;
    if (q0 >= ng) break;                  // uniform
    float v[kLeafGroup];
#pragma unroll
    for (int i = 0; i < kLeafGroup; ++i) {
      const int p = qq * LG + i;
      const bool ok = i < LG && qq < ng && p < P;
      v[i] = partials[(size_t)(ok ? p : 0) * ES + ec];
    }
    float G = 0.f;
#pragma unroll
    for (int i = 0; i < kLeafGroup; ++i)
      if (i < LG && qq * LG + i < P) G += v[i];
    if (qq < ng) part[qq][l] = G;
  }
  __syncthreads();
  if (grp == 0 && e < E) {
    float T = 0.f;
    for (int qq = 0; qq < ng; ++qq) T += part[qq][l];
    out[e] = T;
  }
}

// The per-leaf slab reduce of drsa_run / the fused and sharded steps (LG = kLeafGroup), spread over
// the chip: RW = 256 / CW thread rows per workgroup of CW columns, each thread computing the group
// sums G_q of QPT = kMaxGroups / RW groups with all QPT * kLeafGroup slab loads issued first; the
// same additions in the same order as reduce_grouped (bit-identical), on E / CW workgroups instead of
// E / 64 (C3: 129 instead of 65 CUs, 32 loads per thread in flight instead of 8 rounds of 8;
// A/B at C3 (gpurun_out/r6e): CW 8 / 16 / 32 = 33.9 / 32.4 / 31.7 us per step).
#ifndef DRSA_REDUCE_CW
#define DRSA_REDUCE_CW 32
#endif
// (CW = 64 for the DP = 128 slabs: E / 16 = 1025 workgroups measured slower than E / 64 = 257)
template <int CW>
__global__ __launch_bounds__(256) void drsa_reduce_kernel(const float* __restrict__ partials, int P, int E, int ES,
                                                          float* __restrict__ out) {
  constexpr int RW = 256 / CW, QPT = kMaxGroups / RW;
  static_assert(kMaxGroups % RW == 0, "groups per thread");
  __shared__ float part[kMaxGroups][CW];
  const int c = threadIdx.x % CW, r = threadIdx.x / CW;
  const int e = blockIdx.x * CW + c;
  const int ng = (P + kLeafGroup - 1) / kLeafGroup;
  const int ec = e < E ? e : 0;
  float v[QPT][kLeafGroup];
#pragma unroll
  for (int j = 0; j < QPT; ++j)
#pragma unroll
    for (int i = 0; i < kLeafGroup; ++i) {
      const int p = (r + RW * j) * kLeafGroup + i;
      v[j][i] = partials[(size_t)(p < P ? p : 0) * ES + ec];
    }
#pragma unroll
  for (int j = 0; j < QPT; ++j) {
    const int qq = r + RW * j;
    float G = 0.f;
#pragma unroll
    for (int i = 0; i < kLeafGroup; ++i)
      if (qq * kLeafGroup + i < P) G += v[j][i];
    if (qq < ng) part[qq][c] = G;
  }
  __syncthreads();
  if (r == 0 && e < E) {
    float T = 0.f;
    for (int qq = 0; qq < ng; ++qq) T += part[qq][c];
    out[e] = T;
  }
}

// the polar runs at PD = max(32, DP) (32x32 MFMA tiles; a d <= 16 problem is embedded once more)
template <int DP>
constexpr int polar_dim() { return DP < 32 ? 32 : DP; }
template <int DP>
constexpr size_t finish_lds() {
  // polar_ns16 (DP <= 64): the second X buffer; polar_ns: the k-split scratch
  constexpr int PD = polar_dim<DP>();
  constexpr size_t scr = ns_scratch_floats<PD>();
  return (2 * (size_t)PD * ns_ld<PD>() + 64 + scr) * sizeof(float);
}

// finish prologue: f = (mean_k sqrt(M_k))^2, M_k = sqrt(S_k / N) (evaluated in double from the fp32
// sums), c_k = sqrt(f) / (K N M_k^1.5), and X = embed(U + Gt diag(c)): padded rows pair with the
// padded columns through an identity block.  Returns f; X is built only when build_x.
template <int DP>
__device__ __forceinline__ double finish_prologue(const float* __restrict__ gs, double n_total, int d, int K, int DKP,
                                                  const float* __restrict__ U, float* X, bool build_x,
                                                  double* dterm, float* cvec, double* fsh) {
  constexpr int PD = polar_dim<DP>(), NT = fin_threads<PD>(), LD = ns_ld<PD>();
  constexpr int NQ = (PD * PD + NT - 1) / NT;
  const int tid = threadIdx.x;
  const int dk = d / K;
  // X's U and G entries are loaded first, so their memory latency overlaps the f / c stages
  // (loads from clamped addresses, pinned, so all of them are in flight at once: no exec branches)
  float uq[NQ], gq[NQ];
  if (build_x) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int e = tid + q * NT;
      const int ip = e / PD, jp = e % PD, kc = jp / DKP, l = jp % DKP;
      const bool real = e < PD * PD && ip < d && jp < DP && kc < K && l < dk;
      uq[q] = U[real ? (size_t)ip * d + kc * dk + l : 0];
      gq[q] = gs[real ? ip * DP + jp : 0];
    }
  }
  if (tid < K) dterm[tid] = sqrt(sqrt((double)gs[DP * DP + tid] / n_total));
  __syncthreads();
  if (tid == 0) {
    double sum = 0.0;
    for (int k = 0; k < K; ++k) sum += dterm[k];
    const double mean = sum / K;
    *fsh = mean * mean;
  }
  __syncthreads();
  const double f = *fsh;
  if (tid < K) {
    const double Mk = sqrt((double)gs[DP * DP + tid] / n_total);
    cvec[tid] = (float)((Mk > 0.0) ? sqrt(f) / (K * n_total * Mk * sqrt(Mk)) : 0.0);
  }
  if (!build_x) return f;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int e = tid + q * NT;
    const int ip = e / PD, jp = e % PD, kc = jp / DKP, l = jp % DKP;
    const bool real = e < PD * PD && ip < d && jp < DP && kc < K && l < dk;
    const float u = uq[q], gv = gq[q];
    const float rv = keep_or_zero(u + gv * cvec[kc < K ? kc : 0], real);
    const float v = ip < d ? rv : ((jp == pad_col(ip - d, K, dk, DKP)) ? 1.f : 0.f);
    if (e < PD * PD) X[ip * LD + jp] = v;
  }
  return f;
}

// mode 0: full step (f, U_out = polar(U + G)); mode 1: objective only
template <int DP>
__device__ __forceinline__ void finish_body(const float* __restrict__ gs, double n_total, int d, int K, int DKP,
                                            const float* __restrict__ U, float* __restrict__ U_out,
                                            float* __restrict__ f_out, int* __restrict__ step_counter,
                                            int f_stride_by_counter, int mode, float tol, int max_iter,
                                            int* __restrict__ iters_out) {
  constexpr int PD = polar_dim<DP>(), NT = fin_threads<PD>(), LD = ns_ld<PD>();
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* X = smem;
  float* T = X + PD * LD;
  float* red = T + PD * LD;   // 64 floats
  float* scr = red + 64;      // k-split partial tiles (polar_ns)
  __shared__ double dterm[128];
  __shared__ float cvec[128];
  __shared__ double fsh;
  const int tid = threadIdx.x;
  const int dk = d / K;
  const double f = finish_prologue<DP>(gs, n_total, d, K, DKP, U, X, mode == 0, dterm, cvec, &fsh);
  const int slot = f_stride_by_counter ? *step_counter : 0;
  if (tid == 0) f_out[slot] = (float)f;
  if (mode == 1) return;
  const int it = polar_run<PD>(X, T, red, scr, tol, max_iter);
  for (int e = tid; e < d * d; e += NT) {
    const int i = e / d, j = e % d;
    U_out[e] = X[i * LD + (j / dk) * DKP + j % dk];
  }
  if (tid == 0) {
    if (iters_out) *iters_out = it;
    if (f_stride_by_counter) *step_counter = slot + 1;
  }
}

template <int DP>
__global__ __launch_bounds__(fin_threads<polar_dim<DP>()>()) void drsa_finish_kernel(
    const float* __restrict__ gs, double n_total, int d, int K, int DKP, const float* __restrict__ U,
    float* __restrict__ U_out, float* __restrict__ f_out, int* __restrict__ step_counter, int f_stride_by_counter,
    int mode, float tol, int max_iter, int* __restrict__ iters_out) {
  finish_body<DP>(gs, n_total, d, K, DKP, U, U_out, f_out, step_counter, f_stride_by_counter, mode, tol, max_iter,
                  iters_out);
}

// ---------------------------------------------------------------------------
// Cooperative finish at DP = 128 (drsa_run / run_multi, the C5 shapes): the polar's two 128^3
// products per Newton-Schulz iteration split over kCoopWG = 8 workgroups on as many CUs, workgroup j
// owning the 16 columns [16 j, 16 j + 16) of X.  Per iteration workgroup j forms P_j = X^T X[:, j]
// (8 16x16 tiles, one wave each, two per SIMD), T_j = 1.5 I - 0.5 P_j with its max |P_j - I|, and
// X'[:, j] = X T_j (8 tiles); the new
// column blocks and the error maxima are exchanged through the workspace (one hand-off per
// iteration: agent-scope stores, a ticket counter, agent-scope loads), so every workgroup holds
// the whole X' for the next P.  Bit-identical to drsa_finish_kernel's single-workgroup polar_ns:
//   * every P / X T entry is the same full-k fp32 fma chain (k ascending from +0: the 32x32x2 MFMA
//     there, 16x16x4 here, both exact chains; P's lower tiles there are mirrored from the upper
//     ones, here computed directly: x_k y_k = y_k x_k exactly);
//   * tr(P) from P's diagonal (each workgroup hands its diagonal tile's 32 entries over), folded in
//     the same order; the inf-norm row sums as column sums of workgroup j's block (P is exactly
//     symmetric), in the same order; maxima are order-free;
//   * the X T of an iteration whose error stops the loop is computed speculatively (the error is
//     exchanged with its result) and dropped, so the returned X is the one polar_ns returns.
// The workgroups spin on each other: the launch needs kCoopWG co-resident workgroups (one per CU,
// 141 KB of LDS each), which the callers guarantee by launching nothing else that waits on them.
// Failure is loud, never a hang and never silent: a spin that outlives both the wall-clock budget
// (100 ms) and kCoopMinPolls polls (so a queue preempted mid-spin, whose wall clock jumps, still
// polls ~20 ms after it resumes) gives up, sets the workspace's sticky status word, and poisons
// U_out and f with NaN; every later finish of the run sees the word at its start and skips straight
// to the poison (no further spinning, no diverged ticket to wait on).  drsa_amd_drsa_run /
// _run_multi read the word back and return DRSA_ETIMEOUT; drsa_amd_drsa_coop_status reads it for a
// run the caller captured into its own graph.  coop_reset clears ticket and status per run.
// ---------------------------------------------------------------------------
constexpr int kCoopWG = 8;
constexpr int kCoopBW = 128 / kCoopWG;   // columns per workgroup (16x16x4 MFMA tiles)
constexpr long long kCoopSpinTicks = 10000000;   // s_memrealtime runs at 100 MHz: 100 ms
constexpr int kCoopMinPolls = 20000;             // >= ~20 ms of polling (one sc1 load + s_sleep each)

// diagnostic build (-DDRSA_COOP_STAMP, scripts/probe_coop.py): phase times of the last launch's
// workgroups, read back by drsa_amd_debug_coop_stamps; nothing in the kernel reads them
#ifdef DRSA_COOP_STAMP
__device__ unsigned long long g_coop_stamps[kCoopWG][64];
#define COOP_STAMP(slot) do { if (threadIdx.x == 0 && (slot) < 64) g_coop_stamps[blockIdx.x][(slot)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define COOP_STAMP(slot)
#endif

struct CoopXchg {
  float xb[2][128 * 128];        // X' by iteration parity (column block j written by workgroup j)
  float sc[2][kCoopWG][4];       // per parity and workgroup: error max, inf-norm partial
  unsigned ticket;               // hand-off counter: kCoopWG arrivals per exchange, reset per run
  unsigned status;               // sticky: 1 once any hand-off of the run timed out, reset per run
  unsigned pad[62];
};

__device__ __forceinline__ void coop_st(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float coop_ld(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// every thread calls after its agent-scope stores; returns false if the other workgroups did not
// arrive within the spin budget (then the run's status word is set).
// Visibility without release/acquire fences (MI355X_MICROARCH.md "Valid forms besides Guideline
// 16's R1/R2" and the sc1 hand-off table's first row, which this matches cell for cell): every byte
// handed over is stored by coop_st (a relaxed agent-scope atomic store = global_store_dword sc1,
// 4 B) and read by coop_ld (global_load_dword sc1 to registers); every storing wave waits
// vmcnt(0) before the workgroup barrier; ONE lane per workgroup then signals for all its stores
// with one agent-scope atomic add on the ticket and polls it with relaxed agent-scope (sc1) loads;
// the other waves load only after the barrier that lane joins; one workgroup per CU, hipMalloc'd
// workspace.  (An agent release fence costs ~1.7 us and an acquire ~1.7 us per exchange here,
// 5 exchanges per finish, for no change in what the table guarantees.)
__device__ bool coop_exchange(unsigned* ticket, unsigned* status, int* ok_sh, long long spin_ticks,
                              int min_polls) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = (old / kCoopWG + 1) * kCoopWG;
    const long long t0 = wall_clock64();
    int ok = 1;
    for (int polls = 0;; ++polls) {
      const unsigned v = __hip_atomic_load(ticket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((int)(v - target) >= 0) break;
      if (polls >= min_polls && wall_clock64() - t0 > spin_ticks) { ok = 0; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    if (!ok) __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *ok_sh = ok;
  }
  __syncthreads();
  return *ok_sh != 0;
}

constexpr int kCoopTLD = kCoopBW;   // T_j row stride (one column block)
constexpr size_t coop_lds_bytes() {
  return ((size_t)2 * 128 * ns_ld<128>() + (size_t)128 * kCoopTLD + 64) * sizeof(float);
}

__global__ __launch_bounds__(1024) void drsa_finish_coop_kernel(
    const float* __restrict__ gs, double n_total, int d, int K, int DKP, const float* __restrict__ U,
    float* __restrict__ U_out, float* __restrict__ f_out, int* __restrict__ step_counter, int f_stride_by_counter,
    float tol, int max_iter, CoopXchg* __restrict__ xc, long long spin_ticks, int min_polls) {
  constexpr int DP = 128, LD = ns_ld<DP>(), NT = 1024, TLD = kCoopTLD, TPR = NT / DP;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* X = smem;                 // current X (full)
  float* Xn = X + DP * LD;         // X' being assembled
  float* Tj = Xn + DP * LD;        // T_j = 1.5 I - 0.5 P[:, j-block]
  float* red = Tj + DP * TLD;      // 64 floats
  __shared__ double dterm[128];
  __shared__ float cvec[128];
  __shared__ double fsh;
  __shared__ float diag[128];
  __shared__ int ok_sh;
  constexpr int BW = kCoopBW, NB = DP / BW;   // 16-row / 16-column tiles, NB = 8 per column block
  const int tid = threadIdx.x, lane = lane_id(), w = wave_id(), j = blockIdx.x;
  const int lo = lane & 15, hi = lane >> 4;   // 16x16x4: A/B lane l -> index l & 15 at k = k0 + (l >> 4)
  const int dk = d / K;
  // a hand-off of an earlier step of this run timed out: poison this step too, without spinning
  if (tid == 0) ok_sh = __hip_atomic_load(&xc->status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
  __syncthreads();
  if (!ok_sh) {
    for (int e = tid; e < DP * BW; e += NT) {
      const int i = e / BW, pc = BW * j + e % BW, kc = pc / DKP, l = pc % DKP;
      if (i < d && kc < K && l < dk) U_out[i * d + kc * dk + l] = __builtin_nanf("");
    }
    if (j == 0 && tid == 0) {
      const int slot = f_stride_by_counter ? *step_counter : 0;
      f_out[slot] = __builtin_nanf("");
      if (f_stride_by_counter) *step_counter = slot + 1;
    }
    return;   // uniform per workgroup
  }
  COOP_STAMP(0);
  const double f = finish_prologue<DP>(gs, n_total, d, K, DKP, U, X, true, dterm, cvec, &fsh);
  bool ok = true;
  COOP_STAMP(1);

  // P_j tile (ib = w) of X^T X[:, j-block] for waves 0..7: Tj[row][col - BW j] = raw P (it == 0) or
  // 1.5 I - 0.5 P with err (it > 0).  16x16 D layout: lane l, reg r -> row 4 (l >> 4) + r, col l & 15.
  auto gram_block = [&](int it, float& err) {
    __syncthreads();   // X complete
    if (w < NB) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
      for (int k0 = 0; k0 < DP; k0 += 4) {
        const int kk = k0 + hi;
        acc = mfma16(X[kk * LD + BW * w + lo], X[kk * LD + BW * j + lo], acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = BW * w + 4 * hi + r;
        float v = acc[r];
        if (it > 0) {
          const bool dg = row == BW * j + lo;
          err = fmaxf(err, fabsf(v - (dg ? 1.f : 0.f)));
          v = (dg ? 1.5f : 0.f) - 0.5f * v;
        }
        Tj[row * TLD + lo] = v;
      }
    }
  };
  // X'[:, j-block] = X T_j for waves 0..7 (tile ib = w): into Xn and the exchange buffer
  auto xt_block = [&](int par) {
    __syncthreads();   // T_j complete
    if (w < NB) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
      for (int k0 = 0; k0 < DP; k0 += 4) {
        const int kk = k0 + hi;
        acc = mfma16(X[(BW * w + lo) * LD + kk], Tj[kk * TLD + lo], acc);
      }
      float* xg = xc->xb[par];
      int l = lane;
      asm volatile("" : "+v"(l));
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = BW * w + 4 * (l >> 4) + r, col = BW * j + (l & 15);
        Xn[row * LD + col] = acc[r];
        coop_st(&xg[row * DP + col], acc[r]);
      }
    }
  };
  // the other workgroups' column blocks of X' (after the exchange)
  // (all loads issued before the first LDS store: one memory round trip, not 12)
  auto gather_blocks = [&](int par) {
    constexpr int NQ = (kCoopWG - 1) * BW * DP / NT;
    const float* xg = xc->xb[par];
    unsigned t = (unsigned)tid;
    asm volatile("" : "+v"(t));   // addresses per call: hoisted out of the iteration loop they spill
    float v[NQ];
    unsigned lds[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const unsigned e = t + (unsigned)q * NT;  // over the foreign blocks, BW-float runs
      const unsigned bi = e / (BW * DP), rem = e % (BW * DP);
      const unsigned blk = bi < (unsigned)j ? bi : bi + 1;
      const unsigned row = rem / BW, col = BW * blk + rem % BW;
      v[q] = coop_ld(&xg[row * DP + col]);
      lds[q] = row * LD + col;
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) Xn[lds[q]] = v[q];
  };

  // ---- iteration 0: raw P_j, scaling a^2 = DP / tr(P) unless a^2 ||P||_inf >= 2.9 ----
  float err = 0.f, rowmax_all;
  gram_block(0, err);
  __syncthreads();   // Tj (raw P) complete
  COOP_STAMP(2);
  // row sums of |P| for the rows of block j, as column sums of P[:, j-block] (polar_ns's order)
  float rs = 0.f;
  if (tid < BW * TPR) {
    const int cl = tid / TPR, part = tid % TPR;
#pragma unroll
    for (int c = part; c < DP; c += TPR) rs += fabsf(Tj[c * TLD + cl]);
  }
  for (int m = 1; m < TPR; m <<= 1) rs += shfl_xor(rs, m);
  const float rmax_j = block_max<NT>(tid < BW * TPR ? rs : 0.f, red);
  // hand-off 0: block j's diagonal of P (its own diagonal tile) and its inf-norm partial
  if (tid < BW) {
    const int i = BW * j + tid;
    coop_st(&xc->xb[0][i * DP + i], Tj[i * TLD + tid]);
  }
  if (tid == 0) coop_st(&xc->sc[0][j][1], rmax_j);
  COOP_STAMP(3);
  ok = coop_exchange(&xc->ticket, &xc->status, &ok_sh, spin_ticks, min_polls);
  COOP_STAMP(4);
  {
    const float dv = coop_ld(&xc->xb[0][(tid & (DP - 1)) * (DP + 1)]);
    float rm[kCoopWG];
#pragma unroll
    for (int i = 0; i < kCoopWG; ++i) rm[i] = coop_ld(&xc->sc[0][i][1]);
    if (tid < DP) diag[tid] = dv;
    rowmax_all = rm[0];
#pragma unroll
    for (int i = 1; i < kCoopWG; ++i) rowmax_all = fmaxf(rowmax_all, rm[i]);
  }
  const float rowmax = rowmax_all;
  __syncthreads();   // diag complete
  float tr = 0.f;
  for (int i = lane; i < DP; i += 64) tr += diag[i];
  for (int m = 32; m >= 1; m >>= 1) tr += shfl_xor(tr, m);
  float a2 = (float)DP / tr;
  if (a2 * rowmax >= 2.9f) a2 = 1.f / rowmax;
  const float a = sqrtf(a2);
  for (int e = tid; e < DP * DP; e += NT) {
    const int r = e / DP, c = e % DP;
    X[r * LD + c] *= a;
  }
  for (int e = tid; e < DP * BW; e += NT) {
    const int r = e / BW, cl = e % BW;
    const float pv = Tj[r * TLD + cl] * a2;
    const bool dg = r == BW * j + cl;
    err = fmaxf(err, fabsf(pv - (dg ? 1.f : 0.f)));
    Tj[r * TLD + cl] = (dg ? 1.5f : 0.f) - 0.5f * pv;
  }
  err = block_max<NT>(err, red);
  COOP_STAMP(5);

  int it = 0;
  float err_prev = 1.f;
  for (; ok; ++it) {
    const int par = (it + 1) & 1;   // parity 0 carried iteration 0's scalars
    xt_block(par);                   // speculative: dropped below if err stops the loop
    if (tid == 0) coop_st(&xc->sc[par][j][0], err);
    COOP_STAMP(6 + 5 * it);
    ok = coop_exchange(&xc->ticket, &xc->status, &ok_sh, spin_ticks, min_polls);
    COOP_STAMP(7 + 5 * it);
    if (!ok) break;
    float ev[kCoopWG];
#pragma unroll
    for (int i = 0; i < kCoopWG; ++i) ev[i] = coop_ld(&xc->sc[par][i][0]);
    gather_blocks(par);
    float e_all = ev[0];
#pragma unroll
    for (int i = 1; i < kCoopWG; ++i) e_all = fmaxf(e_all, ev[i]);
    if (e_all < tol || it >= max_iter) break;   // X stays (polar_ns breaks before the update)
    const bool last = (float)DP * e_all < DRSA_NS_LAST || (it > 0 && err_prev < 1e-4f && e_all > 0.25f * err_prev);
    err_prev = e_all;
    float* t = X; X = Xn; Xn = t;
    if (last) { ++it; break; }
    COOP_STAMP(8 + 5 * it);
    err = 0.f;
    gram_block(it + 1, err);
    COOP_STAMP(9 + 5 * it);
    err = block_max<NT>(err, red);
    COOP_STAMP(10 + 5 * it);
  }
  __syncthreads();
  COOP_STAMP(60);
  // U_out: workgroup j writes the real entries of its padded column block
#pragma unroll
  for (int q = 0; q < DP * BW / NT; ++q) {
    const int e = tid + q * NT, i = e / BW, pc = BW * j + e % BW;
    const int kc = pc / DKP, l = pc % DKP;
    if (i < d && kc < K && l < dk) U_out[i * d + kc * dk + l] = ok ? X[i * LD + pc] : __builtin_nanf("");
  }
  if (j == 0 && tid == 0) {
    const int slot = f_stride_by_counter ? *step_counter : 0;
    f_out[slot] = ok ? (float)f : __builtin_nanf("");
    if (f_stride_by_counter) *step_counter = slot + 1;
  }
  COOP_STAMP(61);
}

// ---------------------------------------------------------------------------
// batched independent problems (task-parallel DRSA grid, optsubspaces.py:17-23): one launch per
// phase for every problem of a batch that shares the padded geometry.  Problem p's partial runs
// on G workgroups (blockIdx.y = p; drsa_partial_grouped_kernel, whole leaf groups each), its reduce
// on blockIdx.y = p, its finish on workgroup p.  U ping-pongs between U_io and U_tmp by step parity.
// ---------------------------------------------------------------------------

// the per-leaf form for geometries whose grouped kernel does not fit the register file (concept
// width 64): workgroup l of problem p computes leaf l exactly as drsa_partial_kernel does
template <int DP, int DKP, bool VEC>
__global__ __launch_bounds__((partial_threads<DP, DKP>())) void drsa_partial_leaf_batched_kernel(
    const BatchDesc* __restrict__ bd, int parity) {
  const BatchDesc& q = bd[blockIdx.y];
  if ((int)blockIdx.x >= q.L) return;    // uniform per workgroup: before any barrier
  const float* U = parity ? q.U_tmp : q.U_io;
  const int d = q.d;
  partial_core<DP, DKP, 0, VEC>(
      q.A, q.C, q.N, d, q.K, q.dk, q.partials, q.rb_total, [] {},
      [&](int k, int j, int) { return U[(size_t)k * d + j]; }, [] {}, q.L);
}

__global__ __launch_bounds__(256) void drsa_reduce_batched_kernel(const BatchDesc* __restrict__ bd, int E, int ES) {
  const BatchDesc& q = bd[blockIdx.y];
  if (q.m > 0) reduce_grouped(q.partials, (q.L + kLeafGroup - 1) / kLeafGroup, 1, ES, E, q.gs);
  else reduce_grouped(q.partials, q.L, kLeafGroup, ES, E, q.gs);
}

// mode 0: U_in -> U_out = polar(U_in + G c), f(U_in) -> f_traj[counter++]; mode 1: f only
template <int DP>
__global__ __launch_bounds__(fin_threads<polar_dim<DP>()>()) void drsa_finish_batched_kernel(
    const BatchDesc* __restrict__ bd, int parity, int mode, float tol, int max_iter) {
  const BatchDesc& q = bd[blockIdx.x];
  const float* U = parity ? q.U_tmp : q.U_io;
  float* U_out = parity ? q.U_io : q.U_tmp;
  finish_body<DP>(q.gs, (double)q.N, q.d, q.K, q.DKP, U, U_out, q.f_traj, q.counter, 1, mode, tol, max_iter,
                  nullptr);
}

// One fused DRSA step for DP = 64 (C3, C4): every workgroup first finishes the PREVIOUS step
// redundantly -- f and c from the reduced slab gs, X = embed(U + Gt diag(c)), the same polar -- so
// U_next never leaves the CU before its partial uses it; workgroup 0 stores U_next and f(U).  The
// first tile's A/C loads are issued before the polar and land under it; U_next goes from LDS into
// the partial's registers.  Bit-identical to drsa_finish_kernel followed by drsa_partial_kernel
// (same code, same inputs in every workgroup); one launch and the U round trip fewer per step.
template <int DP, int DKP, bool VEC>
__global__ __launch_bounds__(fin_threads<polar_dim<DP>()>()) void drsa_fused_step_kernel(
    const float* __restrict__ A, const float* __restrict__ C, int64_t N, int d, int K, int dk,
    const float* __restrict__ gs, double n_total, const float* __restrict__ U, float* __restrict__ U_out,
    float* __restrict__ f_out, int* __restrict__ step_counter, float* __restrict__ partials, int64_t rb_total,
    float tol, int max_iter) {
  constexpr int PD = polar_dim<DP>(), NT = fin_threads<PD>(), LD = ns_ld<PD>();
  static_assert(PCfg<DP, DKP>::NT == NT, "fused step: the partial and the polar use one thread count");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* X = smem;
  float* T = X + PD * LD;
  float* red = T + PD * LD;
  float* scr = red + 64;
  __shared__ double dterm[128];
  __shared__ float cvec[128];
  __shared__ double fsh;
  auto pre = [&] {
    const double f = finish_prologue<DP>(gs, n_total, d, K, DKP, U, X, true, dterm, cvec, &fsh);
    polar_run<PD>(X, T, red, scr, tol, max_iter);   // ends with a barrier: X complete
    if (blockIdx.x == 0) {
      for (int e = threadIdx.x; e < d * d; e += NT) {
        const int i = e / d, j = e % d;
        U_out[e] = X[i * LD + (j / dk) * DKP + j % dk];
      }
      if (threadIdx.x == 0) {   // no counter: f_out[0]
        const int slot = step_counter ? *step_counter : 0;
        f_out[slot] = (float)f;
        if (step_counter) *step_counter = slot + 1;
      }
    }
  };
  partial_core<DP, DKP, 0, VEC>(
      A, C, N, d, K, dk, partials, rb_total, pre, [&](int k, int, int jp) { return X[k * LD + jp]; },
      [] { __syncthreads(); }, (int)gridDim.x);   // mid: every wave has read U from X before the tile store overwrites it
}

template <int DP, int DKP>
constexpr size_t fused_lds() {
  return PCfg<DP, DKP>::lds_bytes > finish_lds<DP>() ? PCfg<DP, DKP>::lds_bytes : finish_lds<DP>();
}

// polar only (orthogonalize API): any d <= 128, embedded as diag(V, I) in DP = pow2ceil(max(32, d))
template <int DP>
__global__ __launch_bounds__(fin_threads<DP>()) void polar_kernel(const float* __restrict__ V, int d,
                                                                  float* __restrict__ U_out, float tol, int max_iter,
                                                                  int* iters_out) {
  constexpr int NT = fin_threads<DP>(), LD = ns_ld<DP>();
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* X = smem;
  float* T = X + DP * LD;
  float* red = T + DP * LD;
  float* scr = red + 64;
#pragma unroll
  for (int q = 0; q < (DP * DP + NT - 1) / NT; ++q) {
    const int e = threadIdx.x + q * NT;
    const int i = e / DP, j = e % DP;
    const bool real = e < DP * DP && i < d && j < d;
    const float v = keep_or_zero(V[real ? (size_t)i * d + j : 0], real);
    if (e < DP * DP) X[i * LD + j] = (i < d && j < d) ? v : (i == j ? 1.f : 0.f);
  }
  const int it = polar_run<DP>(X, T, red, scr, tol, max_iter);
  for (int e = threadIdx.x; e < d * d; e += NT) U_out[e] = X[(e / d) * LD + e % d];
  if (iters_out && threadIdx.x == 0) *iters_out = it;
}

// ---------------------------------------------------------------------------
// host-side dispatch
// ---------------------------------------------------------------------------
struct PartialPlan {
  int grid;
  int64_t rb_total;
};

PartialPlan plan_partial(int64_t N) {
  const int64_t rbt = (N + 15) / 16;
  int64_t grid = kLeaves;            // one workgroup per leaf (= per CU on MI355X); 16-row blocks
  if (grid > rbt) grid = rbt;
  if (grid < 1) grid = 1;
  return {(int)grid, rbt};
}

template <int DP, int DKP, int DT>
int launch_partial(const void* A, const void* C, int64_t N, const Geom& g, const float* U, float* partials,
                   const PartialPlan& pl, hipStream_t s) {
  using Cfg = PCfg<DP, DKP>;
  auto kern = (g.d & 3) == 0 ? drsa_partial_kernel<DP, DKP, DT, true> : drsa_partial_kernel<DP, DKP, DT, false>;
  DRSA_SMEM(kern, Cfg::lds_bytes);
  hipLaunchKernelGGL(kern, dim3(pl.grid), dim3(Cfg::NT), Cfg::lds_bytes, s, A, C, N, g.d, g.K, g.dk, U, partials,
                     pl.rb_total);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

template <int DP, int DT>
int dispatch_partial_dp(const void* A, const void* C, int64_t N, const Geom& g, const float* U, float* partials,
                        const PartialPlan& pl, hipStream_t s) {
  switch (g.DKp) {
    case 1: return launch_partial<DP, 1, DT>(A, C, N, g, U, partials, pl, s);
    case 2: return launch_partial<DP, 2, DT>(A, C, N, g, U, partials, pl, s);
    case 4: return launch_partial<DP, 4, DT>(A, C, N, g, U, partials, pl, s);
    case 8: return launch_partial<DP, 8, DT>(A, C, N, g, U, partials, pl, s);
    case 16: return launch_partial<DP, 16, DT>(A, C, N, g, U, partials, pl, s);
    case 32: if constexpr (DP >= 32) return launch_partial<DP, 32, DT>(A, C, N, g, U, partials, pl, s); break;
    case 64: if constexpr (DP >= 64) return launch_partial<DP, 64, DT>(A, C, N, g, U, partials, pl, s); break;
    default: break;
  }
  drsa::set_error("drsa_partial: unsupported d=%d K=%d", g.d, g.K);
  return DRSA_EUNSUPPORTED;
}

int dispatch_partial(const void* A, const void* C, int64_t N, const Geom& g, const float* U, float* partials,
                     const PartialPlan& pl, hipStream_t s, int dt) {
  switch (g.DP) {
    case 16:
      if (dt) break;
      return dispatch_partial_dp<16, 0>(A, C, N, g, U, partials, pl, s);
    case 32: return dt == 1 ? dispatch_partial_dp<32, 1>(A, C, N, g, U, partials, pl, s)
                  : dt == 2 ? dispatch_partial_dp<32, 2>(A, C, N, g, U, partials, pl, s)
                            : dispatch_partial_dp<32, 0>(A, C, N, g, U, partials, pl, s);
    case 64: return dt == 1 ? dispatch_partial_dp<64, 1>(A, C, N, g, U, partials, pl, s)
                  : dt == 2 ? dispatch_partial_dp<64, 2>(A, C, N, g, U, partials, pl, s)
                            : dispatch_partial_dp<64, 0>(A, C, N, g, U, partials, pl, s);
    case 128: return dt == 1 ? dispatch_partial_dp<128, 1>(A, C, N, g, U, partials, pl, s)
                   : dt == 2 ? dispatch_partial_dp<128, 2>(A, C, N, g, U, partials, pl, s)
                             : dispatch_partial_dp<128, 0>(A, C, N, g, U, partials, pl, s);
  }
  drsa::set_error("drsa_partial: unsupported d=%d K=%d%s", g.d, g.K, dt == 1 ? " (bf16)" : dt == 2 ? " (fp16)" : "");
  return DRSA_EUNSUPPORTED;
}

template <int DP>
int launch_finish(const float* gs, double n_total, const Geom& g, const float* U, float* U_out, float* f_out,
                  int* counter, int by_counter, int mode, float tol, int max_iter, int* iters, hipStream_t s) {
  const size_t lds = finish_lds<DP>();
  DRSA_SMEM(drsa_finish_kernel<DP>, lds);
  hipLaunchKernelGGL(drsa_finish_kernel<DP>, dim3(1), dim3(fin_threads<polar_dim<DP>()>()), lds, s, gs, n_total, g.d,
                     g.K, g.DKp,
                     U, U_out, f_out, counter, by_counter, mode, tol, max_iter, iters);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

int dispatch_finish(const float* gs, double n_total, const Geom& g, const float* U, float* U_out, float* f_out,
                    int* counter, int by_counter, int mode, float tol, int max_iter, int* iters, hipStream_t s) {
  switch (g.DP) {
    case 16: return launch_finish<16>(gs, n_total, g, U, U_out, f_out, counter, by_counter, mode, tol, max_iter, iters, s);
    case 32: return launch_finish<32>(gs, n_total, g, U, U_out, f_out, counter, by_counter, mode, tol, max_iter, iters, s);
    case 64: return launch_finish<64>(gs, n_total, g, U, U_out, f_out, counter, by_counter, mode, tol, max_iter, iters, s);
    case 128: return launch_finish<128>(gs, n_total, g, U, U_out, f_out, counter, by_counter, mode, tol, max_iter, iters, s);
  }
  return DRSA_EUNSUPPORTED;
}

constexpr float kPolarTol = 4e-7f;
constexpr int kPolarMaxIter = 40;

int launch_reduce(const float* partials, const PartialPlan& pl, const Geom& g, float* gs_out, hipStream_t s) {
  const size_t E = slab_floats(g), ES = slab_stride(g);
  if (E <= 8192) {
    constexpr int CW = DRSA_REDUCE_CW;
    hipLaunchKernelGGL(drsa_reduce_kernel<CW>, dim3((unsigned)((E + CW - 1) / CW)), dim3(256), 0, s, partials, pl.grid,
                       (int)E, (int)ES, gs_out);
    DRSA_LAUNCH_CHECK();
    return DRSA_OK;
  }
  hipLaunchKernelGGL(drsa_reduce_kernel<64>, dim3((unsigned)((E + 63) / 64)), dim3(256), 0, s, partials, pl.grid, (int)E,
                     (int)ES, gs_out);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

// the fused step (drsa_fused_step_kernel) covers DP = 64 with concept blocks <= 16 wide (one
// 1024-thread workgroup shape for the partial and the polar): C3 and C4.
bool fused_ok(const Geom& g) {
  return g.DP == 64 && g.DKp <= 16;
}

template <int DKP>
int launch_fused(const float* A, const float* C, int64_t N, double n_total, const Geom& g, const float* gs,
                 const float* U, float* U_out, float* f_out, int* counter, float* partials, const PartialPlan& pl,
                 hipStream_t s) {
  auto kern = (g.d & 3) == 0 ? drsa_fused_step_kernel<64, DKP, true> : drsa_fused_step_kernel<64, DKP, false>;
  const size_t lds = fused_lds<64, DKP>();
  DRSA_SMEM(kern, lds);
  hipLaunchKernelGGL(kern, dim3(pl.grid), dim3(fin_threads<64>()), lds, s, A, C, N, g.d, g.K, g.dk, gs, n_total, U,
                     U_out, f_out, counter, partials, pl.rb_total, kPolarTol, kPolarMaxIter);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

// one fused step: gs (gradient slab at U over n_total rows) -> U_out = polar(U + G c), f(U) ->
// f_out[counter++] (f_out[0] without a counter), partial slabs of the N local rows at U_out ->
// reduce -> gs_out (gs_out may be gs: the reduce runs after every workgroup has read gs)
int fused_step(const float* A, const float* C, int64_t N, double n_total, const Geom& g, const float* gs,
               float* gs_out, const float* U, float* U_out, float* f_out, int* counter, void* ws, hipStream_t s) {
  const PartialPlan pl = plan_partial(N);
  float* partials = (float*)ws;
  int rc = DRSA_EUNSUPPORTED;
  switch (g.DKp) {
    case 1: rc = launch_fused<1>(A, C, N, n_total, g, gs, U, U_out, f_out, counter, partials, pl, s); break;
    case 2: rc = launch_fused<2>(A, C, N, n_total, g, gs, U, U_out, f_out, counter, partials, pl, s); break;
    case 4: rc = launch_fused<4>(A, C, N, n_total, g, gs, U, U_out, f_out, counter, partials, pl, s); break;
    case 8: rc = launch_fused<8>(A, C, N, n_total, g, gs, U, U_out, f_out, counter, partials, pl, s); break;
    case 16: rc = launch_fused<16>(A, C, N, n_total, g, gs, U, U_out, f_out, counter, partials, pl, s); break;
    default: drsa::set_error("drsa fused step: unsupported d=%d K=%d", g.d, g.K); return rc;
  }
  if (rc) return rc;
  return launch_reduce(partials, pl, g, gs_out, s);
}

// workspace layout: [partials grid*E] [gs E] [16 B pad]; DP = 128 adds the cooperative finish's
// exchange area (CoopXchg) at the next 256-B boundary after gs
size_t ws_bytes(int64_t N, const Geom& g) {
  const PartialPlan pl = plan_partial(N);
  const size_t base = ((size_t)pl.grid * slab_stride(g) + slab_floats(g)) * sizeof(float) + 64;
  return g.DP == 128 ? base + 256 + sizeof(CoopXchg) : base;
}

int partial_impl(const void* A, const void* C, int64_t N, int d, int K, const float* U, float* gs_out, void* ws,
                 size_t ws_size, void* stream, int dtype) {
  const Geom g = geom(d, K);
  DRSA_REQUIRE(g.ok, "drsa_partial: unsupported d=%d K=%d (need d <= 128, K | d, padded concept width <= 64 and "
               "K * padded width <= 128)", d, K);
  DRSA_REQUIRE(N >= 0, "drsa_partial: N < 0");
  DRSA_REQUIRE(dtype == 0 || ((dtype == 1 || dtype == 2) && g.DP >= 32),
               "drsa_partial: dtype must be 0 (fp32) or 1/2 (bf16/fp16, padded d >= 32)");
  DRSA_REQUIRE(A && C && U && gs_out, "drsa_partial: null pointer");
  hipStream_t s = (hipStream_t)stream;
  const size_t E = slab_floats(g);
  if (N == 0) {
    DRSA_HIP(hipMemsetAsync(gs_out, 0, E * sizeof(float), s));
    return DRSA_OK;
  }
  DRSA_REQUIRE(ws && ws_size >= ws_bytes(N, g), "drsa_partial: workspace too small");
  DRSA_REQUIRE(((uintptr_t)A % 16) == 0 && ((uintptr_t)C % 16) == 0, "drsa_partial: A/C must be 16B aligned");
  const PartialPlan pl = plan_partial(N);
  float* partials = (float*)ws;
  int rc = dispatch_partial(A, C, N, g, U, partials, pl, s, dtype);
  if (rc) return rc;
  return launch_reduce(partials, pl, g, gs_out, s);
}

float* ws_gs(void* ws, int64_t N, const Geom& g) {
  return (float*)ws + (size_t)plan_partial(N).grid * slab_stride(g);
}

CoopXchg* ws_xchg(void* ws, int64_t N, const Geom& g) {
  if (g.DP != 128) return nullptr;
  const uintptr_t e = (uintptr_t)(ws_gs(ws, N, g) + slab_floats(g));
  return (CoopXchg*)((e + 255) / 256 * 256);
}

// the exchange counter starts at 0 (kCoopWG arrivals per hand-off from there), the status word clear
int coop_reset(CoopXchg* xc, hipStream_t s) {
  static_assert(offsetof(CoopXchg, status) == offsetof(CoopXchg, ticket) + sizeof(unsigned), "ticket, status");
  if (xc) DRSA_HIP(hipMemsetAsync(&xc->ticket, 0, 2 * sizeof(unsigned), s));
  return DRSA_OK;
}

// spin budget of the cooperative finish (drsa_amd_debug_coop_spin_budget; default 100 ms + 20k polls)
long long g_coop_spin_ticks = kCoopSpinTicks;
int g_coop_min_polls = kCoopMinPolls;

bool stream_capturing(hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

// reads the run's sticky status word back (synchronises stream s); DRSA_ETIMEOUT if it is set
int coop_check(const CoopXchg* xc, hipStream_t s, const char* what) {
  if (!xc) return DRSA_OK;
  unsigned st = 0;
  DRSA_HIP(hipMemcpyAsync(&st, &xc->status, sizeof(unsigned), hipMemcpyDeviceToHost, s));
  DRSA_HIP(hipStreamSynchronize(s));
  if (st) {
    drsa::set_error("%s: a cooperative finish hand-off timed out (the %d workgroups were not co-resident "
                    "within the spin budget); U and f are NaN from that step on", what, kCoopWG);
    return DRSA_ETIMEOUT;
  }
  return DRSA_OK;
}

// a full finish step at DP = 128 on kCoopWG cooperating workgroups (bit-identical to dispatch_finish)
int launch_finish_coop(const float* gs, double n_total, const Geom& g, const float* U, float* U_out, float* f_out,
                       int* counter, int by_counter, CoopXchg* xc, hipStream_t s) {
  const size_t lds = coop_lds_bytes();
  DRSA_SMEM(drsa_finish_coop_kernel, lds);
  hipLaunchKernelGGL(drsa_finish_coop_kernel, dim3(kCoopWG), dim3(1024), lds, s, gs, n_total, g.d, g.K, g.DKp, U, U_out,
                     f_out, counter, by_counter, kPolarTol, kPolarMaxIter, xc, g_coop_spin_ticks, g_coop_min_polls);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

// finish of one step of drsa_run / run_multi: cooperative at DP = 128, else the one-workgroup kernel
int step_finish(const float* gs, double n_total, const Geom& g, const float* U, float* U_out, float* f_out,
                int* counter, CoopXchg* xc, hipStream_t s) {
  if (U_out && xc && g.DP == 128) return launch_finish_coop(gs, n_total, g, U, U_out, f_out, counter, 1, xc, s);
  return dispatch_finish(gs, n_total, g, U, U_out, f_out, counter, 1, U_out ? 0 : 1, kPolarTol, kPolarMaxIter, nullptr,
                         s);
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

#ifdef DRSA_COOP_STAMP
int drsa_amd_debug_coop_stamps(unsigned long long* host_out) {
  return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_coop_stamps), sizeof(g_coop_stamps));
}
#endif

int drsa_amd_drsa_coop_status(const void* ws, int64_t N, int d, int K, int* status_out, void* stream) {
  const Geom g = geom(d, K);
  DRSA_REQUIRE(g.ok && N > 0, "drsa_coop_status: unsupported d=%d K=%d or N <= 0", d, K);
  DRSA_REQUIRE(ws && status_out, "drsa_coop_status: null pointer");
  hipStream_t s = (hipStream_t)stream;
  DRSA_REQUIRE(!(s && stream_capturing(s)), "drsa_coop_status: the stream is being captured");
  *status_out = 0;
  const CoopXchg* xc = ws_xchg(const_cast<void*>(ws), N, g);
  if (!xc) return DRSA_OK;
  unsigned st = 0;
  DRSA_HIP(hipMemcpyAsync(&st, &xc->status, sizeof(unsigned), hipMemcpyDeviceToHost, s));
  DRSA_HIP(hipStreamSynchronize(s));
  *status_out = st ? 1 : 0;
  return DRSA_OK;
}

int drsa_amd_debug_coop_spin_budget(long long ticks) {
  DRSA_REQUIRE(ticks >= -1, "debug_coop_spin_budget: ticks must be >= -1");
  if (ticks < 0) {
    g_coop_spin_ticks = kCoopSpinTicks;
    g_coop_min_polls = kCoopMinPolls;
  } else {
    g_coop_spin_ticks = ticks;
    g_coop_min_polls = 0;
  }
  return DRSA_OK;
}

size_t drsa_amd_drsa_workspace_bytes(int64_t N, int d, int K) {
  const Geom g = geom(d, K);
  if (!g.ok || N <= 0) return 0;
  return ws_bytes(N, g);
}

size_t drsa_amd_drsa_slab_floats(int d, int K) {
  const Geom g = geom(d, K);
  return g.ok ? slab_floats(g) : 0;
}

int drsa_amd_drsa_partial(const float* A, const float* C, int64_t N, int d, int K, const float* U,
                          float* gs_out, void* ws, size_t ws_size, void* stream) {
  return partial_impl(A, C, N, d, K, U, gs_out, ws, ws_size, stream, 0);
}

int drsa_amd_drsa_partial_bf16(const uint16_t* A, const uint16_t* C, int64_t N, int d, int K, const float* U,
                               float* gs_out, void* ws, size_t ws_size, void* stream) {
  return partial_impl(A, C, N, d, K, U, gs_out, ws, ws_size, stream, 1);
}

int drsa_amd_drsa_partial_f16(const uint16_t* A, const uint16_t* C, int64_t N, int d, int K, const float* U,
                              float* gs_out, void* ws, size_t ws_size, void* stream) {
  return partial_impl(A, C, N, d, K, U, gs_out, ws, ws_size, stream, 2);
}

int drsa_amd_drsa_finish(const float* gs, int64_t N_total, int d, int K, const float* U, float* U_out,
                         float* f_out, int objective_only, int* iters_out, void* stream) {
  const Geom g = geom(d, K);
  DRSA_REQUIRE(g.ok, "drsa_finish: unsupported d=%d K=%d", d, K);
  DRSA_REQUIRE(N_total > 0, "drsa_finish: N_total must be > 0");
  DRSA_REQUIRE(gs && U && f_out && (objective_only || U_out), "drsa_finish: null pointer");
  DRSA_REQUIRE(objective_only || U != U_out, "drsa_finish: U and U_out must not alias");
  return dispatch_finish(gs, (double)N_total, g, U, U_out, f_out, nullptr, 0, objective_only ? 1 : 0, kPolarTol,
                         kPolarMaxIter, iters_out, (hipStream_t)stream);
}

int drsa_amd_drsa_fused_supported(int d, int K) { return fused_ok(geom(d, K)) ? 1 : 0; }

int drsa_amd_drsa_fused_step(const float* A, const float* C, int64_t N, int d, int K, const float* gs,
                             int64_t N_total, const float* U, float* U_out, float* f_out, float* gs_out, void* ws,
                             size_t ws_size, void* stream) {
  const Geom g = geom(d, K);
  DRSA_REQUIRE(g.ok && fused_ok(g), "drsa_fused_step: unsupported d=%d K=%d (drsa_amd_drsa_fused_supported)", d, K);
  DRSA_REQUIRE(N > 0 && N_total >= N, "drsa_fused_step: need 0 < N <= N_total");
  DRSA_REQUIRE(A && C && gs && U && U_out && f_out && gs_out, "drsa_fused_step: null pointer");
  DRSA_REQUIRE(U != U_out, "drsa_fused_step: U and U_out must not alias");
  DRSA_REQUIRE(ws && ws_size >= ws_bytes(N, g), "drsa_fused_step: workspace too small");
  DRSA_REQUIRE(((uintptr_t)A % 16) == 0 && ((uintptr_t)C % 16) == 0, "drsa_fused_step: A/C must be 16B aligned");
  return fused_step(A, C, N, (double)N_total, g, gs, gs_out, U, U_out, f_out, nullptr, ws, (hipStream_t)stream);
}

int drsa_amd_drsa_fused_step_counted(const float* A, const float* C, int64_t N, int d, int K, const float* gs,
                                     int64_t N_total, const float* U, float* U_out, float* f_traj, int* counter,
                                     float* gs_out, void* ws, size_t ws_size, void* stream) {
  const Geom g = geom(d, K);
  DRSA_REQUIRE(g.ok && fused_ok(g), "drsa_fused_step_counted: unsupported d=%d K=%d", d, K);
  DRSA_REQUIRE(N > 0 && N_total >= N, "drsa_fused_step_counted: need 0 < N <= N_total");
  DRSA_REQUIRE(A && C && gs && U && U_out && f_traj && counter && gs_out, "drsa_fused_step_counted: null pointer");
  DRSA_REQUIRE(U != U_out, "drsa_fused_step_counted: U and U_out must not alias");
  DRSA_REQUIRE(ws && ws_size >= ws_bytes(N, g), "drsa_fused_step_counted: workspace too small");
  DRSA_REQUIRE(((uintptr_t)A % 16) == 0 && ((uintptr_t)C % 16) == 0, "drsa_fused_step_counted: A/C must be 16B aligned");
  return fused_step(A, C, N, (double)N_total, g, gs, gs_out, U, U_out, f_traj, counter, ws, (hipStream_t)stream);
}

int drsa_amd_drsa_finish_counted(const float* gs, int64_t N_total, int d, int K, const float* U, float* U_out,
                                 float* f_traj, int* counter, void* stream) {
  const Geom g = geom(d, K);
  DRSA_REQUIRE(g.ok, "drsa_finish_counted: unsupported d=%d K=%d", d, K);
  DRSA_REQUIRE(N_total > 0, "drsa_finish_counted: N_total must be > 0");
  DRSA_REQUIRE(gs && U && U_out && f_traj && counter, "drsa_finish_counted: null pointer");
  DRSA_REQUIRE(U != U_out, "drsa_finish_counted: U and U_out must not alias");
  return dispatch_finish(gs, (double)N_total, g, U, U_out, f_traj, counter, 1, 0, kPolarTol, kPolarMaxIter, nullptr,
                         (hipStream_t)stream);
}

int drsa_amd_drsa_step(const float* A, const float* C, int64_t N, int d, int K, const float* U,
                       float* U_out, float* f_out, void* ws, size_t ws_size, void* stream) {
  const Geom g = geom(d, K);
  DRSA_REQUIRE(g.ok, "drsa_step: unsupported d=%d K=%d", d, K);
  DRSA_REQUIRE(N > 0, "drsa_step: N must be > 0");
  DRSA_REQUIRE(U != U_out, "drsa_step: U and U_out must not alias");
  DRSA_REQUIRE(ws && ws_size >= ws_bytes(N, g), "drsa_step: workspace too small");
  float* gs = ws_gs(ws, N, g);
  int rc = drsa_amd_drsa_partial(A, C, N, d, K, U, gs, ws, ws_size, stream);
  if (rc) return rc;
  return drsa_amd_drsa_finish(gs, N, d, K, U, U_out, f_out, 0, nullptr, stream);
}

int drsa_amd_drsa_objective(const float* A, const float* C, int64_t N, int d, int K, const float* U,
                            float* f_out, void* ws, size_t ws_size, void* stream) {
  const Geom g = geom(d, K);
  DRSA_REQUIRE(g.ok, "drsa_objective: unsupported d=%d K=%d", d, K);
  DRSA_REQUIRE(N > 0, "drsa_objective: N must be > 0");
  DRSA_REQUIRE(ws && ws_size >= ws_bytes(N, g), "drsa_objective: workspace too small");
  float* gs = ws_gs(ws, N, g);
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
  const Geom g = geom(d, K);
  DRSA_REQUIRE(g.ok, "drsa_run: unsupported d=%d K=%d", d, K);
  DRSA_REQUIRE(N > 0 && steps >= 0, "drsa_run: bad N/steps");
  DRSA_REQUIRE(ws && ws_size >= ws_bytes(N, g), "drsa_run: workspace too small");
  DRSA_REQUIRE(A && C && U_io && U_tmp && f_traj && counter, "drsa_run: null pointer");
  hipStream_t s = (hipStream_t)stream;
  float* gs = ws_gs(ws, N, g);
  // already inside a stream capture (e.g. a torch CUDA graph): record the plain sequence, and leave
  // the cooperative finish's status check to the caller (drsa_amd_drsa_coop_status)
  const bool capturing = s && stream_capturing(s);
  if (capturing) use_graph = 0;
  DRSA_HIP(hipMemsetAsync(counter, 0, sizeof(int), s));
  CoopXchg* xc = ws_xchg(ws, N, g);
  if (int rc = coop_reset(xc, s)) return rc;
  // fused: the gradient at U_0 first, then per step one fused launch (finish of the previous step
  // + partial at the new U) and the slab reduce; the final objective reads the last gs
  const bool fused = fused_ok(g);
  if (fused) {
    int rc = drsa_amd_drsa_partial(A, C, N, d, K, U_io, gs, ws, ws_size, stream);
    if (rc) return rc;
  }
  auto one = [&](const float* Uin, float* Uout) -> int {
    if (fused) return fused_step(A, C, N, (double)N, g, gs, gs, Uin, Uout, f_traj, counter, ws, s);
    int rc = drsa_amd_drsa_partial(A, C, N, d, K, Uin, gs, ws, ws_size, stream);
    if (rc) return rc;
    return step_finish(gs, (double)N, g, Uin, Uout, f_traj, counter, xc, s);
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
    hipError_t ie = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    if (ie != hipSuccess) { (void)hipGraphDestroy(graph); DRSA_HIP(ie); }
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
  if (!fused) {
    int rc = drsa_amd_drsa_partial(A, C, N, d, K, U_io, gs, ws, ws_size, stream);
    if (rc) return rc;
  }
  int rc = dispatch_finish(gs, (double)N, g, U_io, nullptr, f_traj, counter, 1, 1, kPolarTol, kPolarMaxIter, nullptr, s);
  if (rc || capturing || steps == 0) return rc;
  return coop_check(xc, s, "drsa_run");
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
    const Geom g = geom(q.d, q.K);
    DRSA_REQUIRE(g.ok, "drsa_run_multi: problem %d unsupported d=%d K=%d", p, q.d, q.K);
    DRSA_REQUIRE(q.N > 0 && q.A && q.C && q.U_io && q.U_tmp && q.f_traj && q.counter && q.ws,
                 "drsa_run_multi: problem %d has null pointers or N <= 0", p);
    DRSA_REQUIRE(q.ws_size >= ws_bytes(q.N, g), "drsa_run_multi: problem %d workspace too small", p);
    DRSA_REQUIRE(q.dtype == 0 || ((q.dtype == 1 || q.dtype == 2) && g.DP >= 32),
                 "drsa_run_multi: problem %d: dtype must be 0 (fp32) or 1/2 (bf16/fp16, padded d >= 32)", p);
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
  // inside a caller's stream capture (a torch CUDA graph of the whole run): record the forked plain
  // sequence into it (no graph of our own, no host synchronisation, no status read-back)
  const bool capturing = s && stream_capturing(s);
  if (capturing) use_graph = 0;
  // side streams and fork/join events come from a per-thread, per-device pool that lives as long
  // as the thread: a captured graph's forks must not be destroyed before the capture ends
  struct SidePool {
    hipStream_t st[64] = {nullptr};
    hipEvent_t join[64] = {nullptr};
    hipEvent_t fork = nullptr;
  };
  thread_local SidePool pools[16];
  int dev = 0;
  DRSA_HIP(hipGetDevice(&dev));
  DRSA_REQUIRE(dev >= 0 && dev < 16, "drsa_run_multi: device index %d >= 16", dev);
  SidePool& pool = pools[dev];
  hipStream_t* side = pool.st;
  hipEvent_t* ev_join = pool.join;
  int rc = DRSA_OK;
  auto cleanup = [&]() {};
  auto hip_ok = [&](hipError_t e, const char* what) -> bool {
    if (e == hipSuccess) return true;
    drsa::set_error("drsa_run_multi: %s: %s", what, hipGetErrorString(e));
    rc = (int)e;
    return false;
  };
  if (!pool.fork && !hip_ok(hipEventCreateWithFlags(&pool.fork, hipEventDisableTiming), "event")) return rc;
  hipEvent_t ev_fork = pool.fork;
  for (int p = 0; p < P; ++p) {
    if ((!side[p] && !hip_ok(hipStreamCreateWithFlags(&side[p], hipStreamNonBlocking), "stream")) ||
        (!ev_join[p] && !hip_ok(hipEventCreateWithFlags(&ev_join[p], hipEventDisableTiming), "event"))) {
      return rc;
    }
    const drsa_amd_problem_t& q = probs[p];
    if (!hip_ok(hipMemsetAsync(q.counter, 0, sizeof(int), s), "memset")) { cleanup(); return rc; }
    if (int r = coop_reset(ws_xchg(q.ws, q.N, geom(q.d, q.K)), s)) { cleanup(); return r; }
  }
  // one step of problem p on stream st: U_in -> U_out, f -> f_traj[counter++]
  auto one = [&](int p, hipStream_t st, const float* Uin, float* Uout) -> int {
    const drsa_amd_problem_t& q = probs[p];
    const Geom g = geom(q.d, q.K);
    float* gs = ws_gs(q.ws, q.N, g);
    int r = partial_impl(q.A, q.C, q.N, q.d, q.K, Uin, gs, q.ws, q.ws_size, st, q.dtype);
    if (r) return r;
    return step_finish(gs, (double)q.N, g, Uin, Uout, q.f_traj, q.counter, ws_xchg(q.ws, q.N, g), st);
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
  if (steps == 0 || capturing) return DRSA_OK;
  for (int p = 0; p < P; ++p) {
    const drsa_amd_problem_t& q = probs[p];
    if (int rc2 = coop_check(ws_xchg(q.ws, q.N, geom(q.d, q.K)), s, "drsa_run_multi")) return rc2;
  }
  return DRSA_OK;
}

// P independent fp32 problems of one padded geometry advanced together, one launch per phase
// (partial / reduce / finish) for all of them -- the task-parallel DRSA grid of optsubspaces.py:17-23.
// blocks: workgroups per problem for the partial (0: about 4 waves of workgroups over the chip).
// Row partition, and so the fp32 summation order, depends on blocks: deterministic for a given
// value.  Graph-captured two steps at a time like drsa_amd_drsa_run.
int drsa_amd_drsa_run_batched(int P, const drsa_amd_problem_t* probs, int steps, int blocks, int use_graph,
                              void* stream) {
  DRSA_REQUIRE(P >= 1 && probs, "drsa_run_batched: P must be >= 1");
  DRSA_REQUIRE(steps >= 0, "drsa_run_batched: steps < 0");
  const Geom g0 = geom(probs[0].d, probs[0].K);
  DRSA_REQUIRE(g0.ok, "drsa_run_batched: problem 0 unsupported d=%d K=%d", probs[0].d, probs[0].K);
  bool vec = true;
  int64_t min_rbt = INT64_MAX;
  for (int p = 0; p < P; ++p) {
    const drsa_amd_problem_t& q = probs[p];
    const Geom g = geom(q.d, q.K);
    DRSA_REQUIRE(g.ok && g.DP == g0.DP && g.DKp == g0.DKp,
                 "drsa_run_batched: problem %d (d=%d K=%d) does not share the padded geometry of problem 0", p,
                 q.d, q.K);
    DRSA_REQUIRE(q.dtype == 0, "drsa_run_batched: fp32 problems only (problem %d)", p);
    DRSA_REQUIRE(q.N > 0 && q.A && q.C && q.U_io && q.U_tmp && q.f_traj && q.counter && q.ws,
                 "drsa_run_batched: problem %d has null pointers or N <= 0", p);
    DRSA_REQUIRE(q.ws_size >= ws_bytes(q.N, g), "drsa_run_batched: problem %d workspace too small", p);
    DRSA_REQUIRE(((uintptr_t)q.A % 16) == 0 && ((uintptr_t)q.C % 16) == 0, "drsa_run_batched: A/C 16B alignment");
    vec = vec && (q.d & 3) == 0;
    const int64_t rbt = (q.N + 15) / 16;
    if (rbt < min_rbt) min_rbt = rbt;
  }
  hipStream_t s = (hipStream_t)stream;
  if (s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    DRSA_REQUIRE(!(hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone),
                 "drsa_run_batched: not capturable (allocates its descriptor table); use drsa_run_multi");
  }
  // workgroups per problem: `blocks`, or about 16 waves of one-workgroup-per-CU launches over the
  // chip (the 90-problem grid: one leaf group per workgroup, 36.4k problem-steps/s against 36.0k
  // at two groups); each owns m = ceil(groups / G) whole leaf groups (the result does not depend on it)
  const int cu = drsa::cu_count();
  int Greq = blocks > 0 ? blocks : (16 * cu + P - 1) / P;
  if (Greq < 1) Greq = 1;
  (void)min_rbt;
  const Geom& g = g0;
  const size_t E = slab_floats(g), ES = slab_stride(g);
  int G = 1;
  const bool leafwise = g0.DKp >= 64;          // see drsa_partial_leaf_batched_kernel
  // descriptor table on the device
  BatchDesc* hd = (BatchDesc*)malloc(sizeof(BatchDesc) * (size_t)P);
  DRSA_REQUIRE(hd, "drsa_run_batched: host allocation failed");
  for (int p = 0; p < P; ++p) {
    const drsa_amd_problem_t& q = probs[p];
    const Geom gq = geom(q.d, q.K);
    const PartialPlan pl = plan_partial(q.N);   // the leaves of drsa_run's partition
    const int ngrp = (pl.grid + kLeafGroup - 1) / kLeafGroup;
    const int m = leafwise ? 0 : (ngrp + Greq - 1) / Greq;
    const int Gp = leafwise ? pl.grid : (ngrp + m - 1) / m;
    if (Gp > G) G = Gp;
    hd[p] = BatchDesc{q.A, q.C, q.N, pl.rb_total, q.d, q.K, q.d / q.K, gq.DKp, Gp, pl.grid, m, q.U_io, q.U_tmp,
                      q.f_traj, q.counter, (float*)q.ws, ws_gs(q.ws, q.N, gq)};
  }
  BatchDesc* dd = nullptr;
  hipError_t e = hipMalloc((void**)&dd, sizeof(BatchDesc) * (size_t)P);
  if (e != hipSuccess) { free(hd); DRSA_HIP(e); }
  int rc = DRSA_OK;
  auto ok = [&](hipError_t err, const char* what) -> bool {
    if (err == hipSuccess) return true;
    drsa::set_error("drsa_run_batched: %s: %s", what, hipGetErrorString(err));
    rc = (int)err;
    return false;
  };
  if (!ok(hipMemcpyAsync(dd, hd, sizeof(BatchDesc) * (size_t)P, hipMemcpyHostToDevice, s), "copy")) goto done;
  for (int p = 0; p < P && !rc; ++p) ok(hipMemsetAsync(probs[p].counter, 0, sizeof(int), s), "memset");
  if (rc) goto done;
  {
    // launchers for the geometry
    auto launch_phase = [&](int parity, int final_obj) -> int {
      auto part = [&](auto dpt, auto dkt) -> int {
        constexpr int DP = decltype(dpt)::value, DKP = decltype(dkt)::value;
        using Cfg = PCfg<DP, DKP>;
        if constexpr (DKP >= 64) {     // = leafwise
          auto kern = vec ? drsa_partial_leaf_batched_kernel<DP, DKP, true> : drsa_partial_leaf_batched_kernel<DP, DKP, false>;
          DRSA_SMEM(kern, Cfg::lds_bytes);
          hipLaunchKernelGGL(kern, dim3(G, P), dim3(Cfg::NT), Cfg::lds_bytes, s, dd, parity);
        } else {
          auto kern = vec ? drsa_partial_grouped_kernel<DP, DKP, true> : drsa_partial_grouped_kernel<DP, DKP, false>;
          DRSA_SMEM(kern, Cfg::glds_bytes);
          hipLaunchKernelGGL(kern, dim3(G, P), dim3(Cfg::NT), Cfg::glds_bytes, s, dd, parity);
        }
        DRSA_LAUNCH_CHECK();
        return DRSA_OK;
      };
      int r = DRSA_EUNSUPPORTED;
      using I = std::integral_constant<int, 1>;
      (void)sizeof(I);
#define PB_DK(DPV)                                                                                            \
  switch (g.DKp) {                                                                                            \
    case 1: r = part(std::integral_constant<int, DPV>{}, std::integral_constant<int, 1>{}); break;            \
    case 2: r = part(std::integral_constant<int, DPV>{}, std::integral_constant<int, 2>{}); break;            \
    case 4: r = part(std::integral_constant<int, DPV>{}, std::integral_constant<int, 4>{}); break;            \
    case 8: r = part(std::integral_constant<int, DPV>{}, std::integral_constant<int, 8>{}); break;            \
    case 16: r = part(std::integral_constant<int, DPV>{}, std::integral_constant<int, 16>{}); break;          \
    case 32: if constexpr (DPV >= 32) r = part(std::integral_constant<int, DPV>{}, std::integral_constant<int, (DPV >= 32 ? 32 : 1)>{}); break; \
    case 64: if constexpr (DPV >= 64) r = part(std::integral_constant<int, DPV>{}, std::integral_constant<int, (DPV >= 64 ? 64 : 1)>{}); break; \
    default: break;                                                                                           \
  }
      switch (g.DP) {
        case 16: PB_DK(16) break;
        case 32: PB_DK(32) break;
        case 64: PB_DK(64) break;
        case 128: PB_DK(128) break;
      }
#undef PB_DK
      if (r) return r;
      hipLaunchKernelGGL(drsa_reduce_batched_kernel, dim3((unsigned)((E + 63) / 64), P), dim3(256), 0, s, dd,
                         (int)E, (int)ES);
      DRSA_LAUNCH_CHECK();
      auto fin = [&](auto dpt) -> int {
        constexpr int DP = decltype(dpt)::value;
        const size_t lds = finish_lds<DP>();
        DRSA_SMEM(drsa_finish_batched_kernel<DP>, lds);
        hipLaunchKernelGGL(drsa_finish_batched_kernel<DP>, dim3(P), dim3(fin_threads<polar_dim<DP>()>()), lds, s, dd,
                           parity, final_obj ? 1 : 0, kPolarTol, kPolarMaxIter);
        DRSA_LAUNCH_CHECK();
        return DRSA_OK;
      };
      switch (g.DP) {
        case 16: return fin(std::integral_constant<int, 16>{});
        case 32: return fin(std::integral_constant<int, 32>{});
        case 64: return fin(std::integral_constant<int, 64>{});
        default: return fin(std::integral_constant<int, 128>{});
      }
    };
    int done_steps = 0;
    if (use_graph && steps >= 2 && s) {
      hipGraph_t graph = nullptr;
      hipGraphExec_t exec = nullptr;
      if (!ok(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal), "capture")) goto done;
      int r1 = launch_phase(0, 0);
      int r2 = r1 ? r1 : launch_phase(1, 0);
      hipError_t ce = hipStreamEndCapture(s, &graph);
      if (r2) { if (graph) (void)hipGraphDestroy(graph); rc = r2; goto done; }
      if (!ok(ce, "end capture") || !ok(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0), "instantiate")) {
        if (graph) (void)hipGraphDestroy(graph);
        goto done;
      }
      for (; done_steps + 2 <= steps; done_steps += 2)
        if (!ok(hipGraphLaunch(exec, s), "graph launch")) break;
      (void)hipGraphExecDestroy(exec);
      (void)hipGraphDestroy(graph);
      if (rc) goto done;
    }
    for (; done_steps < steps; ++done_steps) {
      int r = launch_phase(done_steps & 1, 0);
      if (r) { rc = r; goto done; }
    }
    if (steps & 1) {   // U_S sits in U_tmp: bring it home
      for (int p = 0; p < P; ++p)
        if (!ok(hipMemcpyAsync(probs[p].U_io, probs[p].U_tmp, (size_t)probs[p].d * probs[p].d * sizeof(float),
                               hipMemcpyDeviceToDevice, s), "copy")) goto done;
    }
    {
      int r = launch_phase(0, 1);   // final objective at U_S -> f_traj[steps]
      if (r) { rc = r; goto done; }
    }
  }
done:
  (void)hipStreamSynchronize(s);
  (void)hipFree(dd);
  free(hd);
  return rc;
}

int drsa_amd_polar(const float* V, int d, float* U_out, int* iters_out, void* stream) {
  DRSA_REQUIRE(d >= 1 && d <= 128, "polar: unsupported d=%d (1..128)", d);
  DRSA_REQUIRE(V && U_out, "polar: null pointer");
  hipStream_t s = (hipStream_t)stream;
  auto go = [&](auto tag) -> int {
    constexpr int DP = decltype(tag)::value;
    const size_t lds = finish_lds<DP>();
    DRSA_SMEM(polar_kernel<DP>, lds);
    hipLaunchKernelGGL(polar_kernel<DP>, dim3(1), dim3(fin_threads<DP>()), lds, s, V, d, U_out, kPolarTol,
                       kPolarMaxIter, iters_out);
    DRSA_LAUNCH_CHECK();
    return DRSA_OK;
  };
  const int DP = pow2ceil(d < 32 ? 32 : d);
  switch (DP) {
    case 32: return go(std::integral_constant<int, 32>{});
    case 64: return go(std::integral_constant<int, 64>{});
    default: return go(std::integral_constant<int, 128>{});
  }
}

}  // extern "C"
