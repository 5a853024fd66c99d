// Backward 3x3 conv with all K+1 relevance clones of one sample in one workgroup.
//
// The DRSA subspace backward (reference cxai/xai/explain/explainer.py:92, the batch replicated
// K+1 times) runs every layer below the projection on K+1 relevance clones that share the
// forward state (x, den, the pool argmax).  conv3x3_kernel (lrp_conv_kernel.h) gives every
// (tile, clone) its own workgroup; this kernel gives a tile of ONE sample a workgroup and loops
// over the clones, so
//   * x and den (the rule's input and the next layer's denominator, per sample) are read from
//     HBM once per tile instead of once per clone (L2 holds them between clones);
//   * the epilogue of clone c-1 (x * R, R / stab(den), ReLU mask, store) is spread over the
//     input-channel chunks of clone c and runs in the same basic block as clone c's MFMA loop:
//     its VALU and memory work hides under the MFMAs instead of stalling them.
// Branch-free epilogue: x/den are read and R written with buffer instructions whose offset is
// pushed out of range for masked lanes (the hardware drops the store / returns 0), so the first
// clone's "previous epilogue" (nothing to store) costs no branch either.
//
// Status: opt-in (DRSA_AMD_CONV_CLONES=1).  Its registers (two accumulator sets + staging) allow
// 2 waves/SIMD, and at that occupancy the per-chunk LDS staging latency is exposed: 2.12 ms vs
// 1.92 ms for the per-clone kernel on GTZAN features.3 (B=512 x 5 clones), DESIGN.md section 4.
//
// Arithmetic per output element is exactly conv3x3_kernel's (the same k-ordered MFMA chain and
// the same epilogue expressions), so results are bit-identical to it and to oracle/lrp_exact.c.
#pragma once
#include "lrp_conv_kernel.h"

namespace drsa_conv {

__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float buf_ld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ void buf_st(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, 0);
}
constexpr uint32_t kOOB = 0x80000000u;   // >= every slice size: load -> 0, store dropped

template <int CIN, int COUT, int TH, int TW, int MW, int CIC, int NG, int AMODE>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(
    ConvCfg<CIN, COUT, TH, TW, MW, CIC, NG, AMODE, EPI_BWDC>::WPE))) void conv3x3_bwd_clones_kernel(ConvArgs a) {
  using Cfg = ConvCfg<CIN, COUT, TH, TW, MW, CIC, NG, AMODE, EPI_BWDC>;
  constexpr int MTH = Cfg::MTH, MTW = Cfg::MTW, MTX = Cfg::MTX;
  constexpr int WM = Cfg::WM, MPW = Cfg::MPW, NPW = Cfg::NPW, NCHUNK = Cfg::NCHUNK;
  constexpr int NE = MPW * NPW * 16;                       // output elements per lane and clone
  constexpr int EF = (NE + NCHUNK - 1) / NCHUNK;           // ... handled per chunk of the next clone
  static_assert(NG == 1 || NG == 2, "backward uses one or two weight sets");

  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* halo = smem;                                      // [CIC][PLANE]
  float* wl = smem + CIC * Cfg::PLANE;                     // [NG][KCP][COUT]

  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  const int H = a.H, W = a.W, HW = H * W;
  const int tiles_x = (W + TW - 1) / TW;
  const int ty0 = (blockIdx.x / tiles_x) * TH;
  const int tx0 = (blockIdx.x % tiles_x) * TW;
  const int bs = blockIdx.y, C = a.clones;
  const int wm = w % WM, wn = w / WM;
  const bool active = w < WM * Cfg::WN;
  const int h = lane >> 5;

  // lane l: pixel (pix_y, pix_x) of m-tile u (row-major), registers r: channels
  // (wn*NPW + v)*32 + (r&3) + 8(r>>2) + 4h
  int pix_off[MPW];
  uint32_t pbyte[MPW];                                     // byte offset of the pixel in a plane, or kOOB
#pragma unroll
  for (int u = 0; u < MPW; ++u) {
    const int mt = wm * MPW + u, p = lane & 31;
    const int py = (mt / MTX) * MTH + p / MTW, px = (mt % MTX) * MTW + p % MTW;
    pix_off[u] = py * Cfg::RS + px + XO;
    const int gy = ty0 + py, gx = tx0 + px;
    pbyte[u] = (active && gy < H && gx < W) ? (uint32_t)(gy * W + gx) * 4u : kOOB;
  }
  const int ch_lane = wn * NPW * 32 + 4 * h;               // channel of register 0, n-tile 0
  const uint32_t plane_b = (uint32_t)HW * 4u;
  const uint32_t slice_b = (uint32_t)a.cout * plane_b;    // one sample's [cout][H][W]
  // element e -> byte offset in a slice (or kOOB)
  auto eoff = [&](int e) -> uint32_t {
    const int v = e / (MPW * 16), u = (e / 16) % MPW, r = e & 15;
    const int cr = v * 32 + (r & 3) + 8 * (r >> 2);        // compile-time after unrolling
    const int co = ch_lane + cr;
    return (co < a.cout && pbyte[u] != kOOB) ? pbyte[u] + (uint32_t)co * plane_b : kOOB;
  };

  const bool need_x = a.xmode != XM_NONE || a.post != POST_NONE;
  const bool need_d = a.post == POST_DIV;
  const __amdgpu_buffer_rsrc_t rx = buf_rsrc(need_x ? a.x + (size_t)bs * a.cout * HW : a.out, need_x ? slice_b : 0u);
  const __amdgpu_buffer_rsrc_t rd = buf_rsrc(need_d ? a.den + (size_t)bs * a.cout * HW : a.out, need_d ? slice_b : 0u);
  const bool mul_x = a.xmode != XM_NONE, split_x = a.xmode == XM_SPLIT;
  const bool post_div = a.post == POST_DIV, post_any = a.post != POST_NONE;
  const float eps = a.eps;

  f32x16 acc[NG][MPW][NPW], prev[NG][MPW][NPW];
#pragma unroll
  for (int g = 0; g < NG; ++g)
#pragma unroll
    for (int u = 0; u < MPW; ++u)
#pragma unroll
      for (int v = 0; v < NPW; ++v)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[g][u][v][r] = 0.f;

  // epilogue elements [e0, e0 + EF) of the clone held in prev: loads, then math + stores
  auto epi_load = [&](int e0, float (&xv)[EF], float (&dv)[EF], bool live) {
#pragma unroll
    for (int i = 0; i < EF; ++i) {
      const uint32_t o = (live && e0 + i < NE) ? eoff(e0 + i) : kOOB;
      xv[i] = buf_ld(rx, o);
      dv[i] = buf_ld(rd, o);
    }
  };
  auto epi_store = [&](int e0, const float (&xv)[EF], const float (&dv)[EF], __amdgpu_buffer_rsrc_t ro, bool live) {
#pragma unroll
    for (int i = 0; i < EF; ++i) {
      const int e = e0 + i;
      if (e >= NE) break;
      const int v = e / (MPW * 16), u = (e / 16) % MPW, r = e & 15;
      const float x = xv[i];
      // branch-free forms of conv3x3_kernel's epilogue (uniform selects, same roundings):
      //   XM_NONE: R * 1 = R;  XM_MUL: x * R;  XM_SPLIT: max(x, 0) * R [+ min(x, 0) * R1]
      float xm = split_x ? fmaxf(x, 0.f) : x;
      xm = mul_x ? xm : 1.f;
      float R = xm * prev[0][u][v][r];
      if constexpr (NG >= 2) {
        const float R1 = R + fminf(x, 0.f) * prev[1][u][v][r];   // -ffp-contract=off: two roundings
        R = split_x ? R1 : R;
      }
      //   POST_DIV: x > 0 ? R / stab(den) : 0;  POST_MASK: x > 0 ? R : 0
      const float q = div_nb(R, stab(dv[i], eps));
      R = post_div ? q : R;
      R = (post_any && !(x > 0.f)) ? 0.f : R;
      buf_st(ro, live ? eoff(e) : kOOB, R);
    }
  };

  Stager<Cfg> stg;
  stg.load(a, 0, tid, ty0, tx0, bs * C, bs);
  for (int c = 0; c < C; ++c) {
    const int bq = bs * C + c;
    // the previous clone's accumulators become the epilogue's input
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int u = 0; u < MPW; ++u)
#pragma unroll
        for (int v = 0; v < NPW; ++v) {
          prev[g][u][v] = acc[g][u][v];
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[g][u][v][r] = 0.f;
        }
    const bool live = c > 0;
    // fresh copies per clone: keeps LLVM from hoisting every chunk's staging addresses out of
    // the clone loop (they would stay live across it: spills)
    int tid_c = tid, ty0_c = ty0, tx0_c = tx0;
    asm volatile("" : "+v"(tid_c));
    asm volatile("" : "+s"(ty0_c), "+s"(tx0_c));
    const __amdgpu_buffer_rsrc_t ro = buf_rsrc(a.out + (size_t)(bq - (live ? 1 : 0)) * a.cout * HW, slice_b);
#pragma unroll
    for (int chunk = 0; chunk < NCHUNK; ++chunk) {
      __syncthreads();
      stg.store(halo, wl, tid);
      __syncthreads();
      // the next chunk, or the next clone's first chunk (re-loads the last clone's at the end:
      // unconditional, so the chunk stays one basic block)
      if (chunk + 1 < NCHUNK) stg.load(a, (chunk + 1) * CIC, tid_c, ty0_c, tx0_c, bq, bs);
      else stg.load(a, 0, tid_c, ty0_c, tx0_c, c + 1 < C ? bq + 1 : bq, bs);
      float xv[EF], dv[EF];
      epi_load(chunk * EF, xv, dv, live);
      if (WM * Cfg::WN == 4 || active) mfma_chunk<Cfg, Cfg::PD>(halo, wl, pix_off, lane, wn, acc);
      epi_store(chunk * EF, xv, dv, ro, live);
    }
  }
  // the last clone's epilogue
#pragma unroll
  for (int g = 0; g < NG; ++g)
#pragma unroll
    for (int u = 0; u < MPW; ++u)
#pragma unroll
      for (int v = 0; v < NPW; ++v) prev[g][u][v] = acc[g][u][v];
  const __amdgpu_buffer_rsrc_t ro = buf_rsrc(a.out + (size_t)(bs * C + C - 1) * a.cout * HW, slice_b);
#pragma unroll
  for (int chunk = 0; chunk < NCHUNK; ++chunk) {
    float xv[EF], dv[EF];
    epi_load(chunk * EF, xv, dv, true);
    epi_store(chunk * EF, xv, dv, ro, true);
  }
}

#define CONVC_ENTRY(CIN, COUT, TH, TW, MW, CIC, NG, AM)                                                      \
  drsa_conv::Entry{CIN, COUT, TH, TW, MW, CIC, NG, AM, drsa_conv::EPI_BWDC,                                  \
                   drsa_conv::conv3x3_bwd_clones_kernel<CIN, COUT, TH, TW, MW, CIC, NG, AM>,                 \
                   drsa_conv::ConvCfg<CIN, COUT, TH, TW, MW, CIC, NG, AM, drsa_conv::EPI_BWDC>::lds_floats * \
                       sizeof(float)}

#define CONVC_FAMILY(CIN, COUT, CIC, NG, AM)          \
  CONVC_ENTRY(CIN, COUT, 8, 32, 8, CIC, NG, AM),      \
  CONVC_ENTRY(CIN, COUT, 8, 16, 8, CIC, NG, AM),      \
  CONVC_ENTRY(CIN, COUT, 8, 8, 4, CIC, NG, AM)

#define BWDC_SET(CIN, COUT, CIC)                                \
  CONVC_FAMILY(CIN, COUT, CIC, 1, drsa_conv::A_DENSE),          \
  CONVC_FAMILY(CIN, COUT, CIC, 2, drsa_conv::A_DENSE),          \
  CONVC_FAMILY(CIN, COUT, CIC, 1, drsa_conv::A_POOLSPARSE),     \
  CONVC_FAMILY(CIN, COUT, CIC, 2, drsa_conv::A_POOLSPARSE)

}  // namespace drsa_conv
