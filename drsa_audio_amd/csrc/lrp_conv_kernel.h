// 3x3 'same' convolution on fp32 MFMA (v_mfma_f32_32x32x2_f32) for the LRP engine.
//
// One templated implicit-GEMM kernel serves the whole conv trunk of the VGG-type CNN
// (reference cxai/model/create_model.py:100-137) in both directions:
//
//   forward  (FWD_POOL / FWD_RELU):  z = conv(x; W) + b  ->  y = relu(z)  [-> 2x2 max-pool + argmax]
//            plus, in the same pass over the input tile, the LRP denominator of the layer's rule:
//            Gamma  (zennit 0.5.1):  den = (conv(x+; W+) + b+) + (conv(x-; W-) + b2)
//            (the plan passes b2 = 0: zennit zeroes the x- term's bias)
//            Epsilon:                               den = z
//            WSquare / Flat:                        den = precomputed input-independent map
//            den is stored only where the relevance can arrive: at the pool argmax.
//   backward (BWD): the transposed conv as a 'same' conv with flipped/transposed weights,
//            R_in = x+ (.) J^T_{W+} g  [+ x- (.) J^T_{W-} g]   (Gamma; g_- vanishes because every
//            conv is followed by ReLU), or x (.) J^T_W g (Epsilon) or J^T g (WSquare/Flat/plain),
//            with the pool-backward + ReLU-backward folded into the A-operand prologue (AMODE 1:
//            g lives at pool resolution plus an argmax byte) and the NEXT layer's division folded
//            into the epilogue (POST_DIV: g_next = [x > 0] R / stab(den_next)).
//
// GEMM view: M = output pixels of a TH x TW tile (window-major order so that every 2x2 pool
// window lands in 4 consecutive accumulator registers of one lane), N = output channels
// (32-wide MFMA tiles), K = 9 * Cin in the order k = ci*9 + (ky*3 + kx) (chunks of CIC input
// channels staged in LDS with the halo; weights [k][co] staged next to them).  Every output
// is one k-ordered fp32 fma chain (MFMA f32 semantics), independent of the chunking, which
// is what oracle/lrp_exact.c reproduces bit for bit.
#pragma once
#include "common.h"
#include "lrp_conv.h"

#include <type_traits>

#ifndef DRSA_CONV_PD_BWD
#define DRSA_CONV_PD_BWD 2
#endif
#ifndef DRSA_CONV_BWD_ES
#define DRSA_CONV_BWD_ES 1
#endif
#ifndef DRSA_CONV_BWD_WPE
#define DRSA_CONV_BWD_WPE 3
#endif
// small-chunk rule backward (SMALL_BWD: GTZAN conv_bwd:features.3 / .6): its MFMA operand ring is
// pinned (a sched_barrier per k-step keeps step k + PD's LDS reads ahead of step k's MFMAs; the
// scheduler otherwise sinks each read next to its MFMA behind an lgkmcnt(0) wait) at distance 3.
// Measured in the step (gpurun_out/r6j, r6k): features.3 1.373-1.383 -> 1.335 ms, .6 0.632 ->
// 0.613; pinning the forwards or the wider backwards as well made them 2-6 % slower.
#ifndef DRSA_CONV_PIN_SMALL
#define DRSA_CONV_PIN_SMALL 1
#endif
#ifndef DRSA_CONV_PD_SMALL
#define DRSA_CONV_PD_SMALL 3
#endif
#ifndef DRSA_CONV_SMALL_WPE
#define DRSA_CONV_SMALL_WPE 4      // small-chunk backward: 4 workgroups (16 waves) per CU
#endif
#ifndef DRSA_CONV_SMALL_ES
#define DRSA_CONV_SMALL_ES 2       // small-chunk backward: epilogue in 2 channel passes of 16
#endif
#ifndef DRSA_CONV_PRE_D
#define DRSA_CONV_PRE_D 0
#endif
#ifndef DRSA_CONV_PRE_N
#define DRSA_CONV_PRE_N 64
#endif
#ifndef DRSA_CONV_BF_WPE
#define DRSA_CONV_BF_WPE 2
#endif
#ifndef DRSA_CONV_FWD_WPE_128
#define DRSA_CONV_FWD_WPE_128 3    // 8 x 8-tile forwards into 128 channels with 4-channel chunks: 2 -> 3 waves/SIMD
#endif
#ifndef DRSA_CONV_FWD_WPE_WIDE
#define DRSA_CONV_FWD_WPE_WIDE 3   // forwards into 64 channels (CIC <= 8, NG <= 2): 1 -> 3 conv_fwd:features.6 0.361 -> 0.343 ms
#endif
#ifndef DRSA_CONV_FWD_WPE
#define DRSA_CONV_FWD_WPE 3
#endif

namespace drsa_conv {

constexpr int kThreads = 256;

// diagnostic build only (-DDRSA_CONV_STAMP, scripts/probe_conv_phases.py): phase times of every
// workgroup of the 32 -> 32 pool-sparse backward (GTZAN conv_bwd:features.3) into a buffer of their
// own, set by drsa_amd_debug_conv_stamps; nothing in the kernel reads them
#ifdef DRSA_CONV_STAMP
static __device__ unsigned long long* g_conv_stamps;
#endif

// bias3 of a forward call without bias ([3][COUT], COUT <= 128)
__device__ const float g_zero_bias3[3 * 128] = {};

template <int V, int M>
constexpr int round_up() { return (V + M - 1) / M * M; }

// halo row stride: the 32 lanes of one ds_read_b32 group read a (16/MW x 2) grid of
// MW*2-pixel runs; RS = 16 (mod 32) for 2 rows x 16, RS = 8 (mod 32) for 4 rows x 8 puts the
// runs on disjoint banks.
constexpr int halo_stride(int hx, int mw) {
  int r = hx;
  const int want = (mw == 8) ? 16 : 8;
  while (r % 32 != want) ++r;
  return r;
}

enum AMode { A_DENSE = 0, A_POOLSPARSE = 1 };
enum Epi { EPI_FWD_POOL = 0, EPI_FWD_RELU = 1, EPI_BWD = 2 };

// halo column c (pixel tx0 - 1 + c) lives at LDS column c + XO, so the tile interior starts
// 16-byte aligned (float4 staging stores) and pool cells cover aligned float2 pairs.
constexpr int XO = 3;

// bf16 halo row stride in 16-byte pixels: >= hx and 8 (mod 16), so the two rows of a 2x2-window
// run of 16 lanes land on disjoint bank halves (ds_read_b128)
constexpr int bf_stride(int hx) {
  int r = hx;
  while (r % 16 != 8) ++r;
  return r;
}

// ET (element type of the MFMA operands): 0 = fp32 (v_mfma_f32_32x32x2_f32, the exact k-ordered
// chain), 1 = bf16 (v_mfma_f32_32x32x16_bf16, forward only: conv inputs and weights rounded to
// bf16 when staged, fp32 accumulation, fp32 outputs).  The bf16 chunk is 16 input channels = one
// tap per MFMA (k = tap * 16 + ci); its halo is pixel-major, 8 channels per 16-byte pixel slot.
template <int CIN, int COUT, int TH, int TW, int MW, int CIC, int NG, int AMODE, int EPI, int ET = 0, int PW = 2>
struct ConvCfg {
  static constexpr int CIN_ = CIN, COUT_ = COUT, TH_ = TH, TW_ = TW, MW_ = MW, CIC_ = CIC, NG_ = NG;
  static constexpr int AMODE_ = AMODE, EPI_ = EPI;
  static constexpr bool BF = ET == 1;
  static constexpr int HY = TH + 2, HX = TW + 2;
  static constexpr int HXB = bf_stride(HX);
  // bf16 staging: halo [2 channel halves][HY][HXB] x 16 B, weights [NG][9 taps][2][COUT] x 16 B
  static constexpr size_t bf_halo_floats = (size_t)2 * HY * HXB * 4;
  static constexpr size_t bf_w_floats = (size_t)NG * 9 * 2 * COUT * 4;
  static constexpr int RS = halo_stride(HX + XO, MW);
  static constexpr int PLANE_RAW = HY * RS;
  static constexpr int PLANE = PLANE_RAW + ((PLANE_RAW % 32) == 0 ? 4 : 0);
  // M-tile = the 32 pixels of one MFMA B operand: window-major 2x2 pool windows (MTH = 16/MW rows
  // x 2*MW)
  static constexpr int MTW = 2 * MW;
  static constexpr int MTH = 32 / MTW;
  static constexpr int MTX = TW / MTW;     // M-tiles per tile row
  static constexpr int MT = (TH / MTH) * MTX;
  static constexpr int NT = COUT / 32;
  static constexpr int WM = MT >= 4 ? 4 : MT;
  static constexpr int WN = (4 / WM) < NT ? (4 / WM) : NT;   // waves >= WM*WN idle (tiny layers)
  static constexpr int MPW = MT / WM;      // m-tiles per wave
  static constexpr int NPW = NT / WN;      // n-tiles per wave
  static constexpr int KC = 9 * CIC;
  static constexpr int KCP = round_up<KC, 2>();
  static constexpr int NCHUNK = CIN / CIC;
  static constexpr int TWP = (TW == 32) ? 48 : TW;          // epilogue tile row stride (conflict-free writes)
  // backward epilogue in ES channel passes (halves the epilogue LDS and registers; WN == 1 only)
  // small-chunk rule backward (CIC <= 8, 32 output channels): 24.6 KB LDS and <= 128 VGPRs, so
  // 4 workgroups (16 waves) per CU
  static constexpr bool SMALL_BWD = EPI == EPI_BWD && NG == 1 && CIC <= 8 && COUT <= 32;
  static constexpr int ES = (EPI == EPI_BWD && WN == 1) ? (SMALL_BWD ? DRSA_CONV_SMALL_ES : DRSA_CONV_BWD_ES) : 1;
  static constexpr int TCH = WN * 32 / ES;                     // channels staged per epilogue pass
  static constexpr size_t staging_floats =
      BF ? bf_halo_floats + bf_w_floats : (size_t)CIC * PLANE + (size_t)NG * KCP * COUT;
  static constexpr size_t epi_floats = (size_t)TCH * TH * TWP;
  static constexpr size_t lds_floats = staging_floats > epi_floats ? staging_floats : epi_floats;
  // minimum waves per SIMD the register allocation must allow (1 block = 1 wave per SIMD)
  static constexpr int WPE = BF ? (COUT <= 64 ? DRSA_CONV_BF_WPE : 1)
                             : (EPI == EPI_BWD && NG == 1) ? (SMALL_BWD ? DRSA_CONV_SMALL_WPE : DRSA_CONV_BWD_WPE)
                             : (EPI != EPI_BWD && CIC <= 8 && COUT <= 32 && NG <= 2 ? DRSA_CONV_FWD_WPE
                                : EPI != EPI_BWD && CIC <= 8 && NG <= 2 && COUT == 64 ? DRSA_CONV_FWD_WPE_WIDE
                                : EPI != EPI_BWD && CIC <= 4 && NG <= 2 && COUT == 128 && TW == 8 ? DRSA_CONV_FWD_WPE_128 : 1);
  // operand prefetch distance of the MFMA loop (k-steps)
  static constexpr bool PIN = SMALL_BWD && DRSA_CONV_PIN_SMALL;
  static constexpr int PD = PIN ? DRSA_CONV_PD_SMALL : DRSA_CONV_PD_BWD > 0 && EPI >= EPI_BWD ? DRSA_CONV_PD_BWD : 1;
  static_assert(TH % MTH == 0 && TW % MTW == 0, "tile must be a multiple of the M-tile");
  static_assert(COUT % 32 == 0, "COUT must be padded to 32");
  static_assert(CIN % CIC == 0, "CIN must be a multiple of the chunk");
  static_assert(MT % WM == 0 && NT % WN == 0 && WM * WN <= 4, "wave split");
  static_assert(!BF || (CIC == 16 && (EPI < EPI_BWD ? AMODE == A_DENSE : EPI == EPI_BWD)),
                "bf16: 16-channel chunks; dense forward, or the per-clone backward (dense or pool-sparse g)");
  static_assert(PW == 2 || (PW == 4 && (EPI == EPI_FWD_POOL || (EPI == EPI_BWD && AMODE == A_POOLSPARSE &&
                                                                  (ET == 1 || TW % 16 == 0)))),
                "2x4 pool windows: the forward pool epilogue, or the backward's pool-sparse staging (fp32: "
                "tiles of whole float4 cell groups)");
  static constexpr int PW_ = PW;
};

// ---- staging of one input-channel chunk: registers <- global (load), LDS <- registers
//      (store), split so that the loads of the next chunk can be issued before the MFMA loop
//      of the current one.  NT_ threads take part (tid in [0, NT_)). ----
template <class Cfg, int NT_ = kThreads>
struct Stager {
  static constexpr int CIN = Cfg::CIN_, COUT = Cfg::COUT_, TH = Cfg::TH_, TW = Cfg::TW_, CIC = Cfg::CIC_;
  static constexpr int NG = Cfg::NG_, HY = Cfg::HY, HX = Cfg::HX, RS = Cfg::RS, PLANE = Cfg::PLANE;
  static constexpr int KC = Cfg::KC, KCP = Cfg::KCP;
  static constexpr bool DENSE = Cfg::AMODE_ == A_DENSE;
  // dense halo: interior rows of TW/4 float4 + the two halo columns
  static constexpr int Q4 = TW / 4, DROWS = CIC * HY;
  static constexpr int DI = (DROWS * Q4 + NT_ - 1) / NT_, DH = (DROWS * 2 + NT_ - 1) / NT_;
  // pool-sparse cells: interior rows of TW/8 float4 (4 cells) + the two halo cell columns
  static constexpr int CY = TH / 2 + 2, CX = TW / 2 + 2, Q8 = TW / 8 > 0 ? TW / 8 : 1, SROWS = CIC * CY;
  static constexpr int SI = (SROWS * Q8 + NT_ - 1) / NT_, SH = (SROWS * 2 + NT_ - 1) / NT_;
  // P4: 2 x 4 cells (VGGish's (2,4) pool folded into the staging): interior rows of TW/16 float4
  // (4 cells = 16 pixels each) + the two halo cells, which reach 1 pixel into the halo each
  static constexpr bool P4 = !DENSE && Cfg::PW_ == 4;
  static constexpr int Q16 = TW / 16 > 0 ? TW / 16 : 1;
  static constexpr int SI4 = (SROWS * Q16 + NT_ - 1) / NT_;
  static constexpr int NI = DENSE ? DI : P4 ? SI4 : SI, NH = DENSE ? DH : SH;
  static constexpr int NWV = NG * KCP * (COUT / 4), WIT = (NWV + NT_ - 1) / NT_;
  float4 st_i[NI];
  uint32_t st_ia[DENSE ? 1 : NI];
  float st_h[NH];
  int st_ha[DENSE ? 1 : NH];
  float4 st_w[WIT];

  // Loads are unconditional from a clamped (always valid) address and masked afterwards, so
  // the compiler issues them back to back without exec branches or per-load waits.
  __device__ __forceinline__ void load(const ConvArgs& a, int c0, int tid, int ty0, int tx0, int bq, int bs) {
    const int H = a.H, W = a.W, H2 = H >> 1, W2 = W >> 1;
    // per-sample bases (uniform) + 32-bit per-lane offsets: saddr + voffset loads instead of a
    // 64-bit multiply-add per element (the host keeps one sample's cin x H x W below 2^31)
    const int W4 = W >> 2;
    const float* __restrict__ inb = a.in + (size_t)bq * a.cin * (DENSE ? H * W : H2 * (P4 ? W4 : W2));
    const uint8_t* __restrict__ amb = DENSE ? nullptr : a.in_amax + (size_t)bs * a.cin * H2 * (P4 ? W4 : W2);
    if constexpr (P4) {
      // host contract: W / 4 % 4 == 0, so every 4-cell group is one aligned float4 / uint32
      const int qy0 = (ty0 >> 1) - 1, cx0 = tx0 >> 2;
#pragma unroll
      for (int it = 0; it < SI4; ++it) {
        const int i = tid + it * NT_;
        const int row = i / Q16, q = i % Q16;
        const int ci = row / CY, ry = row % CY;
        const int cy = qy0 + ry, cx = cx0 + 4 * q, c = c0 + ci;
        const bool ok = i < SROWS * Q16 && cy >= 0 && cy < H2 && c < a.cin && cx < W4;
        const int o = ok ? (c * H2 + cy) * W4 + cx : 0;
        const float4 v = *reinterpret_cast<const float4*>(inb + o);
        const uint32_t am = *reinterpret_cast<const uint32_t*>(amb + o);
        st_i[it] = ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
        st_ia[it] = ok ? am : 0xffffffffu;   // 0xff names no pixel of a 2 x 4 window
      }
#pragma unroll
      for (int it = 0; it < SH; ++it) {
        const int i = tid + it * NT_;
        const int row = i >> 1, side = i & 1;
        const int ci = row / CY, ry = row % CY;
        const int cy = qy0 + ry, cx = side ? cx0 + TW / 4 : cx0 - 1, c = c0 + ci;
        const bool ok = i < SROWS * 2 && cy >= 0 && cy < H2 && cx >= 0 && cx < W4 && c < a.cin;
        const int o = ok ? (c * H2 + cy) * W4 + cx : 0;
        const float v = inb[o];
        const int am = (int)amb[o];
        st_h[it] = ok ? v : 0.f;
        st_ha[it] = ok ? am : 0xff;
      }
    } else if constexpr (DENSE) {
      if ((W & 3) == 0) {
#pragma unroll
        for (int it = 0; it < DI; ++it) {
          const int i = tid + it * NT_;
          const int row = i / Q4, q = i % Q4;
          const int ci = row / HY, hy = row % HY;
          const int gy = ty0 - 1 + hy, gx = tx0 + 4 * q, c = c0 + ci;
          const bool ok = i < DROWS * Q4 && gy >= 0 && gy < H && c < a.cin && gx < W;
          const int o = ok ? (c * H + gy) * W + gx : 0;
          const float4 v = *reinterpret_cast<const float4*>(inb + o);
          st_i[it] = ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      } else {
#pragma unroll
        for (int it = 0; it < DI; ++it) {
          const int i = tid + it * NT_;
          const int row = i / Q4, q = i % Q4;
          const int ci = row / HY, hy = row % HY;
          const int gy = ty0 - 1 + hy, gx = tx0 + 4 * q, c = c0 + ci;
          const bool rok = i < DROWS * Q4 && gy >= 0 && gy < H && c < a.cin;
          float vv[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const bool ok = rok && gx + e < W;
            const int o = ok ? (c * H + gy) * W + gx + e : 0;
            const float v = inb[o];
            vv[e] = ok ? v : 0.f;
          }
          st_i[it] = make_float4(vv[0], vv[1], vv[2], vv[3]);
        }
      }
#pragma unroll
      for (int it = 0; it < DH; ++it) {
        const int i = tid + it * NT_;
        const int row = i >> 1, side = i & 1;
        const int ci = row / HY, hy = row % HY;
        const int gy = ty0 - 1 + hy, gx = side ? tx0 + TW : tx0 - 1, c = c0 + ci;
        const bool ok = i < DROWS * 2 && gy >= 0 && gy < H && gx >= 0 && gx < W && c < a.cin;
        const int o = ok ? (c * H + gy) * W + gx : 0;
        const float v = inb[o];
        st_h[it] = ok ? v : 0.f;
      }
    } else {
      const int qy0 = (ty0 >> 1) - 1, qx0 = (tx0 >> 1) - 1;
      if ((W2 & 3) == 0) {
#pragma unroll
        for (int it = 0; it < SI; ++it) {
          const int i = tid + it * NT_;
          const int row = i / Q8, q = i % Q8;
          const int ci = row / CY, ry = row % CY;
          const int cy = qy0 + ry, cx = qx0 + 1 + 4 * q, c = c0 + ci;
          const bool ok = i < SROWS * Q8 && 4 * q < TW / 2 && cy >= 0 && cy < H2 && c < a.cin && cx < W2;
          const int o = ok ? (c * H2 + cy) * W2 + cx : 0;
          const float4 v = *reinterpret_cast<const float4*>(inb + o);
          const uint32_t am = *reinterpret_cast<const uint32_t*>(amb + o);
          st_i[it] = ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
          st_ia[it] = ok ? am : 0x04040404u;
        }
      } else {
#pragma unroll
        for (int it = 0; it < SI; ++it) {
          const int i = tid + it * NT_;
          const int row = i / Q8, q = i % Q8;
          const int ci = row / CY, ry = row % CY;
          const int cy = qy0 + ry, cx = qx0 + 1 + 4 * q, c = c0 + ci;
          const bool rok = i < SROWS * Q8 && 4 * q < TW / 2 && cy >= 0 && cy < H2 && c < a.cin;
          float vv[4];
          uint32_t aa = 0;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const bool ok = rok && cx + e < W2 && 4 * q + e < TW / 2;
            const int o = ok ? (c * H2 + cy) * W2 + cx + e : 0;
            const float v = inb[o];
            const uint32_t am = amb[o];
            vv[e] = ok ? v : 0.f;
            aa |= (ok ? am : 4u) << (8 * e);
          }
          st_i[it] = make_float4(vv[0], vv[1], vv[2], vv[3]);
          st_ia[it] = aa;
        }
      }
#pragma unroll
      for (int it = 0; it < SH; ++it) {
        const int i = tid + it * NT_;
        const int row = i >> 1, side = i & 1;
        const int ci = row / CY, ry = row % CY;
        const int cy = qy0 + ry, cx = side ? qx0 + CX - 1 : qx0, c = c0 + ci;
        const bool ok = i < SROWS * 2 && cy >= 0 && cy < H2 && cx >= 0 && cx < W2 && c < a.cin;
        const int o = ok ? (c * H2 + cy) * W2 + cx : 0;
        const float v = inb[o];
        const int am = (int)amb[o];
        st_h[it] = ok ? v : 0.f;
        st_ha[it] = ok ? am : 4;
      }
    }
    // weights: rows [c0*9, c0*9 + KC) of every set, contiguous (k = ci*9 + tap)
#pragma unroll
    for (int it = 0; it < WIT; ++it) {
      const int idx = tid + it * NT_;
      const int g = idx / (KCP * (COUT / 4)), rem = idx % (KCP * (COUT / 4));
      const int k = rem / (COUT / 4), c4 = (rem % (COUT / 4)) * 4;
      const bool ok = idx < NWV && k < KC;
      const float4 v = *reinterpret_cast<const float4*>(a.wts + (ok ? ((size_t)g * 9 * CIN + c0 * 9 + k) * COUT + c4 : 0));
      st_w[it] = ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }

  // one pool cell -> its 2x2 pixels at halo rows 2ry-1, 2ry and LDS columns 2rx-1+XO, 2rx+XO
  __device__ __forceinline__ static void put_cell(float* halo, int ci, int ry, int rx, float v, int sb) {
    float* d = halo + ci * PLANE + (2 * ry - 1) * RS + 2 * rx - 1 + XO;
    if (ry > 0) *reinterpret_cast<float2*>(d) = make_float2(sb == 0 ? v : 0.f, sb == 1 ? v : 0.f);
    if (ry < CY - 1) *reinterpret_cast<float2*>(d + RS) = make_float2(sb == 2 ? v : 0.f, sb == 3 ? v : 0.f);
  }

  // one 2 x 4 cell -> its 8 pixels: halo rows 2ry-1, 2ry, LDS columns 4rx .. 4rx+3 (halo columns
  // 4rx-3 .. 4rx; rx = 0 and TW/4 + 1 are the halo cells, whose other columns are row padding)
  __device__ __forceinline__ static void put_cell4(float* halo, int ci, int ry, int rx, float v, int sb) {
    float* d = halo + ci * PLANE + (2 * ry - 1) * RS + 4 * rx;
    if (ry > 0)
      *reinterpret_cast<float4*>(d) = make_float4(sb == 0 ? v : 0.f, sb == 1 ? v : 0.f, sb == 2 ? v : 0.f, sb == 3 ? v : 0.f);
    if (ry < CY - 1)
      *reinterpret_cast<float4*>(d + RS) =
          make_float4(sb == 4 ? v : 0.f, sb == 5 ? v : 0.f, sb == 6 ? v : 0.f, sb == 7 ? v : 0.f);
  }

  __device__ __forceinline__ void store(float* halo, float* wl, int tid) const {
    if constexpr (P4) {
      static_assert(XO == 3, "P4 cells land on 16-byte aligned columns 4 rx");
#pragma unroll
      for (int it = 0; it < SI4; ++it) {
        const int i = tid + it * NT_;
        if (i < SROWS * Q16) {
          const int row = i / Q16, q = i % Q16;
          const int ci = row / CY, ry = row % CY;
          const float vv[4] = {st_i[it].x, st_i[it].y, st_i[it].z, st_i[it].w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            put_cell4(halo, ci, ry, 1 + 4 * q + e, vv[e], (int)((st_ia[it] >> (8 * e)) & 0xffu));
        }
      }
#pragma unroll
      for (int it = 0; it < SH; ++it) {
        const int i = tid + it * NT_;
        if (i < SROWS * 2) {
          const int row = i >> 1, side = i & 1;
          put_cell4(halo, row / CY, row % CY, side ? TW / 4 + 1 : 0, st_h[it], st_ha[it]);
        }
      }
    } else if constexpr (DENSE) {
#pragma unroll
      for (int it = 0; it < DI; ++it) {
        const int i = tid + it * NT_;
        if (i < DROWS * Q4) {
          const int row = i / Q4, q = i % Q4;
          const int ci = row / HY, hy = row % HY;
          *reinterpret_cast<float4*>(halo + ci * PLANE + hy * RS + 1 + XO + 4 * q) = st_i[it];
        }
      }
#pragma unroll
      for (int it = 0; it < DH; ++it) {
        const int i = tid + it * NT_;
        if (i < DROWS * 2) {
          const int row = i >> 1, side = i & 1;
          const int ci = row / HY, hy = row % HY;
          halo[ci * PLANE + hy * RS + (side ? HX - 1 : 0) + XO] = st_h[it];
        }
      }
    } else {
#pragma unroll
      for (int it = 0; it < SI; ++it) {
        const int i = tid + it * NT_;
        const int q = i % Q8;
        if (i < SROWS * Q8 && 4 * q < TW / 2) {
          const int row = i / Q8;
          const int ci = row / CY, ry = row % CY;
          const float vv[4] = {st_i[it].x, st_i[it].y, st_i[it].z, st_i[it].w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (4 * q + e < TW / 2) put_cell(halo, ci, ry, 1 + 4 * q + e, vv[e], (int)((st_ia[it] >> (8 * e)) & 0xffu));
        }
      }
#pragma unroll
      for (int it = 0; it < SH; ++it) {
        const int i = tid + it * NT_;
        if (i < SROWS * 2) {
          const int row = i >> 1, side = i & 1;
          put_cell(halo, row / CY, row % CY, side ? CX - 1 : 0, st_h[it], st_ha[it]);
        }
      }
    }
#pragma unroll
    for (int it = 0; it < WIT; ++it) {
      const int idx = tid + it * NT_;
      if (idx < NWV) *reinterpret_cast<float4*>(wl + (size_t)idx * 4) = st_w[it];
    }
  }
};

// ---- MFMA over one staged chunk.  k = k0 + h (h = lane half) with k = ci*9 + tap: the halo
//      offset pattern repeats every 9 k-steps (two channels), so every LDS read in the fully
//      unrolled loop is a per-lane base register + immediate.  Operands of step k0 are read
//      one step ahead (explicit software pipeline). ----
template <class Cfg, int PD = 1>
__device__ __forceinline__ void mfma_chunk(const float* halo, const float* wl, const int (&pix_off)[Cfg::MPW],
                                           int lane, int wn, f32x16 (&acc)[Cfg::NG_][Cfg::MPW][Cfg::NPW]) {
  constexpr int MPW = Cfg::MPW, NPW = Cfg::NPW, NG = Cfg::NG_, COUT = Cfg::COUT_;
  constexpr int KC = Cfg::KC, KCP = Cfg::KCP, PLANE = Cfg::PLANE, RS = Cfg::RS, EPI = Cfg::EPI_;
  const int h = lane >> 5;
  // Halo offset of k = k0 + h (k = ci * 9 + tap):  off(k0) + h * delta(k0 % 9), with off(k0) a
  // compile-time immediate (the loop is unrolled) and delta one of three values: +1 inside a tap
  // row, RS - 2 from the row's last tap to the next row, PLANE - 2 RS - 2 from tap 8 to the next
  // channel's tap 0.  So each m-tile needs three per-lane base registers (pix_off + h * delta)
  // instead of one per k-step pattern, and every operand read is base + immediate.
  constexpr int DLT[3] = {1, RS - 2, PLANE - 2 * RS - 2};
  int xb[MPW][3];
#pragma unroll
  for (int u = 0; u < MPW; ++u)
#pragma unroll
    for (int t = 0; t < 3; ++t) xb[u][t] = pix_off[u] + h * DLT[t];
  auto read_x = [&](int k0, float (&xv)[MPW]) {
    const int r9 = k0 % 9;
    const int off = (k0 / 9) * PLANE + (r9 / 3) * RS + (r9 % 3);
    const int t = (r9 == 8) ? 2 : (r9 == 2 || r9 == 5) ? 1 : 0;
#pragma unroll
    for (int u = 0; u < MPW; ++u) {
      if constexpr (KC % 2 == 0) xv[u] = halo[xb[u][t] + off];
      else xv[u] = (k0 + h < KC) ? halo[xb[u][t] + off] : 0.f;
    }
  };
  auto read_w = [&](int k0, float (&wv)[NG][NPW]) {
#pragma unroll
    for (int v = 0; v < NPW; ++v)
#pragma unroll
      for (int g = 0; g < NG; ++g) wv[g][v] = wl[((size_t)g * KCP + k0 + h) * COUT + (wn * NPW + v) * 32 + (lane & 31)];
  };
  // operand ring: step k0's operands are read PD steps ahead
  float xr[PD + 1][MPW], wr[PD + 1][NG][NPW];
#pragma unroll
  for (int d = 0; d < PD; ++d)
    if (2 * d < KCP) {
      read_x(2 * d, xr[d]);
      read_w(2 * d, wr[d]);
    }
#pragma unroll
  for (int k0 = 0; k0 < KCP; k0 += 2) {
    const int cur = (k0 / 2) % (PD + 1), nxt = (k0 / 2 + PD) % (PD + 1);
    if (k0 + 2 * PD < KCP) {
      read_x(k0 + 2 * PD, xr[nxt]);
      read_w(k0 + 2 * PD, wr[nxt]);
    }
    if constexpr (Cfg::PIN) __builtin_amdgcn_sched_barrier(0);   // keep the ring (see DRSA_CONV_PIN_SMALL)
#pragma unroll
    for (int v = 0; v < NPW; ++v)
#pragma unroll
      for (int g = 0; g < NG; ++g)
#pragma unroll
        for (int u = 0; u < MPW; ++u) {
          float x = xr[cur][u];
          // NG == 2 is the Gamma forward on a non-negative input (ABI contract): x+ = x, so both
          // sets read the same operand with no per-k-step transform
          if constexpr (EPI < EPI_BWD && NG == 3) {
            x = (g == 0) ? x : (g == 1 ? fmaxf(x, 0.f) : fminf(x, 0.f));
          }
          acc[g][u][v] = mfma32(wr[cur][g][v], x, acc[g][u][v]);
        }
  }
}
// ---- bf16 staging (ET = 1) of one 16-channel chunk.  Item (half, hy, hx) = the 8 channels
//      c0 + 8 half .. +7 of halo pixel (hy, hx): 8 coalesced fp32 loads (consecutive lanes on
//      consecutive pixels), rounded and packed at store time into one 16-byte LDS slot.  Weights
//      come pre-laid-out and pre-rounded ([NG][CIN/16][9][2][COUT][8] bf16): a straight copy. ----
template <class Cfg, int NT_ = kThreads>
struct StagerBF {
  static constexpr int CIN = Cfg::CIN_, COUT = Cfg::COUT_, NG = Cfg::NG_, HY = Cfg::HY, HX = Cfg::HX;
  static constexpr int HXB = Cfg::HXB, NCH = CIN / 16;
  static constexpr int NITEM = 2 * HY * HX, IT = (NITEM + NT_ - 1) / NT_;
  static constexpr int NWQ = NG * 18 * COUT, WIT = (NWQ + NT_ - 1) / NT_;
  // (2,4) pool-sparse staging: one item per (channel half, halo row, pool cell): the cell's 8
  // channel values and argmax bytes are loaded once and expanded to its 4 pixels at store time
  // (the generic per-pixel item would load each cell 4 times)
  static constexpr bool P4 = Cfg::AMODE_ == A_POOLSPARSE && Cfg::PW_ == 4;
  static constexpr int NCR = Cfg::TW_ / 4 + 2;                 // cells per halo row (2 partial)
  static constexpr int NITEM4 = 2 * HY * NCR, IT4 = (NITEM4 + NT_ - 1) / NT_;
  static constexpr int ITX = P4 ? IT4 : IT;
  float st_f[ITX][8];
  uint32_t st_a[P4 ? IT4 : 1][2];
  uint4 st_w[WIT];

  __device__ __forceinline__ void load(const ConvArgs& a, int c0, int tid, int ty0, int tx0, int bq, int bs) {
    const int H = a.H, W = a.W;
    const unsigned HW = (unsigned)(H * W);
    // per-sample bases (uniform) + 32-bit per-lane offsets (saddr + voffset loads)
    const int H2s = H >> 1, W2s = W / (P4 ? 4 : Cfg::PW_);
    const float* __restrict__ inb =
        a.in + (size_t)bq * a.cin * (Cfg::AMODE_ == A_POOLSPARSE || P4 ? (size_t)H2s * W2s : (size_t)HW);
    const uint8_t* __restrict__ amb = (Cfg::AMODE_ == A_POOLSPARSE || P4) ? a.in_amax + (size_t)bs * a.cin * H2s * W2s
                                                                          : nullptr;
    if constexpr (P4) {
      const int H2 = H >> 1, W2 = W >> 2;
      const unsigned HW2 = (unsigned)(H2 * W2);
#pragma unroll
      for (int it = 0; it < IT4; ++it) {
        const int i = tid + it * NT_;
        const int cs = i % NCR, r = i / NCR, hy = r % HY, half = r / HY;
        const int gy = ty0 - 1 + hy, cx = (tx0 >> 2) - 1 + cs, cb = c0 + 8 * half;
        const bool ok = i < NITEM4 && gy >= 0 && gy < H && cx >= 0 && cx < W2;
        const unsigned cell = ok ? (unsigned)((gy >> 1) * W2 + cx) : 0u;
        const unsigned base = ok ? (unsigned)cb * HW2 + cell : 0u;
        uint32_t ab[2] = {0u, 0u};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const bool okc = ok && cb + j < a.cin;
          const float v = inb[okc ? base + j * HW2 : 0u];
          const uint32_t am = amb[okc ? base + j * HW2 : 0u];
          st_f[it][j] = okc ? v : 0.f;
          ab[j >> 2] |= (okc ? am : 0xffu) << (8 * (j & 3));   // 0xff matches no pixel
        }
        st_a[it][0] = ab[0];
        st_a[it][1] = ab[1];
      }
    } else if constexpr (Cfg::AMODE_ == A_POOLSPARSE) {
      // backward input at 2 x PW pool resolution + argmax byte (the pool backward; PW = 4: the
      // VGGish (2,4) pool, create_model.py:61): halo pixel (gy, gx) holds g[cell] where the cell's
      // argmax (row-major window position) is this pixel, else 0
      constexpr int PWB = Cfg::PW_;
      const int H2 = H >> 1, W2 = W / PWB;
      const unsigned HW2 = (unsigned)(H2 * W2);
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int i = tid + it * NT_;
        const int hx = i % HX, r = i / HX, hy = r % HY, half = r / HY;
        const int gy = ty0 - 1 + hy, gx = tx0 - 1 + hx, cb = c0 + 8 * half;
        const bool ok = i < NITEM && gy >= 0 && gy < H && gx >= 0 && gx < W;
        const unsigned cell = ok ? (unsigned)((gy >> 1) * W2 + (gx / PWB)) : 0u;
        const unsigned base = ok ? (unsigned)cb * HW2 + cell : 0u;
        const uint32_t sub = (uint32_t)((gy & 1) * PWB + (gx % PWB));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const bool okc = ok && cb + j < a.cin;
          const float v = inb[okc ? base + j * HW2 : 0u];
          const uint32_t am = amb[okc ? base + j * HW2 : 0u];
          st_f[it][j] = (okc && am == sub) ? v : 0.f;
        }
      }
    } else {
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int i = tid + it * NT_;
        const int hx = i % HX, r = i / HX, hy = r % HY, half = r / HY;
        const int gy = ty0 - 1 + hy, gx = tx0 - 1 + hx, cb = c0 + 8 * half;
        const bool ok = i < NITEM && gy >= 0 && gy < H && gx >= 0 && gx < W;
        const unsigned base = ok ? (unsigned)cb * HW + (unsigned)(gy * W + gx) : 0u;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const bool okc = ok && cb + j < a.cin;
          const float v = inb[okc ? base + j * HW : 0u];
          st_f[it][j] = okc ? v : 0.f;
        }
      }
    }
    const uint4* wq = reinterpret_cast<const uint4*>(a.wts);
    const int chunk = c0 / 16;
#pragma unroll
    for (int it = 0; it < WIT; ++it) {
      const int idx = tid + it * NT_;
      const bool ok = idx < NWQ;
      const int g = idx / (18 * COUT), rem = idx % (18 * COUT);
      st_w[it] = wq[ok ? ((size_t)g * NCH + chunk) * 18 * COUT + rem : 0];
    }
  }

  __device__ __forceinline__ void store(float* halo, float* wl, int tid, int ty0 = 0, int tx0 = 0) const {
    uint4* hb = reinterpret_cast<uint4*>(halo);
    if constexpr (P4) {
#pragma unroll
      for (int it = 0; it < IT4; ++it) {
        const int i = tid + it * NT_;
        if (i < NITEM4) {
          const int cs = i % NCR, r = i / NCR, hy = r % HY;
          const uint32_t rowsub = (uint32_t)(((ty0 - 1 + hy) & 1) * 4);
          // cell cs covers halo columns 4 cs - 3 .. 4 cs (halo column hx = pixel tx0 - 1 + hx)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int hx = 4 * cs - 3 + e;
            if (hx >= 0 && hx < HX) {
              float v8[8];
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const uint32_t am = (st_a[it][j >> 2] >> (8 * (j & 3))) & 0xffu;
                v8[j] = am == rowsub + (uint32_t)e ? st_f[it][j] : 0.f;
              }
              uint4 q;
              q.x = pack_bf16x2(v8[0], v8[1]);
              q.y = pack_bf16x2(v8[2], v8[3]);
              q.z = pack_bf16x2(v8[4], v8[5]);
              q.w = pack_bf16x2(v8[6], v8[7]);
              hb[r * HXB + hx] = q;
            }
          }
        }
      }
    } else {
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int i = tid + it * NT_;
      if (i < NITEM) {
        const int hx = i % HX, r = i / HX;
        uint4 q;
        q.x = pack_bf16x2(st_f[it][0], st_f[it][1]);
        q.y = pack_bf16x2(st_f[it][2], st_f[it][3]);
        q.z = pack_bf16x2(st_f[it][4], st_f[it][5]);
        q.w = pack_bf16x2(st_f[it][6], st_f[it][7]);
        hb[r * HXB + hx] = q;   // r = half * HY + hy
      }
    }
    }
    uint4* wb = reinterpret_cast<uint4*>(wl);
#pragma unroll
    for (int it = 0; it < WIT; ++it) {
      const int idx = tid + it * NT_;
      if (idx < NWQ) wb[idx] = st_w[it];
    }
  }
};

// x+ / x- of 8 packed bf16 (sign bit per 16-bit half): Gamma's NG = 3 forward on a signed input
__device__ __forceinline__ uint32_t bf2_neg_mask(uint32_t w) { return ((w >> 15) & 0x00010001u) * 0xffffu; }

// ---- bf16 MFMA over one staged 16-channel chunk: one v_mfma_f32_32x32x16_bf16 per tap and
//      (set, m-tile, n-tile); lane l reads its 8 channels (half l>>5) of pixel l&31 (B) and of
//      output channel l&31 (A) as one ds_read_b128 each, one tap ahead. ----
template <class Cfg>
__device__ __forceinline__ void mfma_chunk_bf(const uint4* hb, const uint4* wb, const int (&pix_off)[Cfg::MPW],
                                              int lane, int wn, f32x16 (&acc)[Cfg::NG_][Cfg::MPW][Cfg::NPW]) {
  constexpr int MPW = Cfg::MPW, NPW = Cfg::NPW, NG = Cfg::NG_, COUT = Cfg::COUT_, HXB = Cfg::HXB;
  const uint4* wlane = wb + (lane >> 5) * COUT + wn * NPW * 32 + (lane & 31);
  uint4 xr[2][MPW], wr[2][NG][NPW];
  auto rd = [&](int t, uint4 (&x)[MPW], uint4 (&w)[NG][NPW]) {
    const int toff = (t / 3) * HXB + t % 3;
#pragma unroll
    for (int u = 0; u < MPW; ++u) x[u] = hb[pix_off[u] + toff];
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int v = 0; v < NPW; ++v) w[g][v] = wlane[(g * 9 + t) * 2 * COUT + v * 32];
  };
  rd(0, xr[0], wr[0]);
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int cur = t & 1;
    if (t + 1 < 9) rd(t + 1, xr[cur ^ 1], wr[cur ^ 1]);
#pragma unroll
    for (int v = 0; v < NPW; ++v)
#pragma unroll
      for (int g = 0; g < NG; ++g)
#pragma unroll
        for (int u = 0; u < MPW; ++u) {
          uint4 b = xr[cur][u];
          if constexpr (NG == 3) {
            if (g > 0) {
              const uint4 m = make_uint4(bf2_neg_mask(b.x), bf2_neg_mask(b.y), bf2_neg_mask(b.z), bf2_neg_mask(b.w));
              b = (g == 1) ? make_uint4(b.x & ~m.x, b.y & ~m.y, b.z & ~m.z, b.w & ~m.w)
                           : make_uint4(b.x & m.x, b.y & m.y, b.z & m.z, b.w & m.w);
            }
          }
          acc[g][u][v] = mfma32_bf16(__builtin_bit_cast(u16x8, wr[cur][g][v]), __builtin_bit_cast(u16x8, b),
                                     acc[g][u][v]);
        }
  }
}

// PW: pool window width of EPI_FWD_POOL (2 x PW windows; 4 = VGGish's (2,4) pool)
template <int CIN, int COUT, int TH, int TW, int MW, int CIC, int NG, int AMODE, int EPI, int ET = 0, int PW = 2>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(ConvCfg<CIN, COUT, TH, TW, MW, CIC, NG, AMODE, EPI, ET, PW>::WPE))) void conv3x3_kernel(ConvArgs a) {
  using Cfg = ConvCfg<CIN, COUT, TH, TW, MW, CIC, NG, AMODE, EPI, ET, PW>;
  constexpr int HY = Cfg::HY, HX = Cfg::HX, RS = Cfg::RS, PLANE = Cfg::PLANE;
  constexpr int MTH = Cfg::MTH, MTW = Cfg::MTW, MTX = Cfg::MTX;
  constexpr int WM = Cfg::WM, MPW = Cfg::MPW, NPW = Cfg::NPW;
  constexpr int KC = Cfg::KC, KCP = Cfg::KCP;

  extern __shared__ __attribute__((aligned(16))) float smem[];
#ifdef DRSA_CONV_STAMP
  constexpr bool kStamp = EPI == EPI_BWD && CIN == 32 && COUT == 32 && AMODE == A_POOLSPARSE && ET == 0;
  unsigned long long* const stp = kStamp && g_conv_stamps && threadIdx.x == 0
                                      ? g_conv_stamps + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 16 : nullptr;
#define CONV_STAMP(slot) do { if (stp) stp[(slot)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define CONV_STAMP(slot) do {} while (0)
#endif
  CONV_STAMP(0);
  float* halo = smem;                          // [CIC][PLANE]   (bf16: [2][HY][HXB] x 16 B)
  float* wl = smem + (Cfg::BF ? Cfg::bf_halo_floats : (size_t)CIC * PLANE);   // [NG][KCP][COUT]

  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  const int H = a.H, W = a.W;
  const int tiles_x = (W + TW - 1) / TW;
  const int tile_id = blockIdx.x, bq = blockIdx.y;  // bq: batch index (incl. clones)
  const int ty0 = (tile_id / tiles_x) * TH;
  const int tx0 = (tile_id % tiles_x) * TW;
  const int bs = bq / a.clones;               // sample index (shared forward state)
  const int wm = w % WM, wn = w / WM;
  const bool active = w < WM * Cfg::WN;
  const int h = lane >> 5;

  // MFMA orientation: D[channel][pixel] = W^T[channel][k] * X[k][pixel]
  //   A operand (lane l): W[k = k0 + (l>>5)][co = n0 + (l&31)]
  //   B operand (lane l): X[k = k0 + (l>>5)][pixel p = l&31 of the m-tile]
  //   D: lane l holds pixel p = l&31, registers r hold channels n0 + (r&3) + 8(r>>2) + 4(l>>5)
  // pixel p of an m-tile -> pool window win = p>>2, sub = p&3 (window-major order)
  int pix_off[MPW], pix_y[MPW], pix_x[MPW];
#pragma unroll
  for (int u = 0; u < MPW; ++u) {
    const int mt = wm * MPW + u;
    const int p = lane & 31, win = p >> 2, sub = p & 3;
    pix_y[u] = (mt / MTX) * MTH + 2 * (win / MW) + (sub >> 1);
    pix_x[u] = (mt % MTX) * MTW + 2 * (win % MW) + (sub & 1);
    pix_off[u] = Cfg::BF ? (h * HY + pix_y[u]) * Cfg::HXB + pix_x[u] : pix_y[u] * RS + pix_x[u] + XO;
  }

  f32x16 acc[NG][MPW][NPW];
#pragma unroll
  for (int g = 0; g < NG; ++g)
#pragma unroll
    for (int u = 0; u < MPW; ++u)
#pragma unroll
      for (int v = 0; v < NPW; ++v)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[g][u][v][r] = 0.f;

  // ---- epilogue, staged through LDS so global I/O is coalesced float4 rows ----
  // pass (v, kind): every active wave writes its 32-channel slice (n-tile wn*NPW + v) of its
  // m-tiles into T[TCH][TH][TWP] (lane = pixel, register = channel: conflict-free rows),
  // then all threads walk T in row order.
  constexpr int TWP = Cfg::TWP, TCH = Cfg::TCH;
  constexpr int NV4 = TCH * TH * TW / 4;                 // float4 groups per pass
  constexpr int V4T = (NV4 + kThreads - 1) / kThreads;   // per thread
  constexpr int NCELL = TCH * (TH / 2) * (TW / 2);
  constexpr int CT = (NCELL + kThreads - 1) / kThreads;
  float* T = smem;
  constexpr int ES = Cfg::ES;
  static_assert(ES == 1 || ES == 2 || ES == 4, "epilogue split must be 1, 2 or 4");
  // pass `sub` of ES stages the registers whose channel lies in [sub*TCH, (sub+1)*TCH)
  // (channel = (r&3) + 8(r>>2) + 4h: ES = 2 takes r >> 3 == sub, ES = 4 r >> 2 == sub)
  auto stage = [&](int v, auto valfn, int sub = 0) {
    __syncthreads();
    if (active) {
#pragma unroll
      for (int u = 0; u < MPW; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int cf = (r & 3) + 8 * (r >> 2) + 4 * h;
          if constexpr (ES == 1) {
            T[((wn * 32 + cf) * TH + pix_y[u]) * TWP + pix_x[u]] = valfn(u, r);
          } else {
            if ((r >> (ES == 2 ? 3 : 2)) == sub) T[((cf - TCH * sub) * TH + pix_y[u]) * TWP + pix_x[u]] = valfn(u, r);
          }
        }
    }
    __syncthreads();
  };
  auto gch = [&](int cl, int v) { return ((cl >> 5) * NPW + v) * 32 + (cl & 31); };   // global channel
  // global channel of staged row cl in pass sub (ES = 2 implies WN = 1)
  auto gchs = [&](int cl, int v, int sub) { return ES == 1 ? gch(cl, v) : v * 32 + sub * TCH + cl; };
  typename std::conditional<Cfg::BF, StagerBF<Cfg>, Stager<Cfg>>::type stg;
  stg.load(a, 0, tid, ty0, tx0, bq, bs);
  CONV_STAMP(11);
  // backward: all chunks but the last here, the last one peeled below (after the epilogue
  // addressing is set up, so that none of it is live across the loop)
  for (int chunk = 0; chunk + (EPI == EPI_BWD ? 1 : 0) < Cfg::NCHUNK; ++chunk) {
    __syncthreads();
    if (chunk == 0) CONV_STAMP(9);
    if constexpr (Cfg::BF) stg.store(halo, wl, tid, ty0, tx0);
    else stg.store(halo, wl, tid);
    if (chunk == 0) CONV_STAMP(10);
    __syncthreads();
    CONV_STAMP(1 + 2 * chunk);
    if (chunk + 1 < Cfg::NCHUNK) stg.load(a, (chunk + 1) * CIC, tid, ty0, tx0, bq, bs);
    if (!active) continue;
    if constexpr (Cfg::BF)
      mfma_chunk_bf<Cfg>(reinterpret_cast<const uint4*>(halo), reinterpret_cast<const uint4*>(wl), pix_off, lane, wn, acc);
    else
      mfma_chunk<Cfg, Cfg::PD>(halo, wl, pix_off, lane, wn, acc);
    CONV_STAMP(2 + 2 * chunk);
  }
  constexpr int Q = TH * TW / 4, CS = kThreads / Q;
  static_assert(kThreads % Q == 0, "float4 groups per tile must divide the block");
  const int cl0 = tid / Q, rem = tid % Q;
  const int py = rem / (TW / 4), px = (rem % (TW / 4)) * 4;
  const bool pix_ok = ty0 + py < H && tx0 + px < W;
  const int HW = H * W;
  const size_t pix = pix_ok ? (size_t)(ty0 + py) * W + tx0 + px : 0;
  const float* xs = a.x ? a.x + (size_t)bs * a.cout * HW + pix : nullptr;
  // den_shared: the next layer's denominator is an input-independent map [cout][H][W] (WSquare /
  // Flat without a pool between): every sample reads the same plane (L2-resident), nothing per sample
  const float* ds = a.den ? a.den + (a.den_shared ? (size_t)0 : (size_t)bs * a.cout * HW) + pix : nullptr;
  float* oqp = a.out + (size_t)bq * a.cout * HW + pix;
  // x and den come from clamped, always valid addresses (den falls back to x or out when the
  // mode does not use it) and are ALL issued before any arithmetic; the rule / post modes are
  // uniform selects, not branches (a branch around the division would put each den load in
  // its own basic block, one full memory round trip after another)
  const bool need_x = a.xmode != XM_NONE || a.post != POST_NONE;
  const bool mul_x = a.xmode != XM_NONE, split_x = a.xmode == XM_SPLIT;
  // POST_DIV_RING: float4 groups off the image's border ring read the map's per-channel value
  // (den_const4, one 16-byte line per channel: an L1 broadcast) instead of the per-sample copy,
  // which the forward writes on the ring only; the pointer is a per-lane select, no branch
  const bool ring = a.post == POST_DIV_RING && a.den_const4;
  const bool post_div = a.post == POST_DIV || ring, post_any = a.post != POST_NONE;
  const float* xsrc = xs ? xs : oqp;
  const float* dsrc = (ds && post_div && !ring) ? ds : xsrc;
  const float eps = a.eps;
  const bool on_ring = !pix_ok || ty0 + py == 0 || ty0 + py == H - 1 || tx0 + px == 0 || tx0 + px + 4 >= W;
  const bool use_c4 = ring && !on_ring;
  // the compact ring of plane (sample, channel): [row 0 | row H-1 | rows 1..H-2 x (4 + 4 columns)]
  const int ring_n = 2 * W + 8 * (H - 2);
  const int Y = ty0 + py, X = tx0 + px;
  const int ring_i = !pix_ok ? 0 : Y == 0 ? X : Y == H - 1 ? W + X : 2 * W + (Y - 1) * 8 + (X == 0 ? 0 : 4);
  const float* rsrc = ring ? a.den + (size_t)bs * a.cout * ring_n + ring_i : dsrc;
  const size_t dstride = ring ? (size_t)ring_n : (size_t)HW;
  // x loads and R stores as a uniform per-sample base + a 32-bit per-lane offset (saddr + voffset
  // addressing; the host keeps one sample's cout x H x W below 2^31)
  const unsigned upix = (unsigned)pix;
  float* const obase = a.out + (size_t)bq * a.cout * HW;
  const float* const xbase = a.x ? a.x + (size_t)bs * a.cout * HW : obase;
  // epilogue x/den loads of (n-tile v, pass sub); (0, 0) is issued before the last chunk's MFMAs
  auto epi_loads = [&](int v, int sub, float4 (&xk)[V4T], float4 (&dk)[V4T], bool lx = true, bool ld = true,
                       int i0 = 0, int i1 = -1) {
    if (i1 < 0) i1 = V4T;
#pragma unroll
    for (int it = i0; it < i1; ++it) {
      const int cl = cl0 + it * CS;
      const int co = gchs(cl, v, sub);
      const bool ok = cl < TCH && co < a.cout;
      const int coc = ok ? co : 0;
      if (lx) xk[it] = *reinterpret_cast<const float4*>(xbase + (upix + (unsigned)coc * (unsigned)HW));
      if (ld) dk[it] = *reinterpret_cast<const float4*>(use_c4 ? a.den_const4 + (size_t)coc * 4 : rsrc + coc * dstride);
    }
  };
  // x groups prefetched before the last chunk's MFMAs (all of them spill a few registers)
  constexpr int kPreN = DRSA_CONV_PRE_N < V4T ? DRSA_CONV_PRE_N : V4T;
  float4 pre_x[V4T], pre_d[V4T];
  if constexpr (EPI == EPI_BWD) {
    // last chunk, peeled: the staging registers are free, so the epilogue's first x loads go
    // out here and their latency hides under the MFMAs (den too would spill: measured slower)
    __syncthreads();
    if constexpr (Cfg::BF) stg.store(halo, wl, tid, ty0, tx0);
    else stg.store(halo, wl, tid);
    __syncthreads();
    CONV_STAMP(2 * Cfg::NCHUNK - 1);
    epi_loads(0, 0, pre_x, pre_d, true, DRSA_CONV_PRE_D, 0, kPreN);

    if (active) {
      if constexpr (Cfg::BF)
        mfma_chunk_bf<Cfg>(reinterpret_cast<const uint4*>(halo), reinterpret_cast<const uint4*>(wl), pix_off, lane, wn,
                           acc);
      else
        mfma_chunk<Cfg, Cfg::PD>(halo, wl, pix_off, lane, wn, acc);
    }
    CONV_STAMP(2 * Cfg::NCHUNK);
  }

  // the pool cells of the staged tile T (2 x PWc windows), one per thread and iteration `it`
  // (it < CT; CT is sized for 2x2 cells, the most)
  auto pool_cells = [&](auto pwc, auto&& fn) {
    constexpr int PWc = decltype(pwc)::value;
    constexpr int CW = TW / PWc, NC = TCH * (TH / 2) * CW;
    const int H2 = H >> 1, W2 = W / PWc;
#pragma unroll
    for (int it = 0; it < CT; ++it) {
      const int i = tid + it * kThreads;
      if (i < NC) {
        const int cl = i / ((TH / 2) * CW), rem = i % ((TH / 2) * CW);
        const int cy = rem / CW, cx = rem % CW;
        fn(it, cl, cy, cx, (ty0 >> 1) + cy, tx0 / PWc + cx, H2, W2);
      }
    }
  };
#pragma unroll
  for (int v = 0; v < NPW; ++v) {
    if constexpr (EPI == EPI_FWD_POOL || EPI == EPI_FWD_RELU) {
      // the lane's 16 channels' biases, loaded unconditionally (bias3 is [3][COUT]; a missing bias
      // reads a zero table) and all issued before any use: a branch around each load had put
      // every one of them in its own basic block behind its own wait
      const float* bb = a.bias ? a.bias : g_zero_bias3;
      float b0[16], b1[16], b2[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = gch(wn * 32 + (r & 3) + 8 * (r >> 2) + 4 * h, v);
        const bool cok = co < a.cout;
        const float x0 = bb[co], x1 = bb[COUT + co], x2 = bb[2 * COUT + co];
        b0[r] = cok ? x0 : 0.f;
        b1[r] = cok ? x1 : 0.f;
        b2[r] = cok ? x2 : 0.f;
      }
      // pass 0: y = relu(z)
      stage(v, [&](int u, int r) {
        const float z = acc[0][u][v][r] + b0[r];
        float y = z > 0.f ? z : 0.f;
        if (z != z) y = z;   // relu(NaN) = NaN (torch semantics)
        return y;
      });
      int am_keep[CT];
      if constexpr (EPI == EPI_FWD_POOL) {
        // 2 x PWc pool windows (PWc = PW: 2, or 4 for VGGish's (2,4) pool): first maximum
        // in row-major window order, NaN wins (torch max_pool2d); argmax byte = row * PWc + col
        auto pass0 = [&](auto pwc) {
          constexpr int PWc = decltype(pwc)::value;
          pool_cells(pwc, [&](int it, int cl, int cy, int cx, int qy, int qx, int H2, int W2) {
            const int co = gch(cl, v);
            const float* t = T + (cl * TH + 2 * cy) * TWP + PWc * cx;
            int am = 0;
            float m = t[0];
#pragma unroll
            for (int s4 = 1; s4 < 2 * PWc; ++s4) {
              const float yv = t[(s4 / PWc) * TWP + s4 % PWc];
              if (yv > m || (yv != yv && m == m)) { m = yv; am = s4; }
            }
            am_keep[it] = am;
            if (co < a.cout && qy < H2 && qx < W2) {
              const size_t o = (size_t)bq * a.cout * H2 * W2 + (unsigned)((co * H2 + qy) * W2 + qx);
              a.out[o] = m;
              a.out_amax[o] = (uint8_t)am;
            }
          });
        };
        if constexpr (PW == 4) {
#pragma unroll
          for (int it = 0; it < CT; ++it) am_keep[it] = 0;
          pass0(std::integral_constant<int, 4>{});
        } else {
          // 2x2 (the GTZAN trunk): the original straight-line form (the generic lambda form costs
          // the fp32 forward kernels ~2-10 %: one more spilled register)
          const int H2 = H >> 1, W2 = W >> 1;
#pragma unroll
          for (int it = 0; it < CT; ++it) {
            const int i = tid + it * kThreads;
            am_keep[it] = 0;
            if (i < NCELL) {
              const int cl = i / ((TH / 2) * (TW / 2)), rem = i % ((TH / 2) * (TW / 2));
              const int cy = rem / (TW / 2), cx = rem % (TW / 2);
              const int co = gch(cl, v);
              const int qy = (ty0 >> 1) + cy, qx = (tx0 >> 1) + cx;
              const float* t = T + (cl * TH + 2 * cy) * TWP + 2 * cx;
              const float yy[4] = {t[0], t[1], t[TWP], t[TWP + 1]};
              int am = 0;
              float m = yy[0];
#pragma unroll
              for (int s4 = 1; s4 < 4; ++s4)
                if (yy[s4] > m || (yy[s4] != yy[s4] && m == m)) { m = yy[s4]; am = s4; }
              am_keep[it] = am;
              if (co < a.cout && qy < H2 && qx < W2) {
                const size_t o = (size_t)bq * a.cout * H2 * W2 + (unsigned)((co * H2 + qy) * W2 + qx);
                a.out[o] = m;
                a.out_amax[o] = (uint8_t)am;
              }
            }
          }
        }
      } else {
#pragma unroll
        for (int it = 0; it < V4T; ++it) {
          const int i = tid + it * kThreads;
          if (i < NV4) {
            const int cl = i / (TH * TW / 4), rem = i % (TH * TW / 4);
            const int py = rem / (TW / 4), px = (rem % (TW / 4)) * 4;
            const int co = gch(cl, v);
            if (co < a.cout && ty0 + py < H && tx0 + px < W) {
              const float4 val = *reinterpret_cast<const float4*>(T + (cl * TH + py) * TWP + px);
              *reinterpret_cast<float4*>(a.out + (size_t)bq * a.cout * H * W + (unsigned)((co * H + ty0 + py) * W + tx0 + px)) = val;
            }
          }
        }
      }
      if (a.out_den && a.den_map) {
        // WSquare / Flat: input-independent map, read directly (coalesced) where it is stored
        if constexpr (EPI == EPI_FWD_POOL) {
          auto gather_map = [&](auto pwc) {
            constexpr int PWc = decltype(pwc)::value;
            pool_cells(pwc, [&](int it, int cl, int, int, int qy, int qx, int H2, int W2) {
              const int co = gch(cl, v);
              const int am = am_keep[it];
              if (co < a.cout && qy < H2 && qx < W2)
                a.out_den[(size_t)bq * a.cout * H2 * W2 + (unsigned)((co * H2 + qy) * W2 + qx)] =
                    a.den_map[(unsigned)((co * H + 2 * qy + am / PWc) * W + PWc * qx + am % PWc)];
            });
          };
          if constexpr (PW == 4) {
            gather_map(std::integral_constant<int, 4>{});
          } else {
            const int H2 = H >> 1, W2 = W >> 1;
#pragma unroll
            for (int it = 0; it < CT; ++it) {
              const int i = tid + it * kThreads;
              if (i < NCELL) {
                const int cl = i / ((TH / 2) * (TW / 2)), rem = i % ((TH / 2) * (TW / 2));
                const int cy = rem / (TW / 2), cx = rem % (TW / 2);
                const int co = gch(cl, v);
                const int qy = (ty0 >> 1) + cy, qx = (tx0 >> 1) + cx;
                const int am = am_keep[it];
                if (co < a.cout && qy < H2 && qx < W2)
                  a.out_den[(size_t)bq * a.cout * H2 * W2 + (unsigned)((co * H2 + qy) * W2 + qx)] =
                      a.den_map[(unsigned)((co * H + 2 * qy + (am >> 1)) * W + 2 * qx + (am & 1))];
              }
            }
          }
        } else {
#pragma unroll
          for (int it = 0; it < V4T; ++it) {
            const int i = tid + it * kThreads;
            if (i < NV4) {
              const int cl = i / (TH * TW / 4), rem = i % (TH * TW / 4);
              const int py = rem / (TW / 4), px = (rem % (TW / 4)) * 4;
              const int co = gch(cl, v);
              if (co < a.cout && ty0 + py < H && tx0 + px < W)
                *reinterpret_cast<float4*>(a.out_den + (size_t)bq * a.cout * H * W + (unsigned)((co * H + ty0 + py) * W + tx0 + px)) =
                    *reinterpret_cast<const float4*>(a.den_map + (unsigned)((co * H + ty0 + py) * W + tx0 + px));
            }
          }
        }
      } else if (a.out_den) {
        // pass 1: the rule's denominator
        stage(v, [&](int u, int r) {
          if constexpr (NG >= 2) {
            const float z0 = acc[1][u][v][r] + b1[r];
            float z1 = b2[r];
            if constexpr (NG == 3) z1 = acc[2][u][v][r] + b2[r];
            return z0 + z1;
          }
          // Epsilon: den = conv(x; W) + b_den (b_den = b, or 0 under zero_params=['bias'])
          return acc[0][u][v][r] + b1[r];
        });
        if constexpr (EPI == EPI_FWD_POOL) {
          auto gather_den = [&](auto pwc) {
            constexpr int PWc = decltype(pwc)::value;
            pool_cells(pwc, [&](int it, int cl, int cy, int cx, int qy, int qx, int H2, int W2) {
              const int co = gch(cl, v);
              const int am = am_keep[it];
              if (co < a.cout && qy < H2 && qx < W2)
                a.out_den[(size_t)bq * a.cout * H2 * W2 + (unsigned)((co * H2 + qy) * W2 + qx)] =
                    T[(cl * TH + 2 * cy + am / PWc) * TWP + PWc * cx + am % PWc];
            });
          };
          if constexpr (PW == 4) {
            gather_den(std::integral_constant<int, 4>{});
          } else {
            const int H2 = H >> 1, W2 = W >> 1;
#pragma unroll
            for (int it = 0; it < CT; ++it) {
              const int i = tid + it * kThreads;
              if (i < NCELL) {
                const int cl = i / ((TH / 2) * (TW / 2)), rem = i % ((TH / 2) * (TW / 2));
                const int cy = rem / (TW / 2), cx = rem % (TW / 2);
                const int co = gch(cl, v);
                const int qy = (ty0 >> 1) + cy, qx = (tx0 >> 1) + cx;
                const int am = am_keep[it];
                if (co < a.cout && qy < H2 && qx < W2)
                  a.out_den[(size_t)bq * a.cout * H2 * W2 + (unsigned)((co * H2 + qy) * W2 + qx)] =
                      T[(cl * TH + 2 * cy + (am >> 1)) * TWP + 2 * cx + (am & 1)];
              }
            }
          }
        } else {
#pragma unroll
          for (int it = 0; it < V4T; ++it) {
            const int i = tid + it * kThreads;
            if (i < NV4) {
              const int cl = i / (TH * TW / 4), rem = i % (TH * TW / 4);
              const int py = rem / (TW / 4), px = (rem % (TW / 4)) * 4;
              const int co = gch(cl, v);
              if (co < a.cout && ty0 + py < H && tx0 + px < W) {
                const float4 val = *reinterpret_cast<const float4*>(T + (cl * TH + py) * TWP + px);
                *reinterpret_cast<float4*>(a.out_den + (size_t)bq * a.cout * H * W + (unsigned)((co * H + ty0 + py) * W + tx0 + px)) = val;
              }
            }
          }
        }
      }
    } else {   // EPI_BWD: R = xmode(acc, x) -> post -> out
      // float4 group i = tid + it * 256: the pixel (py, px) is fixed per thread and the staged
      // row advances by CS = 256 / Q per iteration, so every address is a per-thread base plus
      // a channel offset.  Loads come from clamped (always valid) addresses and the arithmetic
      // runs unconditionally (no exec branches that would serialise the load latency); only the
      // store is masked.  x is loaded once for the rule and the division.
#pragma unroll
     for (int sub = 0; sub < ES; ++sub) {
      float4 Rk[V4T], xk[V4T], dk[V4T];
      if (v == 0 && sub == 0) {
#pragma unroll
        for (int it = 0; it < kPreN; ++it) xk[it] = pre_x[it];
        epi_loads(v, sub, xk, dk, true, false, kPreN, V4T);
        if (DRSA_CONV_PRE_D) {
#pragma unroll
          for (int it = 0; it < V4T; ++it) dk[it] = pre_d[it];
        } else {
          epi_loads(v, sub, xk, dk, false, true);
        }
      } else {
        epi_loads(v, sub, xk, dk);
      }
      stage(v, [&](int u, int r) { return acc[0][u][v][r]; }, sub);
      // the common mode (Epsilon-type rule: R = x * J^T g, then the next layer's division)
      // specialised: the loads above are already in flight, this branch is uniform
      if (NG == 1 && a.xmode == XM_MUL && post_div) {
#pragma unroll
        for (int it = 0; it < V4T; ++it) {
          const int cl = cl0 + it * CS;
          const int co = gchs(cl, v, sub);
          const bool ok = cl < TCH && co < a.cout;
          const int clc = ok ? cl : 0, coc = ok ? co : 0;
          const float4 t = *reinterpret_cast<const float4*>(T + (clc * TH + py) * TWP + px);
          const float4 x = xk[it], d = dk[it];
          auto f = [&](float tt, float xx, float dd) {
            const float q = div_nb(xx * tt, stab(dd, eps));
            return (xx > 0.f) ? q : 0.f;
          };
          const float4 R = make_float4(f(t.x, x.x, d.x), f(t.y, x.y, d.y), f(t.z, x.z, d.z), f(t.w, x.w, d.w));
          if (ok && pix_ok) *reinterpret_cast<float4*>(obase + (upix + (unsigned)coc * (unsigned)HW)) = R;
        }
        continue;
      }
#pragma unroll
      for (int it = 0; it < V4T; ++it) {
        const int cl = cl0 + it * CS;
        const int co = gchs(cl, v, sub);
        const int clc = (cl < TCH && co < a.cout) ? cl : 0;
        const float4 t = *reinterpret_cast<const float4*>(T + (clc * TH + py) * TWP + px);
        if (!need_x) xk[it] = make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 x = xk[it];
        // XM_NONE: 1 * t = t;  XM_MUL: x * t;  XM_SPLIT: max(x, 0) * t
        auto xm = [&](float xx) { const float m = split_x ? fmaxf(xx, 0.f) : xx; return mul_x ? m : 1.f; };
        Rk[it] = make_float4(xm(x.x) * t.x, xm(x.y) * t.y, xm(x.z) * t.z, xm(x.w) * t.w);
      }
      if constexpr (NG >= 2) {
        if (split_x) {
          stage(v, [&](int u, int r) { return acc[1][u][v][r]; }, sub);
#pragma unroll
          for (int it = 0; it < V4T; ++it) {
            const int cl = cl0 + it * CS;
            const int co = gchs(cl, v, sub);
            const int clc = (cl < TCH && co < a.cout) ? cl : 0;
            const float4 t = *reinterpret_cast<const float4*>(T + (clc * TH + py) * TWP + px);
            const float4 x = xk[it];
            Rk[it].x += fminf(x.x, 0.f) * t.x;
            Rk[it].y += fminf(x.y, 0.f) * t.y;
            Rk[it].z += fminf(x.z, 0.f) * t.z;
            Rk[it].w += fminf(x.w, 0.f) * t.w;
          }
        }
      }
#pragma unroll
      for (int it = 0; it < V4T; ++it) {
        const int cl = cl0 + it * CS;
        const int co = gchs(cl, v, sub);
        const bool ok = cl < TCH && co < a.cout;
        const int coc = ok ? co : 0;
        float4 R = Rk[it];
        // POST_DIV: x > 0 ? R / stab(den) : 0;  POST_MASK: x > 0 ? R : 0 (quotients evaluated for
        // every lane and mode, then selected)
        const float4 x = xk[it], d = dk[it];
        auto post = [&](float rr, float xx, float dd) {
          const float q = div_nb(rr, stab(dd, eps));
          const float y = post_div ? q : rr;
          return (post_any && !(xx > 0.f)) ? 0.f : y;
        };
        R = make_float4(post(R.x, x.x, d.x), post(R.y, x.y, d.y), post(R.z, x.z, d.z), post(R.w, x.w, d.w));
        if (ok && pix_ok) *reinterpret_cast<float4*>(obase + (upix + (unsigned)coc * (unsigned)HW)) = R;
      }
     }
    }
  }
#ifdef DRSA_CONV_STAMP
  if (stp) {
    stp[13] = __builtin_amdgcn_s_memtime();
    stp[14] = (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_ID
    stp[15] = (unsigned long long)__builtin_amdgcn_s_getreg(20 | (31 << 11));   // XCC_ID
  }
#endif
#undef CONV_STAMP
}

typedef void (*KernFn)(ConvArgs);

struct Entry {
  int cin_p, cout_p, th, tw, mw, cic, ng, amode, epi;
  KernFn fn;
  size_t lds;
  int et = 0;   // operand type (ConvCfg ET)
  int pw = 2;   // pool window width (ConvCfg PW)
};

#define CONV_ENTRY(CIN, COUT, TH, TW, MW, CIC, NG, AM, EP)                                                 \
  drsa_conv::Entry{CIN, COUT, TH, TW, MW, CIC, NG, AM, EP,                                                 \
                   drsa_conv::conv3x3_kernel<CIN, COUT, TH, TW, MW, CIC, NG, AM, EP>,                      \
                   drsa_conv::ConvCfg<CIN, COUT, TH, TW, MW, CIC, NG, AM, EP>::lds_floats * sizeof(float)}

// fp32 per-clone backward with g at (2,4)-pool resolution (VGGish block 1, create_model.py:61)
#define CONV_ENTRY_P4B(CIN, COUT, TH, TW, MW, CIC)                                                          \
  drsa_conv::Entry{CIN, COUT, TH, TW, MW, CIC, 1, drsa_conv::A_POOLSPARSE, drsa_conv::EPI_BWD,              \
                   drsa_conv::conv3x3_kernel<CIN, COUT, TH, TW, MW, CIC, 1, drsa_conv::A_POOLSPARSE, drsa_conv::EPI_BWD, 0, 4>, \
                   drsa_conv::ConvCfg<CIN, COUT, TH, TW, MW, CIC, 1, drsa_conv::A_POOLSPARSE, drsa_conv::EPI_BWD, 0, 4>::lds_floats * sizeof(float), 0, 4}

#define CONV_ENTRY_BFA(CIN, COUT, TH, TW, MW, NG, AM, EP)                                                 \
  drsa_conv::Entry{CIN, COUT, TH, TW, MW, 16, NG, AM, EP,                                                 \
                   drsa_conv::conv3x3_kernel<CIN, COUT, TH, TW, MW, 16, NG, AM, EP, 1>,                   \
                   drsa_conv::ConvCfg<CIN, COUT, TH, TW, MW, 16, NG, AM, EP, 1>::lds_floats * sizeof(float), 1}
// bf16-operand per-clone backward (ET = 1), dense and pool-sparse g, one weight set
#define BWD_SET_BF(CIN, COUT)                                                                    \
  CONV_ENTRY_BFA(CIN, COUT, 8, 32, 8, 1, drsa_conv::A_DENSE, drsa_conv::EPI_BWD),                \
  CONV_ENTRY_BFA(CIN, COUT, 8, 16, 8, 1, drsa_conv::A_DENSE, drsa_conv::EPI_BWD),                \
  CONV_ENTRY_BFA(CIN, COUT, 8, 8, 4, 1, drsa_conv::A_DENSE, drsa_conv::EPI_BWD),                 \
  CONV_ENTRY_BFA(CIN, COUT, 8, 32, 8, 1, drsa_conv::A_POOLSPARSE, drsa_conv::EPI_BWD),           \
  CONV_ENTRY_BFA(CIN, COUT, 8, 16, 8, 1, drsa_conv::A_POOLSPARSE, drsa_conv::EPI_BWD),           \
  CONV_ENTRY_BFA(CIN, COUT, 8, 8, 4, 1, drsa_conv::A_POOLSPARSE, drsa_conv::EPI_BWD)

// bf16-operand per-clone backward with g at (2,4)-pool resolution (VGGish block 1)
#define CONV_ENTRY_BFA_P4(CIN, COUT, TH, TW, MW)                                                           \
  drsa_conv::Entry{CIN, COUT, TH, TW, MW, 16, 1, drsa_conv::A_POOLSPARSE, drsa_conv::EPI_BWD,              \
                   drsa_conv::conv3x3_kernel<CIN, COUT, TH, TW, MW, 16, 1, drsa_conv::A_POOLSPARSE, drsa_conv::EPI_BWD, 1, 4>, \
                   drsa_conv::ConvCfg<CIN, COUT, TH, TW, MW, 16, 1, drsa_conv::A_POOLSPARSE, drsa_conv::EPI_BWD, 1, 4>::lds_floats * sizeof(float), 1, 4}
#define BWD_SET_BF_P4(CIN, COUT)                       \
  CONV_ENTRY_BFA_P4(CIN, COUT, 8, 32, 8),              \
  CONV_ENTRY_BFA_P4(CIN, COUT, 8, 16, 8),              \
  CONV_ENTRY_BFA_P4(CIN, COUT, 8, 8, 4)

#define CONV_ENTRY_BF(CIN, COUT, TH, TW, MW, NG, EP)                                                     \
  drsa_conv::Entry{CIN, COUT, TH, TW, MW, 16, NG, drsa_conv::A_DENSE, EP,                                 \
                   drsa_conv::conv3x3_kernel<CIN, COUT, TH, TW, MW, 16, NG, drsa_conv::A_DENSE, EP, 1>,   \
                   drsa_conv::ConvCfg<CIN, COUT, TH, TW, MW, 16, NG, drsa_conv::A_DENSE, EP, 1>::lds_floats * sizeof(float), 1}

// 2x4-pool forward (VGGish block 1, create_model.py:61): fp32 and bf16 operands
#define CONV_ENTRY_P4(CIN, COUT, TH, TW, MW, CIC, NG, ET)                                                  \
  drsa_conv::Entry{CIN, COUT, TH, TW, MW, CIC, NG, drsa_conv::A_DENSE, drsa_conv::EPI_FWD_POOL,           \
                   drsa_conv::conv3x3_kernel<CIN, COUT, TH, TW, MW, CIC, NG, drsa_conv::A_DENSE, drsa_conv::EPI_FWD_POOL, ET, 4>, \
                   drsa_conv::ConvCfg<CIN, COUT, TH, TW, MW, CIC, NG, drsa_conv::A_DENSE, drsa_conv::EPI_FWD_POOL, ET, 4>::lds_floats * sizeof(float), ET, 4}
#define CONV_FAMILY_P4(CIN, COUT, CIC, NG, ET)                    \
  CONV_ENTRY_P4(CIN, COUT, 8, 32, 8, CIC, NG, ET),                 \
  CONV_ENTRY_P4(CIN, COUT, 8, 16, 8, CIC, NG, ET),                 \
  CONV_ENTRY_P4(CIN, COUT, 8, 8, 4, CIC, NG, ET)
#define FWD_SET_P4(CIN, COUT, CIC, ET)                                                  \
  CONV_FAMILY_P4(CIN, COUT, CIC, 1, ET), CONV_FAMILY_P4(CIN, COUT, CIC, 2, ET), CONV_FAMILY_P4(CIN, COUT, CIC, 3, ET)

// tile families (the choice: lrp_conv.hip find): 8x32 / 8x16 (MW 8), 8x8 (MW 4)
#define CONV_FAMILY(CIN, COUT, CIC, NG, AM, EP)                      \
  CONV_ENTRY(CIN, COUT, 8, 32, 8, CIC, NG, AM, EP),                  \
  CONV_ENTRY(CIN, COUT, 8, 16, 8, CIC, NG, AM, EP),                  \
  CONV_ENTRY(CIN, COUT, 8, 8, 4, CIC, NG, AM, EP)

#define FWD_SET(CIN, COUT, CIC)                                                        \
  CONV_FAMILY(CIN, COUT, CIC, 1, drsa_conv::A_DENSE, drsa_conv::EPI_FWD_POOL),          \
  CONV_FAMILY(CIN, COUT, CIC, 2, drsa_conv::A_DENSE, drsa_conv::EPI_FWD_POOL),          \
  CONV_FAMILY(CIN, COUT, CIC, 3, drsa_conv::A_DENSE, drsa_conv::EPI_FWD_POOL),          \
  CONV_FAMILY(CIN, COUT, CIC, 1, drsa_conv::A_DENSE, drsa_conv::EPI_FWD_RELU),          \
  CONV_FAMILY(CIN, COUT, CIC, 2, drsa_conv::A_DENSE, drsa_conv::EPI_FWD_RELU),          \
  CONV_FAMILY(CIN, COUT, CIC, 3, drsa_conv::A_DENSE, drsa_conv::EPI_FWD_RELU)

#define BWD_SET(CIN, COUT, CIC)                                                        \
  CONV_FAMILY(CIN, COUT, CIC, 1, drsa_conv::A_DENSE, drsa_conv::EPI_BWD),               \
  CONV_FAMILY(CIN, COUT, CIC, 2, drsa_conv::A_DENSE, drsa_conv::EPI_BWD),               \
  CONV_FAMILY(CIN, COUT, CIC, 1, drsa_conv::A_POOLSPARSE, drsa_conv::EPI_BWD),          \
  CONV_FAMILY(CIN, COUT, CIC, 2, drsa_conv::A_POOLSPARSE, drsa_conv::EPI_BWD)

#define CONV_FAMILY_BF(CIN, COUT, NG, EP)                      \
  CONV_ENTRY_BF(CIN, COUT, 8, 32, 8, NG, EP),                  \
  CONV_ENTRY_BF(CIN, COUT, 8, 16, 8, NG, EP),                  \
  CONV_ENTRY_BF(CIN, COUT, 8, 8, 4, NG, EP)

// bf16-operand forward (ET = 1), every denominator set count and both epilogues
#define FWD_SET_BF(CIN, COUT)                                                 \
  CONV_FAMILY_BF(CIN, COUT, 1, drsa_conv::EPI_FWD_POOL),                      \
  CONV_FAMILY_BF(CIN, COUT, 2, drsa_conv::EPI_FWD_POOL),                      \
  CONV_FAMILY_BF(CIN, COUT, 3, drsa_conv::EPI_FWD_POOL),                      \
  CONV_FAMILY_BF(CIN, COUT, 1, drsa_conv::EPI_FWD_RELU),                      \
  CONV_FAMILY_BF(CIN, COUT, 2, drsa_conv::EPI_FWD_RELU),                      \
  CONV_FAMILY_BF(CIN, COUT, 3, drsa_conv::EPI_FWD_RELU)

struct Table {
  const Entry* entries;
  int n;
};


}  // namespace drsa_conv
