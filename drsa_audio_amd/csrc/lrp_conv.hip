// 3x3 'same' convolution on fp32 MFMA (v_mfma_f32_32x32x2_f32) for the LRP engine.
//
// One templated implicit-GEMM kernel serves the whole conv trunk of the VGG-type CNN
// (reference cxai/model/create_model.py:100-137) in both directions:
//
//   forward  (FWD_POOL / FWD_RELU):  z = conv(x; W) + b  ->  y = relu(z)  [-> 2x2 max-pool + argmax]
//            plus, in the same pass over the input tile, the LRP denominator of the layer's rule:
//            Gamma  (zennit 0.5.1):  den = (conv(x+; W+) + b+) + (conv(x-; W-) + b-)
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
#include "common.h"
#include "lrp_conv.h"

namespace {

constexpr int kThreads = 256;

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

template <int CIN, int COUT, int TH, int TW, int MW, int CIC, int NG, int AMODE, int EPI>
struct ConvCfg {
  static constexpr int HY = TH + 2, HX = TW + 2;
  static constexpr int RS = halo_stride(HX, MW);
  static constexpr int PLANE_RAW = HY * RS;
  static constexpr int PLANE = PLANE_RAW + ((PLANE_RAW % 32) == 0 ? 4 : 0);
  static constexpr int MTH = 16 / MW;      // M-tile height (pixels)
  static constexpr int MTW = 2 * MW;       // M-tile width (pixels)
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
  static constexpr size_t lds_floats = (size_t)CIC * PLANE + (size_t)NG * KCP * COUT;
  static_assert(TH % MTH == 0 && TW % MTW == 0, "tile must be a multiple of the M-tile");
  static_assert(COUT % 32 == 0, "COUT must be padded to 32");
  static_assert(CIN % CIC == 0, "CIN must be a multiple of the chunk");
  static_assert(MT % WM == 0 && NT % WN == 0 && WM * WN <= 4, "wave split");
};

template <int CIN, int COUT, int TH, int TW, int MW, int CIC, int NG, int AMODE, int EPI>
__global__ __launch_bounds__(kThreads) void conv3x3_kernel(ConvArgs a) {
  using Cfg = ConvCfg<CIN, COUT, TH, TW, MW, CIC, NG, AMODE, EPI>;
  constexpr int HY = Cfg::HY, HX = Cfg::HX, RS = Cfg::RS, PLANE = Cfg::PLANE;
  constexpr int MTH = Cfg::MTH, MTW = Cfg::MTW, MTX = Cfg::MTX;
  constexpr int WM = Cfg::WM, MPW = Cfg::MPW, NPW = Cfg::NPW;
  constexpr int KC = Cfg::KC, KCP = Cfg::KCP;

  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* halo = smem;                          // [CIC][PLANE]
  float* wl = smem + CIC * PLANE;              // [NG][KCP][COUT]

  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  const int H = a.H, W = a.W;
  const int tiles_x = (W + TW - 1) / TW;
  const int ty0 = (blockIdx.x / tiles_x) * TH;
  const int tx0 = (blockIdx.x % tiles_x) * TW;
  const int bq = blockIdx.y;                  // batch index (incl. clones)
  const int bs = bq / a.clones;               // sample index (shared forward state)
  const int wm = w % WM, wn = w / WM;
  const bool active = w < WM * Cfg::WN;

  // per-lane pixel of MFMA row i = lane & 31 in each of this wave's m-tiles (tile-local)
  int pix_y[MPW], pix_x[MPW];
#pragma unroll
  for (int u = 0; u < MPW; ++u) {
    const int mt = wm * MPW + u;
    const int i = lane & 31, win = i >> 2, sub = i & 3;
    pix_y[u] = (mt / MTX) * MTH + 2 * (win / MW) + (sub >> 1);
    pix_x[u] = (mt % MTX) * MTW + 2 * (win % MW) + (sub & 1);
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

  const int HIN = (AMODE == A_POOLSPARSE) ? H / 2 : H;
  const int WIN = (AMODE == A_POOLSPARSE) ? W / 2 : W;

  for (int chunk = 0; chunk < Cfg::NCHUNK; ++chunk) {
    const int c0 = chunk * CIC;
    __syncthreads();
    // ---- stage the input halo [CIC][HY][HX] (zero outside the image / beyond cin) ----
    for (int idx = tid; idx < CIC * HY * HX; idx += kThreads) {
      const int ci = idx / (HY * HX);
      const int rem = idx - ci * (HY * HX);
      const int hy = rem / HX, hx = rem - (rem / HX) * HX;
      const int gy = ty0 - 1 + hy, gx = tx0 - 1 + hx;
      const int c = c0 + ci;
      float v = 0.f;
      if (gy >= 0 && gy < H && gx >= 0 && gx < W && c < a.cin) {
        if constexpr (AMODE == A_DENSE) {
          v = a.in[(((size_t)bq * a.cin + c) * H + gy) * W + gx];
        } else {
          const size_t q = (((size_t)bq * a.cin + c) * HIN + (gy >> 1)) * WIN + (gx >> 1);
          const size_t qa = (((size_t)bs * a.cin + c) * HIN + (gy >> 1)) * WIN + (gx >> 1);
          const int sub = ((gy & 1) << 1) | (gx & 1);
          v = (a.in_amax[qa] == sub) ? a.in[q] : 0.f;
        }
      }
      halo[ci * PLANE + hy * RS + hx] = v;
    }
    // ---- stage the weight chunk: rows k = ci*9 + tap (channel-major) <- global row c0*9 + k ----
    for (int idx = tid; idx < NG * KCP * (COUT / 4); idx += kThreads) {
      const int g = idx / (KCP * (COUT / 4));
      const int rem = idx - g * (KCP * (COUT / 4));
      const int k = rem / (COUT / 4), c4 = (rem - k * (COUT / 4)) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k < KC) v = *reinterpret_cast<const float4*>(a.wts + ((size_t)g * 9 * CIN + c0 * 9 + k) * COUT + c4);
      *reinterpret_cast<float4*>(wl + ((size_t)g * KCP + k) * COUT + c4) = v;
    }
    __syncthreads();
    // ---- MFMA over the chunk ----
    if (!active) continue;
    const int h = lane >> 5;
#pragma unroll 2
    for (int k0 = 0; k0 < KCP; k0 += 2) {
      const int k = k0 + h;
      const int ci = k / 9, tap = k - ci * 9;     // accumulation order: channel-major, tap-minor
      const int ky = tap / 3, kx = tap - ky * 3;
      const bool kvalid = k < KC;
      const int off = ci * PLANE + ky * RS + kx;
      float av[MPW];
#pragma unroll
      for (int u = 0; u < MPW; ++u) av[u] = kvalid ? halo[off + pix_y[u] * RS + pix_x[u]] : 0.f;
#pragma unroll
      for (int v = 0; v < NPW; ++v) {
        const int co = (wn * NPW + v) * 32 + (lane & 31);
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          const float bv = wl[((size_t)g * KCP + k) * COUT + co];
#pragma unroll
          for (int u = 0; u < MPW; ++u) {
            float x = av[u];
            if constexpr (EPI != EPI_BWD && NG == 3) {
              // forward Gamma with possibly negative inputs: (x, x+, x-) against (W, W+, W-)
              x = (g == 0) ? x : (g == 1 ? fmaxf(x, 0.f) : fminf(x, 0.f));
            } else if constexpr (EPI != EPI_BWD && NG == 2) {
              x = (g == 0) ? x : fmaxf(x, 0.f);
            }
            acc[g][u][v] = mfma32(x, bv, acc[g][u][v]);
          }
        }
      }
    }
  }

  // ---- epilogue ----
  if (!active) return;
  // lane holds, for m-tile u / n-tile v: channel co = n0 + (lane&31), MFMA rows
  // i = (r&3) + 8(r>>2) + 4(lane>>5) -> window win = 2(r>>2) + (lane>>5), sub = r&3.
#pragma unroll
  for (int u = 0; u < MPW; ++u) {
    const int mt = wm * MPW + u;
    const int mty = (mt / MTX) * MTH, mtx = (mt % MTX) * MTW;
#pragma unroll
    for (int v = 0; v < NPW; ++v) {
      const int co = (wn * NPW + v) * 32 + (lane & 31);
      if (co >= a.cout) continue;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int win = 2 * g4 + (lane >> 5);
        const int wy = win / MW, wx = win % MW;
        const int py0 = ty0 + mty + 2 * wy, px0 = tx0 + mtx + 2 * wx;   // top-left pixel of window
        if (py0 >= H || px0 >= W) continue;                             // partial tile (small maps)
        if constexpr (EPI == EPI_FWD_POOL || EPI == EPI_FWD_RELU) {
          const float b0 = a.bias ? a.bias[co] : 0.f;
          float y[4];
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const float z = acc[0][u][v][4 * g4 + s] + b0;
            y[s] = z > 0.f ? z : 0.f;
            if (z != z) y[s] = z;   // relu(NaN) = NaN (torch semantics)
          }
          auto den_at = [&](int s) -> float {
            const int py = py0 + (s >> 1), px = px0 + (s & 1);
            if (a.den_map) return a.den_map[((size_t)co * H + py) * W + px];
            if constexpr (NG >= 2) {
              const float bp = a.bias ? a.bias[COUT + co] : 0.f;
              const float bn = a.bias ? a.bias[2 * COUT + co] : 0.f;
              const float z0 = acc[1][u][v][4 * g4 + s] + bp;
              float z1 = bn;
              if constexpr (NG == 3) z1 = acc[2][u][v][4 * g4 + s] + bn;
              return z0 + z1;
            }
            // Epsilon: den = conv(x; W) + b_den (b_den = b, or 0 under zero_params=['bias'])
            return acc[0][u][v][4 * g4 + s] + (a.bias ? a.bias[COUT + co] : 0.f);
          };
          if constexpr (EPI == EPI_FWD_POOL) {
            // torch max_pool2d: first maximum in row-major window order; NaN wins
            int am = 0;
            float m = y[0];
#pragma unroll
            for (int s = 1; s < 4; ++s)
              if (y[s] > m || (y[s] != y[s] && m == m)) { m = y[s]; am = s; }
            const int H2 = H >> 1, W2 = W >> 1;
            const size_t o = (((size_t)bq * a.cout + co) * H2 + (py0 >> 1)) * W2 + (px0 >> 1);
            a.out[o] = m;
            a.out_amax[o] = (uint8_t)am;
            if (a.out_den) a.out_den[o] = den_at(am);
          } else {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              const int py = py0 + (s >> 1), px = px0 + (s & 1);
              const size_t o = (((size_t)bq * a.cout + co) * H + py) * W + px;
              a.out[o] = y[s];
              if (a.out_den) a.out_den[o] = den_at(s);
            }
          }
        } else {   // EPI_BWD
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const int py = py0 + (s >> 1), px = px0 + (s & 1);
            const size_t os = (((size_t)bs * a.cout + co) * H + py) * W + px;
            const size_t oq = (((size_t)bq * a.cout + co) * H + py) * W + px;
            float R;
            if (a.xmode == XM_NONE) {
              R = acc[0][u][v][4 * g4 + s];
            } else {
              const float x = a.x[os];
              if (a.xmode == XM_MUL) {
                R = x * acc[0][u][v][4 * g4 + s];
              } else {   // XM_SPLIT: x+ * acc0 + x- * acc1
                const float xp = fmaxf(x, 0.f);
                R = xp * acc[0][u][v][4 * g4 + s];
                if constexpr (NG >= 2) R += fminf(x, 0.f) * acc[1][u][v][4 * g4 + s];
              }
            }
            if (a.post == POST_DIV) {
              const float x = a.x[os];
              R = (x > 0.f) ? R / stab(a.den[os], a.eps) : 0.f;
            } else if (a.post == POST_MASK) {
              R = (a.x[os] > 0.f) ? R : 0.f;
            }
            a.out[oq] = R;
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// dispatch table
// ---------------------------------------------------------------------------
typedef void (*KernFn)(ConvArgs);

struct Entry {
  int cin_p, cout_p, th, tw, mw, cic, ng, amode, epi;
  KernFn fn;
  size_t lds;
};

#define CONV_ENTRY(CIN, COUT, TH, TW, MW, CIC, NG, AM, EP)                                              \
  Entry{CIN, COUT, TH, TW, MW, CIC, NG, AM, EP, conv3x3_kernel<CIN, COUT, TH, TW, MW, CIC, NG, AM, EP>, \
        ConvCfg<CIN, COUT, TH, TW, MW, CIC, NG, AM, EP>::lds_floats * sizeof(float)}

// Tile choice by output width: W >= 32 -> 8x32 (MW 8); W == 16 -> 8x16 (MW 8); W == 8 -> 8x8 (MW 4);
// W == 4 -> 4x4?  (not needed: pooled 4x4 maps feed the dense head)
#define CONV_FAMILY(CIN, COUT, CIC, NG, AM, EP)                      \
  CONV_ENTRY(CIN, COUT, 8, 32, 8, CIC, NG, AM, EP),                  \
  CONV_ENTRY(CIN, COUT, 8, 16, 8, CIC, NG, AM, EP),                  \
  CONV_ENTRY(CIN, COUT, 8, 8, 4, CIC, NG, AM, EP)

// forward: (cin_p, cout_p) pairs of GTZAN-128 / toy (padded to 32 output channels)
#define FWD_SET(CIN, COUT, CIC)                                                        \
  CONV_FAMILY(CIN, COUT, CIC, 1, A_DENSE, EPI_FWD_POOL),                               \
  CONV_FAMILY(CIN, COUT, CIC, 2, A_DENSE, EPI_FWD_POOL),                               \
  CONV_FAMILY(CIN, COUT, CIC, 3, A_DENSE, EPI_FWD_POOL),                               \
  CONV_FAMILY(CIN, COUT, CIC, 1, A_DENSE, EPI_FWD_RELU),                               \
  CONV_FAMILY(CIN, COUT, CIC, 2, A_DENSE, EPI_FWD_RELU),                               \
  CONV_FAMILY(CIN, COUT, CIC, 3, A_DENSE, EPI_FWD_RELU)

#define BWD_SET(CIN, COUT, CIC)                                                        \
  CONV_FAMILY(CIN, COUT, CIC, 1, A_DENSE, EPI_BWD),                                    \
  CONV_FAMILY(CIN, COUT, CIC, 2, A_DENSE, EPI_BWD),                                    \
  CONV_FAMILY(CIN, COUT, CIC, 1, A_POOLSPARSE, EPI_BWD),                               \
  CONV_FAMILY(CIN, COUT, CIC, 2, A_POOLSPARSE, EPI_BWD)

const Entry kTable[] = {
    // forward: cin_p -> cout_p
    FWD_SET(1, 32, 1),
    FWD_SET(32, 32, 16),
    FWD_SET(32, 64, 16),
    FWD_SET(64, 64, 8),
    FWD_SET(64, 128, 8),
    // backward (transposed): cin_p = forward cout_p, cout_p = forward cin_p (padded to 32)
    BWD_SET(128, 64, 16),
    BWD_SET(64, 64, 16),
    BWD_SET(64, 32, 16),
    BWD_SET(32, 32, 16),
};

int pad32(int c) { return (c + 31) / 32 * 32; }

const Entry* find(int cin_p, int cout_p, int W, int ng, int amode, int epi) {
  int th = 8, tw, mw;
  if (W >= 32) { tw = 32; mw = 8; }
  else if (W > 8) { tw = 16; mw = 8; }
  else { tw = 8; mw = 4; }
  for (const Entry& e : kTable)
    if (e.cin_p == cin_p && e.cout_p == cout_p && e.th == th && e.tw == tw && e.mw == mw && e.ng == ng &&
        e.amode == amode && e.epi == epi)
      return &e;
  return nullptr;
}

int launch(const Entry* e, const ConvArgs& args, int batch, hipStream_t s) {
  static bool attr_done[sizeof(kTable) / sizeof(kTable[0])] = {false};
  const int idx = (int)(e - kTable);
  if (!attr_done[idx]) {
    DRSA_HIP(hipFuncSetAttribute((const void*)e->fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)e->lds));
    attr_done[idx] = true;
  }
  const int tiles = ((args.H + e->th - 1) / e->th) * ((args.W + e->tw - 1) / e->tw);
  hipLaunchKernelGGL(e->fn, dim3(tiles, batch), dim3(kThreads), e->lds, s, args);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

int cin_pad(int cin) { return cin == 1 ? 1 : pad32(cin); }

}  // namespace

extern "C" {

size_t drsa_amd_conv_weight_floats(int cin, int cout, int ng) {
  return (size_t)ng * 9 * cin_pad(cin) * pad32(cout);
}

int drsa_amd_conv_fwd(const float* in, const float* wts, const float* bias, const float* den_map, float* out,
                      uint8_t* out_amax, float* out_den, int B, int cin, int cout, int H, int W, int ng,
                      int pool, void* stream) {
  DRSA_REQUIRE(B > 0 && H > 0 && W > 0, "conv_fwd: bad shape");
  DRSA_REQUIRE(ng >= 1 && ng <= 3, "conv_fwd: ng must be 1..3");
  DRSA_REQUIRE(H % 2 == 0 && W % 2 == 0, "conv_fwd: H and W must be even (got %dx%d)", H, W);
  DRSA_REQUIRE(!pool || out_amax, "conv_fwd: pool needs out_amax");
  const int cin_p = cin_pad(cin), cout_p = pad32(cout);
  const Entry* e = find(cin_p, cout_p, W, ng, A_DENSE, pool ? EPI_FWD_POOL : EPI_FWD_RELU);
  if (!e) {
    drsa::set_error("conv_fwd: no kernel for cin=%d cout=%d W=%d ng=%d pool=%d", cin, cout, W, ng, pool);
    return DRSA_EUNSUPPORTED;
  }
  ConvArgs a{};
  a.in = in; a.wts = wts; a.bias = bias; a.den_map = den_map; a.out = out; a.out_amax = out_amax;
  a.out_den = out_den; a.H = H; a.W = W; a.cin = cin; a.cout = cout; a.clones = 1;
  return launch(e, a, B, (hipStream_t)stream);
}

int drsa_amd_conv_bwd(const float* g, const uint8_t* g_amax, const float* wts, const float* x, const float* den,
                      float* out, int Bq, int clones, int cin, int cout, int H, int W, int ng, int xmode,
                      int post, float eps, void* stream) {
  DRSA_REQUIRE(Bq > 0 && clones > 0 && Bq % clones == 0, "conv_bwd: bad batch/clones");
  DRSA_REQUIRE(ng >= 1 && ng <= 2, "conv_bwd: ng must be 1..2");
  DRSA_REQUIRE(H % 2 == 0 && W % 2 == 0, "conv_bwd: H and W must be even");
  DRSA_REQUIRE(xmode == XM_NONE || x, "conv_bwd: xmode needs x");
  DRSA_REQUIRE(post == POST_NONE || (x && (den || post == POST_MASK)), "conv_bwd: POST_DIV needs x and den");
  const int cin_p = pad32(cin), cout_p = pad32(cout);
  const Entry* e = find(cin_p, cout_p, W, ng, g_amax ? A_POOLSPARSE : A_DENSE, EPI_BWD);
  if (!e) {
    drsa::set_error("conv_bwd: no kernel for cin=%d cout=%d W=%d ng=%d sparse=%d", cin, cout, W, ng, g_amax != nullptr);
    return DRSA_EUNSUPPORTED;
  }
  ConvArgs a{};
  a.in = g; a.in_amax = g_amax; a.wts = wts; a.x = x; a.den = den; a.out = out; a.H = H; a.W = W;
  a.cin = cin; a.cout = cout; a.clones = clones; a.xmode = xmode; a.post = post; a.eps = eps;
  return launch(e, a, Bq, (hipStream_t)stream);
}

}  // extern "C"
