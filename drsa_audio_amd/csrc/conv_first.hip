// First-layer forward (Cin = 1) with the fused ReLU + 2x2 max-pool + argmax + LRP denominator.
//
// The generic MFMA conv (lrp_conv_kernel.h) does only 9 useful k-steps per staged chunk here
// and spends its time in the LDS staging and the epilogue; the layer is HBM-bound on its
// pooled outputs (y, argmax, den: 9 B per pooled cell and channel).  This kernel keeps the
// whole 4x10 input patch of four adjacent pool windows in registers, runs every output
// pixel's 9-tap fma chain on the VALU as packed fmas (v_pk_fma_f32: a window column's upper and
// lower pixel per instruction; weights and bias as scalar operands) in the k order of the MFMA
// kernel and oracle/lrp_exact.c:conv2d_exact, so the result is bit-identical, pools with
// branch-free selects, and writes float4 rows of y and den plus one packed uint32 of argmax
// bytes per channel.
//
// Reference: cxai/model/create_model.py:100-137 (conv -> ReLU -> MaxPool2d) and the rule
// denominators of SURVEY App. A (WSquare map / Epsilon z / Gamma z+ + z-).
#include "common.h"
#include "lrp_conv.h"

#include <stdlib.h>

namespace {

constexpr int kThreads = 256;
#ifndef DRSA_FIRST_FWD_PK
#define DRSA_FIRST_FWD_PK 1
#endif
typedef float fp2 __attribute__((ext_vector_type(2)));

// DEN: 0 none, 1 input-independent map (WSquare / Flat), 2 computed from the rule's sets,
//      3 the map of 1 with the per-sample copy on the border ring only (den_ring_only)
template <int NG, int DEN>
#ifndef DRSA_FIRST_FWD_RING2
#define DRSA_FIRST_FWD_RING2 1
#endif
#ifndef DRSA_FIRST_FWD_RUNROLL
#define DRSA_FIRST_FWD_RUNROLL 8   // ring pass: 8 channels of gathers in flight (4: +3 %, 16: +1 %, micro-benchmark)
#endif
#ifndef DRSA_FIRST_FWD_WPE
#define DRSA_FIRST_FWD_WPE 1
#endif
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(DRSA_FIRST_FWD_WPE))) void first_conv_pool_kernel(ConvArgs a, const float* __restrict__ wts, const float* __restrict__ bias,
                                                            const float* __restrict__ den_map, int cout_p, int total) {
  const int t = blockIdx.x * kThreads + threadIdx.x;
  if (t >= total) return;
  const int H = a.H, W = a.W, H2 = H >> 1, W2 = W >> 1, gq = W2 >> 2;
  const int b = t / (H2 * gq), rem = t % (H2 * gq);
  const int qy = rem / gq, g4 = rem % gq;
  const int y0 = 2 * qy - 1, x0 = 8 * g4 - 1;

  // input patch rows y0..y0+3, columns x0..x0+9 (zero outside the image)
  float xin[4][10];
  const float* src = a.in + (size_t)b * H * W;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int yy = y0 + r;
    const bool rok = yy >= 0 && yy < H;
    const float* row = src + (size_t)(rok ? yy : 0) * W;
    const float4 v0 = *reinterpret_cast<const float4*>(row + x0 + 1);
    const float4 v1 = *reinterpret_cast<const float4*>(row + x0 + 5);
    const float l = row[x0 >= 0 ? x0 : 0];
    const float rr = row[x0 + 9 < W ? x0 + 9 : W - 1];
    xin[r][0] = (rok && x0 >= 0) ? l : 0.f;
    xin[r][1] = rok ? v0.x : 0.f; xin[r][2] = rok ? v0.y : 0.f; xin[r][3] = rok ? v0.z : 0.f; xin[r][4] = rok ? v0.w : 0.f;
    xin[r][5] = rok ? v1.x : 0.f; xin[r][6] = rok ? v1.y : 0.f; xin[r][7] = rok ? v1.z : 0.f; xin[r][8] = rok ? v1.w : 0.f;
    xin[r][9] = (rok && x0 + 9 < W) ? rr : 0.f;
  }

  const size_t plane2 = (size_t)H2 * W2;
  const size_t obase = ((size_t)b * a.cout) * plane2 + (size_t)qy * W2 + 4 * g4;
  // den_ring_only (map den): the backward needs the per-sample copy only on the border ring of
  // float4 groups (POST_DIV_RING; the map is one value per channel elsewhere), stored compactly:
  // per plane [row 0 | row H2-1 | rows 1..H2-2 x (first 4, last 4 columns)], coalesced float4s
  const bool den_ring = (DEN == 1 && a.den_ring_only) || DEN == 3;
  const bool on_ring = qy == 0 || qy == H2 - 1 || g4 == 0 || 4 * g4 + 4 >= W2;
  const int ring_n = 2 * W2 + 8 * (H2 - 2);
  const int ring_i = qy == 0 ? 4 * g4 : qy == H2 - 1 ? W2 + 4 * g4 : 2 * W2 + (qy - 1) * 8 + (g4 == 0 ? 0 : 4);
  const size_t rbase = (size_t)b * a.cout * ring_n + ring_i;

  // blockIdx.y: channel slice (more waves in flight for the store stream)
  const int cper = (a.cout + gridDim.y - 1) / gridDim.y;
  const int c_lo = blockIdx.y * cper, c_hi = min(a.cout, c_lo + cper);
#if DRSA_FIRST_FWD_PK
  // vertical pixel pairs of the patch: pr[ky][c] = (x[ky][c], x[ky + 1][c]), so one packed fma
  // (v_pk_fma_f32) advances the chains of the window's upper and lower pixel of one column
  fp2 pr[3][10];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int c = 0; c < 10; ++c) pr[ky][c] = fp2{xin[ky][c], xin[ky + 1][c]};
#endif
  // 32-bit offsets of the den map (C * H * W < 2^31, checked by the host)
  const int mrow = (2 * qy) * W + 8 * g4;
#ifndef DRSA_FIRST_FWD_CUNROLL
#define DRSA_FIRST_FWD_CUNROLL 4
#endif
  // DEN 3: the channel loop keeps no map loads (none of its waits); each chunk of 32 channels
  // parks its argmax words in LDS (thread-private slots) and the ring lanes then gather the map
  // at their argmax pixels in a second, load-only pass
  constexpr int kChunk = DEN == 3 ? 32 : (1 << 30);
  __shared__ uint32_t am_sh[DEN == 3 ? kChunk : 1][kThreads];
  for (int cc = c_lo; cc < c_hi; cc += kChunk) {
    const int ce = min(c_hi, cc + kChunk);
    // unrolled over channels: the next channels' weight / bias scalar loads issue ahead of this
    // channel's fma chains instead of one load latency per channel
#pragma unroll DRSA_FIRST_FWD_CUNROLL
    for (int co = cc; co < ce; ++co) {
      float w[NG][9];
#pragma unroll
      for (int g = 0; g < NG; ++g)
#pragma unroll
        for (int k = 0; k < 9; ++k) w[g][k] = wts[(g * 9 + k) * cout_p + co];
      const float b0 = bias ? bias[co] : 0.f;

      float ym[4], dn[4];
      uint32_t amw = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        // window pixels in torch's row-major order: s = 2 * py + px
        float yy[4];
#if DRSA_FIRST_FWD_PK
        // the window's two columns as two interleaved chains (independent packed fmas back to back)
        fp2 acc[2] = {fp2{0.f, 0.f}, fp2{0.f, 0.f}};
#pragma unroll
        for (int k = 0; k < 9; ++k)
#pragma unroll
          for (int px = 0; px < 2; ++px)
            acc[px] = __builtin_elementwise_fma(pr[k / 3][2 * j + px + k % 3], fp2{w[0][k], w[0][k]}, acc[px]);
#pragma unroll
        for (int px = 0; px < 2; ++px) {
          const fp2 z = acc[px] + fp2{b0, b0};
          // relu with NaN passed through: !(z <= 0) ? z : 0
          yy[px] = z.x <= 0.f ? 0.f : z.x;
          yy[2 + px] = z.y <= 0.f ? 0.f : z.y;
        }
#else
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int py = s >> 1, px = s & 1;
          float acc = 0.f;
#pragma unroll
          for (int k = 0; k < 9; ++k) acc = __builtin_fmaf(xin[py + k / 3][2 * j + px + k % 3], w[0][k], acc);
          const float z = acc + b0;
          yy[s] = z <= 0.f ? 0.f : z;   // relu(NaN) = NaN
        }
#endif
        // torch max_pool2d: first maximum in window order; NaN wins (branch-free selects)
        int am = 0;
        float m = yy[0];
#pragma unroll
        for (int s = 1; s < 4; ++s) {
          // (y > m) | (isnan(y) & !isnan(m))  ==  !(y <= m) & !isnan(m)
          const bool take = !(yy[s] <= m) & (m == m);
          m = take ? yy[s] : m;
          am = take ? s : am;
        }
        ym[j] = m;
        amw |= (uint32_t)am << (8 * j);
        if constexpr (DEN == 1) {
          // off the ring (den_ring) nothing is stored: those lanes read one address (an L1
          // broadcast) instead of their scattered map pixel
          const int py = am >> 1, px = am & 1;
          const int mi = co * H * W + mrow + py * W + 2 * j + px;
          dn[j] = den_map[(den_ring && !on_ring) ? 0 : mi];
        } else if constexpr (DEN == 2) {
          // the rule's denominator at the argmax pixel only (every chain is per pixel)
          float xs[9];
#pragma unroll
          for (int k = 0; k < 9; ++k) {
            // select the tap inputs of pixel `am` (4-way, branch-free)
            const float c0 = xin[k / 3][2 * j + k % 3], c1 = xin[k / 3][2 * j + 1 + k % 3];
            const float c2 = xin[1 + k / 3][2 * j + k % 3], c3 = xin[1 + k / 3][2 * j + 1 + k % 3];
            xs[k] = am == 0 ? c0 : (am == 1 ? c1 : (am == 2 ? c2 : c3));
          }
          const float bpos = bias ? bias[cout_p + co] : 0.f;
          if constexpr (NG >= 2) {
            const float bneg = bias ? bias[2 * cout_p + co] : 0.f;
            float a1 = 0.f;
#pragma unroll
            for (int k = 0; k < 9; ++k) a1 = __builtin_fmaf(NG == 3 ? fmaxf(xs[k], 0.f) : xs[k], w[1][k], a1);
            const float z0 = a1 + bpos;
            float z1 = bneg;
            if constexpr (NG == 3) {
              float a2 = 0.f;
#pragma unroll
              for (int k = 0; k < 9; ++k) a2 = __builtin_fmaf(fminf(xs[k], 0.f), w[2][k], a2);
              z1 = a2 + bneg;
            }
            dn[j] = z0 + z1;
          } else {
            // Epsilon: den = conv(x; W) + b_den
            float a0 = 0.f;
#pragma unroll
            for (int k = 0; k < 9; ++k) a0 = __builtin_fmaf(xs[k], w[0][k], a0);
            dn[j] = a0 + bpos;
          }
        }
      }
      const size_t o = obase + (size_t)co * plane2;
      *reinterpret_cast<float4*>(a.out + o) = make_float4(ym[0], ym[1], ym[2], ym[3]);
      *reinterpret_cast<uint32_t*>(a.out_amax + o) = amw;
      if constexpr (DEN == 3) {
        am_sh[co - cc][threadIdx.x] = amw;
      } else if constexpr (DEN != 0) {
        if (!den_ring)
          *reinterpret_cast<float4*>(a.out_den + o) = make_float4(dn[0], dn[1], dn[2], dn[3]);
        else if (on_ring)
          *reinterpret_cast<float4*>(a.out_den + rbase + (size_t)co * ring_n) = make_float4(dn[0], dn[1], dn[2], dn[3]);
      }
    }
    if constexpr (DEN == 3) {
      if (on_ring) {
#pragma unroll DRSA_FIRST_FWD_RUNROLL
        for (int co = cc; co < ce; ++co) {
          const uint32_t amw = am_sh[co - cc][threadIdx.x];
          float dn[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int am = (amw >> (8 * j)) & 3;
            dn[j] = den_map[co * H * W + mrow + (am >> 1) * W + 2 * j + (am & 1)];
          }
          *reinterpret_cast<float4*>(a.out_den + rbase + (size_t)co * ring_n) = make_float4(dn[0], dn[1], dn[2], dn[3]);
        }
      }
    }
  }
}

template <int NG>
int launch_ng(const ConvArgs& a, int cout_p, int B, hipStream_t s) {
  const int total = B * (a.H / 2) * (a.W / 8);
  // the kernel can split the channels over grid.y; more waves measured no gain at the bench shape
  // (store-bound), so one split
  const int cs = 1;
  const dim3 grid((total + kThreads - 1) / kThreads, cs);
  if (!a.out_den) hipLaunchKernelGGL((first_conv_pool_kernel<NG, 0>), grid, dim3(kThreads), 0, s, a, a.wts, a.bias, a.den_map, cout_p, total);
  else if (a.den_map && a.den_ring_only && DRSA_FIRST_FWD_RING2)
    hipLaunchKernelGGL((first_conv_pool_kernel<NG, 3>), grid, dim3(kThreads), 0, s, a, a.wts, a.bias, a.den_map, cout_p, total);
  else if (a.den_map) hipLaunchKernelGGL((first_conv_pool_kernel<NG, 1>), grid, dim3(kThreads), 0, s, a, a.wts, a.bias, a.den_map, cout_p, total);
  else hipLaunchKernelGGL((first_conv_pool_kernel<NG, 2>), grid, dim3(kThreads), 0, s, a, a.wts, a.bias, a.den_map, cout_p, total);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}

}  // namespace

// Cin = 1, pooled output, W % 8 == 0 (checked by the caller, drsa_amd_conv_fwd)
int drsa_first_conv_pool(const ConvArgs& a, int cout_p, int ng, int B, hipStream_t s) {
  DRSA_REQUIRE((long long)a.cout * a.H * a.W < (1LL << 31), "conv_fwd: cout*H*W must be < 2^31 (32-bit den-map offsets)");
  if (ng == 1) return launch_ng<1>(a, cout_p, B, s);
  if (ng == 2) return launch_ng<2>(a, cout_p, B, s);
  return launch_ng<3>(a, cout_p, B, s);
}
