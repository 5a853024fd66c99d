// Host dispatch of the 3x3 conv kernels (kernel: lrp_conv_kernel.h; instantiations: conv_*.hip).
#include "common.h"
#include "lrp_conv.h"
#include "lrp_conv_kernel.h"

#include <stdlib.h>

// ---------------------------------------------------------------------------
// dispatch table
// ---------------------------------------------------------------------------
namespace drsa_conv {
extern const Table kTableFwdA, kTableFwdB, kTableFwdC, kTableFwdD, kTableFwdE, kTableBwdA, kTableBwdB, kTableBwdC,
    kTableFwdBfA, kTableFwdBfB, kTableFwdBfC, kTableFwdP4, kTableBwdBfA, kTableBwdBfB, kTableSmall;
}

namespace {
using drsa_conv::Entry;
using namespace drsa_conv;

const drsa_conv::Table* kTables[] = {&drsa_conv::kTableFwdA,  &drsa_conv::kTableFwdB,   &drsa_conv::kTableFwdC,
                                     &drsa_conv::kTableFwdD,  &drsa_conv::kTableFwdE,   &drsa_conv::kTableBwdA,
                                     &drsa_conv::kTableBwdB,  &drsa_conv::kTableBwdC,   &drsa_conv::kTableFwdBfA,
                                     &drsa_conv::kTableFwdBfB, &drsa_conv::kTableFwdBfC, &drsa_conv::kTableFwdP4,
                                     &drsa_conv::kTableBwdBfA, &drsa_conv::kTableBwdBfB};

int pad32(int c) { return (c + 31) / 32 * 32; }


// Tile shape per direction, channel width and map width (measured choices; variant builds change
// them with -D, scripts/build_variant.py):
// * W >= 32: 8 x 32 tiles, except 8 x 16 for the fp32 forward into 64 channels (half the
//   accumulators: 2 waves/SIMD instead of 1; GTZAN conv_fwd:features.6 0.391 -> 0.356 ms, VGGish
//   features.3 1.43 -> 1.36 ms), the fp32 backward into 64 channels (the 8 x 32 tile with 16-channel
//   chunks spills 91-115 VGPRs) and into 128 channels (VGGish features.17: the 8 x 32 tile spills
//   358-435 VGPRs; 0.291 -> 0.101 ms); the fp32 forward into 128 channels on 8 x 8 tiles (4 times the
//   workgroups at 3 waves/SIMD instead of 1: VGGish conv_fwd:features.17 0.318 -> 0.175 ms, .14 0.168
//   -> 0.100 ms, fp32 standard LRP 7.6k -> 8.0k samples/s; 8 x 16: 0.189 / 0.101 ms);
// * 8 < W < 32: 8 x 8 tiles (more workgroups for the small layers: conv_fwd:features.9 0.287 -> 0.266
//   ms, conv_bwd 0.218 -> 0.214 at B = 512);  W <= 8: 8 x 8.
// Measured slower and dropped: 16-row tiles, 32-channel fp32 forwards / backwards on 8 x 16 tiles.
#ifndef DRSA_CONV_FWD128_TW
#define DRSA_CONV_FWD128_TW 8    // fp32 forward into 128 channels at W >= 32: tile width (32, 16 or 8)
#endif
const Entry* find(int cin_p, int cout_p, int W, int ng, int amode, int epi, int et = 0, int pw = 2) {
  int th = 8, tw, mw;
  const bool fwd_t16 = epi != EPI_BWD && et == 0 && cout_p == 64;
  const bool bwd_t16 = epi == EPI_BWD && et == 0 && ((cout_p == 64 && cin_p <= 128) || cout_p == 128);
  if (W >= 32 && epi != EPI_BWD && et == 0 && cout_p == 128 && DRSA_CONV_FWD128_TW != 32) {
    tw = DRSA_CONV_FWD128_TW;
    mw = tw == 8 ? 4 : 8;
  } else if (W >= 32 && (fwd_t16 || bwd_t16)) { tw = 16; mw = 8; }
  else if (W >= 32) { tw = 32; mw = 8; }
  else { tw = 8; mw = 4; }
  for (const drsa_conv::Table* t : kTables)
    for (int i = 0; i < t->n; ++i) {
      const Entry& e = t->entries[i];
      if (e.cin_p == cin_p && e.cout_p == cout_p && e.th == th && e.tw == tw && e.mw == mw && e.ng == ng &&
          e.amode == amode && e.epi == epi && e.et == et && e.pw == pw)
        return &e;
    }
  return nullptr;
}

// 4 x 8 tiles (conv_small.hip) replace an 8 x 8 entry whose grid would have fewer workgroups than
// this (two per CU): twice the workgroups for the small maps at small batches.  VGGish (B = 32):
// conv_fwd:features.24 / .28 0.108 / 0.103 -> 0.064 / 0.061 ms, conv_bwd:features.31 0.060 ->
// 0.044, fp32 standard LRP 8.2k -> 8.6k samples/s; at GTZAN's 512 workgroups (features.12, B = 512)
// 8 x 8 stays faster (4 x 8: 0.093 -> 0.119 ms forward, 0.051 -> 0.080 backward)
#ifndef DRSA_CONV_SMALL_WG
#define DRSA_CONV_SMALL_WG 512
#endif
const Entry* small_tile(const Entry* e, int H, int W, int batch) {
  if (e->th != 8 || e->tw != 8) return e;
  if ((int64_t)((H + 7) / 8) * ((W + 7) / 8) * batch >= DRSA_CONV_SMALL_WG) return e;
  for (int i = 0; i < drsa_conv::kTableSmall.n; ++i) {
    const Entry& c = drsa_conv::kTableSmall.entries[i];
    if (c.cin_p == e->cin_p && c.cout_p == e->cout_p && c.ng == e->ng && c.amode == e->amode && c.epi == e->epi &&
        c.et == e->et && c.pw == e->pw)
      return &c;
  }
  return e;
}

int launch(const Entry* e0, const ConvArgs& args, int batch, hipStream_t s) {   // batch = grid.y
  // the kernels address one sample's planes with 32-bit offsets from a per-sample base
  DRSA_REQUIRE((int64_t)(args.cin > args.cout ? args.cin : args.cout) * args.H * args.W < ((int64_t)1 << 31),
               "conv: one sample's channels x H x W must stay below 2^31");
  const Entry* e = small_tile(e0, args.H, args.W, batch);
  DRSA_SMEM(e->fn, e->lds);   // per device, thread-safe
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
  DRSA_REQUIRE(pool >= 0 && pool <= 2, "conv_fwd: pool must be 0 (none), 1 (2x2) or 2 (2x4)");
  DRSA_REQUIRE(!pool || out_amax, "conv_fwd: pool needs out_amax");
  DRSA_REQUIRE(pool || W % 4 == 0, "conv_fwd: an unpooled output needs W %% 4 == 0 (float4 epilogue; got W=%d)", W);
  DRSA_REQUIRE(pool != 2 || W % 4 == 0, "conv_fwd: a 2x4 pool needs W %% 4 == 0 (got W=%d)", W);
  const int cin_p = cin_pad(cin), cout_p = pad32(cout);
  if (cin == 1 && pool == 1 && W % 8 == 0) {   // the Cin = 1 VALU kernel (conv_first.hip)
    ConvArgs a{};
    a.in = in; a.wts = wts; a.bias = bias; a.den_map = den_map; a.out = out; a.out_amax = out_amax;
    a.out_den = out_den; a.H = H; a.W = W; a.cin = cin; a.cout = cout; a.clones = 1;
    return drsa_first_conv_pool(a, cout_p, ng, B, (hipStream_t)stream);
  }
  const Entry* e = find(cin_p, cout_p, W, ng, A_DENSE, pool ? EPI_FWD_POOL : EPI_FWD_RELU, 0, pool == 2 ? 4 : 2);
  if (!e) {
    drsa::set_error("conv_fwd: no kernel for cin=%d cout=%d W=%d ng=%d pool=%d", cin, cout, W, ng, pool);
    return DRSA_EUNSUPPORTED;
  }
  ConvArgs a{};
  a.in = in; a.wts = wts; a.bias = bias; a.den_map = den_map; a.out = out; a.out_amax = out_amax;
  a.out_den = out_den; a.H = H; a.W = W; a.cin = cin; a.cout = cout; a.clones = 1;
  return launch(e, a, B, (hipStream_t)stream);
}

int drsa_amd_conv_fwd_has_kernel(int cin, int cout, int W, int ng, int pool, int bf16) {
  if (cin == 1 && !bf16 && pool == 1) return 1;   // conv_first (W % 8 == 0) or the generic Cin = 1 kernels
  if (pool < 0 || pool > 2 || ng < 1 || ng > 3 || (bf16 && cin == 1)) return 0;
  return find(bf16 ? pad32(cin) : cin_pad(cin), pad32(cout), W, ng, A_DENSE, pool ? EPI_FWD_POOL : EPI_FWD_RELU, bf16 ? 1 : 0,
              pool == 2 ? 4 : 2) != nullptr;
}

size_t drsa_amd_conv_weight_bf16_elems(int cin, int cout, int ng) {
  return (size_t)ng * 9 * pad32(cin) * pad32(cout);
}

int drsa_amd_conv_fwd_bf16(const float* in, const uint16_t* wts, const float* bias, const float* den_map, float* out,
                           uint8_t* out_amax, float* out_den, int B, int cin, int cout, int H, int W, int ng,
                           int pool, void* stream) {
  DRSA_REQUIRE(B > 0 && H > 0 && W > 0, "conv_fwd_bf16: bad shape");
  DRSA_REQUIRE(cin > 1, "conv_fwd_bf16: cin = 1 runs on drsa_amd_conv_fwd (fp32 VALU kernel)");
  DRSA_REQUIRE(ng >= 1 && ng <= 3, "conv_fwd_bf16: ng must be 1..3");
  DRSA_REQUIRE(H % 2 == 0 && W % 2 == 0, "conv_fwd_bf16: H and W must be even (got %dx%d)", H, W);
  DRSA_REQUIRE(pool >= 0 && pool <= 2, "conv_fwd_bf16: pool must be 0 (none), 1 (2x2) or 2 (2x4)");
  DRSA_REQUIRE(!pool || out_amax, "conv_fwd_bf16: pool needs out_amax");
  DRSA_REQUIRE(pool || W % 4 == 0, "conv_fwd_bf16: an unpooled output needs W %% 4 == 0 (got W=%d)", W);
  DRSA_REQUIRE(pool != 2 || W % 4 == 0, "conv_fwd_bf16: a 2x4 pool needs W %% 4 == 0 (got W=%d)", W);
  DRSA_REQUIRE(((uintptr_t)wts & 15) == 0, "conv_fwd_bf16: weights must be 16-byte aligned");
  const Entry* e = find(pad32(cin), pad32(cout), W, ng, A_DENSE, pool ? EPI_FWD_POOL : EPI_FWD_RELU, 1, pool == 2 ? 4 : 2);
  if (!e) {
    drsa::set_error("conv_fwd_bf16: no kernel for cin=%d cout=%d W=%d ng=%d pool=%d", cin, cout, W, ng, pool);
    return DRSA_EUNSUPPORTED;
  }
  ConvArgs a{};
  a.in = in; a.wts = reinterpret_cast<const float*>(wts); a.bias = bias; a.den_map = den_map; a.out = out;
  a.out_amax = out_amax; a.out_den = out_den; a.H = H; a.W = W; a.cin = cin; a.cout = cout; a.clones = 1;
  return launch(e, a, B, (hipStream_t)stream);
}

int drsa_amd_conv_bwd(const float* g, const uint8_t* g_amax, const float* wts, const float* x, const float* den,
                      float* out, int Bq, int clones, int cin, int cout, int H, int W, int ng, int xmode,
                      int post, float eps, void* stream) {
  DRSA_REQUIRE(Bq > 0 && clones > 0 && Bq % clones == 0, "conv_bwd: bad batch/clones");
  DRSA_REQUIRE(ng >= 1 && ng <= 2, "conv_bwd: ng must be 1..2");
  DRSA_REQUIRE(H % 2 == 0 && W % 4 == 0, "conv_bwd: H must be even and W %% 4 == 0 (got %dx%d)", H, W);
  DRSA_REQUIRE(xmode == XM_NONE || x, "conv_bwd: xmode needs x");
  DRSA_REQUIRE(post == POST_NONE || (x && (den || post == POST_MASK)), "conv_bwd: POST_DIV needs x and den");
  const int cin_p = pad32(cin), cout_p = pad32(cout);
  ConvArgs a{};
  a.in = g; a.in_amax = g_amax; a.wts = wts; a.x = x; a.den = den; a.out = out; a.H = H; a.W = W;
  a.cin = cin; a.cout = cout; a.clones = clones; a.xmode = xmode; a.post = post; a.eps = eps;
  const Entry* e = find(cin_p, cout_p, W, ng, g_amax ? A_POOLSPARSE : A_DENSE, EPI_BWD);
  if (!e) {
    drsa::set_error("conv_bwd: no kernel for cin=%d cout=%d W=%d ng=%d sparse=%d", cin, cout, W, ng, g_amax != nullptr);
    return DRSA_EUNSUPPORTED;
  }
  return launch(e, a, Bq, (hipStream_t)stream);
}

int drsa_amd_conv_bwd_has_kernel_bf16(int cin, int cout, int W, int ng, int sparse) {
  if (cin < 16 || ng != 1) return 0;
  return find(pad32(cin), pad32(cout), W, ng, sparse ? A_POOLSPARSE : A_DENSE, EPI_BWD, 1) != nullptr;
}

int drsa_amd_conv_bwd_has_kernel_pw(int cin, int cout, int W, int ng, int pool_w) {
  if (cin < 2 || (pool_w != 2 && pool_w != 4) || (pool_w == 4 && (W / 4) % 4 != 0)) return 0;
  return find(pad32(cin), pad32(cout), W, ng, A_POOLSPARSE, EPI_BWD, 0, pool_w) != nullptr;
}

int drsa_amd_conv_bwd_has_kernel_bf16_pw(int cin, int cout, int W, int pool_w) {
  if (cin < 16 || (pool_w != 2 && pool_w != 4)) return 0;
  return find(pad32(cin), pad32(cout), W, 1, A_POOLSPARSE, EPI_BWD, 1, pool_w) != nullptr;
}

int drsa_amd_conv_bwd_bf16_pw(const float* g, const uint8_t* g_amax, int pool_w, const uint16_t* wts, const float* x,
                              const float* den, float* out, int Bq, int clones, int cin, int cout, int H, int W,
                              int xmode, int post, float eps, void* stream) {
  DRSA_REQUIRE(g_amax && (pool_w == 2 || pool_w == 4), "conv_bwd_bf16_pw: needs g_amax and pool_w 2 or 4");
  DRSA_REQUIRE(Bq > 0 && clones > 0 && Bq % clones == 0, "conv_bwd_bf16_pw: bad batch/clones");
  DRSA_REQUIRE(cin >= 16, "conv_bwd_bf16_pw: cin >= 16 (16-channel bf16 chunks)");
  DRSA_REQUIRE(H % 2 == 0 && W % pool_w == 0 && W % 4 == 0, "conv_bwd_bf16_pw: H even, W %% pool_w == 0, W %% 4 == 0");
  DRSA_REQUIRE(xmode == XM_NONE || x, "conv_bwd_bf16_pw: xmode needs x");
  DRSA_REQUIRE(post == POST_NONE || (x && (den || post == POST_MASK)), "conv_bwd_bf16_pw: POST_DIV needs x and den");
  DRSA_REQUIRE(((uintptr_t)wts & 15) == 0, "conv_bwd_bf16_pw: weights must be 16-byte aligned");
  const Entry* e = find(pad32(cin), pad32(cout), W, 1, A_POOLSPARSE, EPI_BWD, 1, pool_w);
  if (!e) {
    drsa::set_error("conv_bwd_bf16_pw: no kernel for cin=%d cout=%d W=%d pool 2x%d", cin, cout, W, pool_w);
    return DRSA_EUNSUPPORTED;
  }
  ConvArgs a{};
  a.in = g; a.in_amax = g_amax; a.wts = reinterpret_cast<const float*>(wts); a.x = x; a.den = den; a.out = out;
  a.H = H; a.W = W; a.cin = cin; a.cout = cout; a.clones = clones; a.xmode = xmode; a.post = post; a.eps = eps;
  return launch(e, a, Bq, (hipStream_t)stream);
}

int drsa_amd_conv_bwd_den_map(const float* g, const uint8_t* g_amax, int pool_w, const void* wts, int wts_bf16,
                              const float* x, const float* den_map, float* out, int Bq, int clones, int cin, int cout,
                              int H, int W, int ng, int xmode, float eps, void* stream) {
  DRSA_REQUIRE(Bq > 0 && clones > 0 && Bq % clones == 0, "conv_bwd_den_map: bad batch/clones");
  DRSA_REQUIRE(x && den_map, "conv_bwd_den_map: needs x and den_map");
  DRSA_REQUIRE(!g_amax || pool_w == 2 || pool_w == 4, "conv_bwd_den_map: pool_w must be 2 or 4");
  DRSA_REQUIRE(H % 2 == 0 && W % 4 == 0, "conv_bwd_den_map: H must be even and W %% 4 == 0 (got %dx%d)", H, W);
  DRSA_REQUIRE(xmode == XM_NONE || xmode == XM_MUL || xmode == XM_SPLIT, "conv_bwd_den_map: bad xmode");
  const int et = wts_bf16 ? 1 : 0;
  DRSA_REQUIRE(!et || (ng == 1 && cin >= 16 && ((uintptr_t)wts & 15) == 0),
               "conv_bwd_den_map: bf16 weights need ng == 1, cin >= 16 and 16-byte alignment");
  DRSA_REQUIRE(et || (ng >= 1 && ng <= 2 && (!g_amax || pool_w == 2 || ng == 1)),
               "conv_bwd_den_map: fp32 weights need ng 1..2 (ng 1 under a 2x4 pool)");
  DRSA_REQUIRE(!g_amax || pool_w == 2 || (W / 4) % 4 == 0,
               "conv_bwd_den_map: a 2x4 pool-sparse g needs W / 4 %% 4 == 0 (got W=%d)", W);
  const int pw = g_amax ? pool_w : 2;
  const Entry* e = find(pad32(cin), pad32(cout), W, ng, g_amax ? A_POOLSPARSE : A_DENSE, EPI_BWD, et, pw);
  if (!e) {
    drsa::set_error("conv_bwd_den_map: no kernel for cin=%d cout=%d W=%d ng=%d sparse=%d bf16=%d pool_w=%d", cin, cout,
                    W, ng, g_amax != nullptr, et, pw);
    return DRSA_EUNSUPPORTED;
  }
  ConvArgs a{};
  a.in = g; a.in_amax = g_amax; a.wts = reinterpret_cast<const float*>(wts); a.x = x; a.den = den_map;
  a.den_shared = 1; a.out = out; a.H = H; a.W = W; a.cin = cin; a.cout = cout; a.clones = clones; a.xmode = xmode;
  a.post = POST_DIV; a.eps = eps;
  return launch(e, a, Bq, (hipStream_t)stream);
}

int drsa_amd_conv_bwd_bf16(const float* g, const uint8_t* g_amax, const uint16_t* wts, const float* x, const float* den,
                           float* out, int Bq, int clones, int cin, int cout, int H, int W, int ng, int xmode,
                           int post, float eps, void* stream) {
  DRSA_REQUIRE(Bq > 0 && clones > 0 && Bq % clones == 0, "conv_bwd_bf16: bad batch/clones");
  DRSA_REQUIRE(ng == 1, "conv_bwd_bf16: ng must be 1 (the Gamma x-/W- term is for the fp32 first layer)");
  DRSA_REQUIRE(cin >= 16, "conv_bwd_bf16: cin >= 16 (16-channel bf16 chunks)");
  DRSA_REQUIRE(H % 2 == 0 && W % 4 == 0, "conv_bwd_bf16: H must be even and W %% 4 == 0 (got %dx%d)", H, W);
  DRSA_REQUIRE(xmode == XM_NONE || x, "conv_bwd_bf16: xmode needs x");
  DRSA_REQUIRE(post == POST_NONE || (x && (den || post == POST_MASK)), "conv_bwd_bf16: POST_DIV needs x and den");
  DRSA_REQUIRE(((uintptr_t)wts & 15) == 0, "conv_bwd_bf16: weights must be 16-byte aligned");
  const Entry* e = find(pad32(cin), pad32(cout), W, ng, g_amax ? A_POOLSPARSE : A_DENSE, EPI_BWD, 1);
  if (!e) {
    drsa::set_error("conv_bwd_bf16: no kernel for cin=%d cout=%d W=%d sparse=%d", cin, cout, W, g_amax != nullptr);
    return DRSA_EUNSUPPORTED;
  }
  ConvArgs a{};
  a.in = g; a.in_amax = g_amax; a.wts = reinterpret_cast<const float*>(wts); a.x = x; a.den = den; a.out = out;
  a.H = H; a.W = W; a.cin = cin; a.cout = cout; a.clones = clones; a.xmode = xmode; a.post = post; a.eps = eps;
  return launch(e, a, Bq, (hipStream_t)stream);
}

int drsa_amd_conv_fwd_den_ring(const float* in, const float* wts, const float* bias, const float* den_map, float* out,
                               uint8_t* out_amax, float* den_ring, int B, int cout, int H, int W, int ng,
                               void* stream) {
  DRSA_REQUIRE(in && wts && den_map && out && out_amax && den_ring, "conv_fwd_den_ring: null pointer");
  DRSA_REQUIRE(B > 0 && H >= 4 && W > 0 && H % 2 == 0 && W % 16 == 0,
               "conv_fwd_den_ring: needs H >= 4 even and W %% 16 == 0 (got %dx%d)", H, W);
  DRSA_REQUIRE(ng >= 1 && ng <= 3, "conv_fwd_den_ring: ng must be 1..3");
  ConvArgs a{};
  a.in = in; a.wts = wts; a.bias = bias; a.den_map = den_map; a.out = out; a.out_amax = out_amax;
  a.out_den = den_ring; a.H = H; a.W = W; a.cin = 1; a.cout = cout; a.clones = 1; a.den_ring_only = 1;
  return drsa_first_conv_pool(a, pad32(cout), ng, B, (hipStream_t)stream);
}

int drsa_amd_conv_bwd_den_ring(const float* g, const uint8_t* g_amax, const void* wts, int wts_bf16, const float* x,
                               const float* den_ring, const float* den_const4, float* out, int Bq, int clones, int cin,
                               int cout, int H, int W, int ng, int xmode, float eps, void* stream) {
  DRSA_REQUIRE(Bq > 0 && clones > 0 && Bq % clones == 0, "conv_bwd_den_ring: bad batch/clones");
  DRSA_REQUIRE(x && den_ring && den_const4, "conv_bwd_den_ring: needs x, den_ring and den_const4");
  // the compact ring (2W + 8(H - 2) floats per channel at the pooled resolution) needs distinct
  // first / last float4 groups per row and at least two rows: the forward's W % 16, H >= 4 unpooled
  DRSA_REQUIRE(H >= 2 && W >= 8 && W % 8 == 0,
               "conv_bwd_den_ring: needs pooled H >= 2 and W >= 8, W %% 8 == 0 (got %dx%d)", H, W);
  DRSA_REQUIRE(xmode == XM_NONE || xmode == XM_MUL || xmode == XM_SPLIT, "conv_bwd_den_ring: bad xmode");
  DRSA_REQUIRE(((uintptr_t)den_const4 & 15) == 0, "conv_bwd_den_ring: den_const4 must be 16-byte aligned");
  const int et = wts_bf16 ? 1 : 0;
  DRSA_REQUIRE(!et || (ng == 1 && cin >= 16 && ((uintptr_t)wts & 15) == 0),
               "conv_bwd_den_ring: bf16 weights need ng == 1, cin >= 16 and 16-byte alignment");
  DRSA_REQUIRE(et || (ng >= 1 && ng <= 2), "conv_bwd_den_ring: ng must be 1..2");
  const Entry* e = find(pad32(cin), pad32(cout), W, ng, g_amax ? A_POOLSPARSE : A_DENSE, EPI_BWD, et);
  if (!e) {
    drsa::set_error("conv_bwd_den_ring: no kernel for cin=%d cout=%d W=%d ng=%d sparse=%d bf16=%d", cin, cout, W, ng,
                    g_amax != nullptr, et);
    return DRSA_EUNSUPPORTED;
  }
  ConvArgs a{};
  a.in = g; a.in_amax = g_amax; a.wts = reinterpret_cast<const float*>(wts); a.x = x; a.den = den_ring;
  a.den_const4 = den_const4; a.out = out; a.H = H; a.W = W; a.cin = cin; a.cout = cout;
  a.clones = clones; a.xmode = xmode; a.post = POST_DIV_RING; a.eps = eps;
  return launch(e, a, Bq, (hipStream_t)stream);
}

}  // extern "C"
