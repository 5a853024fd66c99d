// Internal kernel-argument structs for the LRP engine (not part of the public ABI).
#pragma once
#include <stdint.h>

enum XMode { XM_NONE = 0, XM_MUL = 1, XM_SPLIT = 2 };
// POST_DIV_RING: POST_DIV where the next layer's denominator is a WSquare / Flat map under a 2x2
// pool: one value per channel (den_const4[c][0..3]) off the border ring of float4 groups, and the
// per-sample copy at the argmax (den) only on that ring (the forward writes nothing else)
enum PostMode { POST_NONE = 0, POST_DIV = 1, POST_MASK = 2, POST_DIV_RING = 3 };

struct ConvArgs {
  const float* in;          // A source: NCHW input (dense) or g at pool resolution (sparse)
  const uint8_t* in_amax;   // pool argmax (0..3) of the sparse source, per sample
  const float* wts;         // [NG][9 * cin_p][cout_p], k = ci * 9 + ky * 3 + kx
  const float* bias;        // forward: [3][cout_p] = (b, b+, b-)
  const float* den_map;     // forward, WSquare/Flat: [cout][H][W] input-independent denominator
  const float* den_const4;  // backward POST_DIV_RING: [cout][4] the map's value off the ring
  const float* x;           // backward: activation at output resolution (per sample)
  const float* den;         // backward POST_DIV: next layer's denominator at output resolution
  float* out;
  uint8_t* out_amax;
  float* out_den;
  int H, W;                 // output resolution
  int cin, cout;            // real channel counts (<= padded template sizes)
  int clones;               // batch index / clones = sample index
  int xmode, post;
  float eps;
  int den_ring_only;        // forward (first layer, map den): write out_den on the ring groups only
  int den_shared;           // backward POST_DIV: den is one [cout][H][W] plane for every sample
  int dbg;                  // ablation only (DRSA_AMD_CONV_DBG): 1 no staging loads, 2 no epilogue I/O, 4 no MFMA
  // backward with the first-layer contraction fused (template FF = 1; drsa_amd_conv_bwd_first_fused):
  // out holds R on the tile border ring only, ff_out the first layer's input relevance [Bq][2H][2W]
  // off the tile footprints' border (drsa_amd_first_layer_bwd_border completes it)
  const uint8_t* ff_amax;   // first layer's 2x2 pool argmax [B][cout][H][W]
  const float* ff_w2;       // first layer's squared weights [cout][9]
  float* ff_out;
};

// conv_first.hip: Cin = 1 forward with fused ReLU + 2x2 pool + argmax + den (VALU; W % 8 == 0)
#include <hip/hip_runtime.h>
int drsa_first_conv_pool(const ConvArgs& a, int cout_p, int ng, int B, hipStream_t s);
// lrp_misc.hip: the first layer's w^2 contraction at the border pixels of the FY x FX footprints of
// drsa_amd_conv_bwd_first_fused (g holds R on the footprints' cell rings; H, W at pixel resolution)
int drsa_first_layer_border(const float* g, const uint8_t* amax, const float* w2, float* out, int Bq, int clones,
                            int C, int H, int W, int FY, int FX, hipStream_t s);
