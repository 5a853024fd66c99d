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
};

// conv_first.hip: Cin = 1 forward with fused ReLU + 2x2 pool + argmax + den (VALU; W % 8 == 0)
#include <hip/hip_runtime.h>
int drsa_first_conv_pool(const ConvArgs& a, int cout_p, int ng, int B, hipStream_t s);

