// Log-mel front end: get_slice -> peak_normalizer -> |STFT| -> HTK mel
// -> log10(+eps) -> clamp -> frames frame0..frame0+width-1, fused into one launch.
//
// Reference: cxai/utils/dataloading.py:62-74 (torchaudio Spectrogram(n_fft, hop, power=None) +
// MelScale), :138-176 (transform_wav); cxai/utils/sound.py:8-44 (get_slice), :67-70
// (peak_normalizer).
//
// One workgroup per audio chunk, 8 waves.  The chunk's samples stream through LDS in blocks of
// 8 frames (one frame per wave, reflect padding resolved on the load); each wave runs the
// n_fft-point real FFT as an n_fft/2-point complex Stockham FFT (radices 4/2/3/5) in its own
// LDS ping-pong buffers, the real-input split, |X|, and the sparse triangular mel filterbank
// (each filter is a contiguous band of FFT bins).  Mel columns collect in LDS so the
// [n_mels][width] output leaves as coalesced rows.  The STFT and the filterbank are
// linear and |.| is positively homogeneous, so the per-chunk peak division is applied to the
// mel energies at the end: one read of the waveform (HBM roofline: 4*(L + n_mels*width) B per
// chunk).
#include "common.h"
#include "drsa_amd.h"

#include <stdlib.h>

namespace {

constexpr int LM_WAVES = 8;
constexpr int LM_THREADS = LM_WAVES * 64;
constexpr int LM_MAX_STAGES = 8;

struct LogmelArgs {
  const float* wav;
  int64_t song_stride;       // floats between songs
  int64_t chunk_hop;         // floats between consecutive chunks of a song
  int chunks_per_song;
  int n_chunks;
  int L;                     // chunk length in samples
  int nfft, hop, n_mels, width, frame0;
  int n_stages;
  int radix[LM_MAX_STAGES];
  const float* window;       // [nfft]
  const int* band_lo;        // [n_mels] first FFT bin of filter m
  const int* band_n;         // [n_mels] bins in filter m
  const int* band_off;       // [n_mels] offset of filter m in band_w
  const float* band_w;       // [nnz]
  int nnz;
  int peak_norm, do_clamp;
  float clamp_min, log_eps;
  float* out;                // [n_chunks][n_mels][width]
  // LDS carve (floats), computed on the host
  int o_tw, o_ptw, o_win, o_blo, o_bn, o_boff, o_bw, o_samp, o_fft, o_mel, o_red, smem_floats;
  int o_bwt;                 // n_fft = 800 kernel: band weights transposed [LF_NBT][n_mels + 1]
};

struct cf {
  float x, y;
};
__device__ __forceinline__ cf cadd(cf a, cf b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ cf csub(cf a, cf b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ cf cmul(cf a, cf b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
__device__ __forceinline__ cf cscale(cf a, float s) { return {a.x * s, a.y * s}; }
__device__ __forceinline__ cf mul_negi(cf a) { return {a.y, -a.x}; }   // -i * a

// Wave-local LDS hand-off: all lanes' LDS writes are visible to the wave's later reads.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// forward DFT butterflies (sign -i), in place on v[0..R)
__device__ __forceinline__ void bfly2(cf* v) {
  cf a = v[0], b = v[1];
  v[0] = cadd(a, b);
  v[1] = csub(a, b);
}
__device__ __forceinline__ void bfly4(cf* v) {
  cf t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]);
  cf t2 = cadd(v[1], v[3]), t3 = mul_negi(csub(v[1], v[3]));
  v[0] = cadd(t0, t2);
  v[2] = csub(t0, t2);
  v[1] = cadd(t1, t3);
  v[3] = csub(t1, t3);
}
__device__ __forceinline__ void bfly3(cf* v) {
  const float s = 0.86602540378443864676f;
  cf sm = cadd(v[1], v[2]);
  cf y0 = cadd(v[0], sm);
  cf t = csub(v[0], cscale(sm, 0.5f));
  cf u = mul_negi(cscale(csub(v[1], v[2]), s));
  v[0] = y0;
  v[1] = cadd(t, u);
  v[2] = csub(t, u);
}
__device__ __forceinline__ void bfly5(cf* v) {
  const float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;
  const float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;
  cf b1 = cadd(v[1], v[4]), b2 = cadd(v[2], v[3]);
  cf d1 = csub(v[1], v[4]), d2 = csub(v[2], v[3]);
  cf a0 = v[0];
  cf r1 = cadd(a0, cadd(cscale(b1, c1), cscale(b2, c2)));
  cf r2 = cadd(a0, cadd(cscale(b1, c2), cscale(b2, c1)));
  cf q1 = mul_negi(cadd(cscale(d1, s1), cscale(d2, s2)));   // -i (s1 d1 + s2 d2)
  cf q2 = mul_negi(csub(cscale(d1, s2), cscale(d2, s1)));   // -i (s2 d1 - s1 d2)
  v[0] = cadd(a0, cadd(b1, b2));
  v[1] = cadd(r1, q1);
  v[4] = csub(r1, q1);
  v[2] = cadd(r2, q2);
  v[3] = csub(r2, q2);
}

// One Stockham pass of radix R over M points (Govindaraju et al. 2008 indexing):
//   v[r] = in[j + r*M/R] * W_M^{r*k*M/(Ns*R)}, k = j % Ns;  out[(j/Ns)*Ns*R + k + r*Ns] = DFT_R(v)[r]
template <int R>
__device__ __forceinline__ void stockham_pass(const cf* __restrict__ in, cf* __restrict__ out, const cf* tw, int M,
                                              int Ns, int lane) {
  const int MR = M / R;
  const int tstep = M / (Ns * R);
  for (int j = lane; j < MR; j += 64) {
    const int k = j % Ns;
    cf v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = in[j + r * MR];
    if (Ns > 1) {
#pragma unroll
      for (int r = 1; r < R; ++r) v[r] = cmul(v[r], tw[r * k * tstep]);
    }
    if constexpr (R == 2) bfly2(v);
    if constexpr (R == 3) bfly3(v);
    if constexpr (R == 4) bfly4(v);
    if constexpr (R == 5) bfly5(v);
    const int base = (j / Ns) * Ns * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) out[base + r * Ns] = v[r];
  }
}

__global__ __launch_bounds__(LM_THREADS) void logmel_kernel(LogmelArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  const int chunk = blockIdx.x;
  const int M = a.nfft >> 1, half = a.nfft >> 1;
  const float* x = a.wav + (int64_t)(chunk / a.chunks_per_song) * a.song_stride +
                   (int64_t)(chunk % a.chunks_per_song) * a.chunk_hop;
  cf* tw = reinterpret_cast<cf*>(sm + a.o_tw);      // W_M^j, j < M
  cf* ptw = reinterpret_cast<cf*>(sm + a.o_ptw);    // W_N^k, k <= M
  float* win = sm + a.o_win;
  int* blo = reinterpret_cast<int*>(sm + a.o_blo);
  int* bn = reinterpret_cast<int*>(sm + a.o_bn);
  int* boff = reinterpret_cast<int*>(sm + a.o_boff);
  float* bw = sm + a.o_bw;
  float* samp = sm + a.o_samp;
  cf* fa = reinterpret_cast<cf*>(sm + a.o_fft) + (size_t)w * 2 * M;
  cf* fb = fa + M;
  float* mel = sm + a.o_mel;
  float* red = sm + a.o_red;

  // ---- tables (twiddles from exact fp64 angles rounded once to fp32) ----
  for (int j = tid; j < M; j += LM_THREADS) {
    double s, c;
    sincospi(2.0 * (double)j / (double)M, &s, &c);
    tw[j] = {(float)c, (float)-s};
  }
  for (int k = tid; k <= M; k += LM_THREADS) {
    double s, c;
    sincospi((double)k / (double)M, &s, &c);          // 2*pi*k/N, N = 2M
    ptw[k] = {(float)c, (float)-s};
  }
  for (int i = tid; i < a.nfft; i += LM_THREADS) win[i] = a.window[i];
  for (int m = tid; m < a.n_mels; m += LM_THREADS) {
    blo[m] = a.band_lo[m];
    bn[m] = a.band_n[m];
    boff[m] = a.band_off[m];
  }
  for (int i = tid; i < a.nnz; i += LM_THREADS) bw[i] = a.band_w[i];

  float pk = 0.f;   // running max |x| over this thread's loads
  const int nblk_samp = (LM_WAVES - 1) * a.hop + a.nfft;
  for (int tb = 0; tb < a.width; tb += LM_WAVES) {
    const int nw = min(LM_WAVES, a.width - tb);
    const int base = (a.frame0 + tb) * a.hop - half;
    const int cnt = (nw - 1) * a.hop + a.nfft;
    __syncthreads();   // previous block's frames are done with samp (and the tables are ready)
    for (int i = tid; i < cnt; i += LM_THREADS) {
      int j = base + i;
      j = j < 0 ? -j : j;                                  // reflect (torch pad_mode="reflect")
      j = j >= a.L ? 2 * (a.L - 1) - j : j;
      const float v = x[j];
      samp[i] = v;
      pk = fmaxf(pk, fabsf(v));
    }
    __syncthreads();
    if (w < nw) {
      const float* fr = samp + w * a.hop;
      // pack the windowed real frame as M complex points z[n] = x[2n] + i x[2n+1]
      for (int n = lane; n < M; n += 64) fa[n] = {fr[2 * n] * win[2 * n], fr[2 * n + 1] * win[2 * n + 1]};
      wave_lds_sync();
      cf* src = fa;
      cf* dst = fb;
      int Ns = 1;
      for (int s = 0; s < a.n_stages; ++s) {
        const int R = a.radix[s];
        if (R == 4) stockham_pass<4>(src, dst, tw, M, Ns, lane);
        else if (R == 5) stockham_pass<5>(src, dst, tw, M, Ns, lane);
        else if (R == 3) stockham_pass<3>(src, dst, tw, M, Ns, lane);
        else stockham_pass<2>(src, dst, tw, M, Ns, lane);
        wave_lds_sync();
        Ns *= R;
        cf* t = src;
        src = dst;
        dst = t;
      }
      // real-input split: X[k] = E[k] + W_N^k O[k], E = (Z_k + conj Z_{M-k})/2, O = (Z_k - conj Z_{M-k})/(2i)
      float* mag = reinterpret_cast<float*>(dst);
      for (int k = lane; k <= M; k += 64) {
        const cf zk = src[k == M ? 0 : k];
        const cf zr = src[k == 0 ? 0 : M - k];
        const cf zc = {zr.x, -zr.y};
        const cf e = cscale(cadd(zk, zc), 0.5f);
        const cf d = csub(zk, zc);
        const cf o = {0.5f * d.y, -0.5f * d.x};
        const cf X = cadd(e, cmul(ptw[k], o));
        mag[k] = sqrtf(X.x * X.x + X.y * X.y);
      }
      wave_lds_sync();
      for (int m = lane; m < a.n_mels; m += 64) {
        const float* wm = bw + boff[m];
        const float* mg = mag + blo[m];
        float acc = 0.f;
        for (int q = 0; q < bn[m]; ++q) acc += wm[q] * mg[q];
        mel[m * a.width + tb + w] = acc;
      }
    }
  }
  // samples of the chunk no frame touched still count for the peak
  {
    const int c0 = max(0, a.frame0 * a.hop - half);
    const int c1 = min(a.L, (a.frame0 + a.width - 1) * a.hop - half + a.nfft);
    for (int i = tid; i < c0; i += LM_THREADS) pk = fmaxf(pk, fabsf(x[i]));
    for (int i = c1 + tid; i < a.L; i += LM_THREADS) pk = fmaxf(pk, fabsf(x[i]));
  }
  for (int o = 32; o > 0; o >>= 1) pk = fmaxf(pk, shfl_xor(pk, o));
  if (lane == 0) red[w] = pk;
  __syncthreads();
  float p = red[0];
  for (int i = 1; i < LM_WAVES; ++i) p = fmaxf(p, red[i]);
  const float inv_scale = a.peak_norm ? p : 1.f;
  float* o = a.out + (size_t)chunk * a.n_mels * a.width;
  const int total = a.n_mels * a.width;
  for (int i = tid; i < total; i += LM_THREADS) {
    float v = log10f(mel[i] / inv_scale + a.log_eps);
    if (a.do_clamp) v = (v < a.clamp_min) ? a.clamp_min : v;   // torch.clamp keeps NaN (silent chunk: 0/0)
    o[i] = v;
  }
}

// ===========================================================================
// Fast path for n_fft = 800 (GTZAN, AUDIO_PARAMS['gtzan']).  One workgroup of 12 waves per chunk,
// three frames per wave per round (36 frames per round).
//   pass A: lane (frame, n2) loads z[20 n1 + n2] = x[2n] w[2n] + i x[2n+1] w[2n+1] (n1 < 20),
//           DFT20 over n1 in registers, twiddle W_400^{n2 k1};
//   transpose through a per-frame 420-float LDS slab, real and imaginary parts in turn (half
//           the LDS of a complex slab, so 12 waves fit beside the [n_mels][width + 1] mel tile);
//   pass B: lane (frame, k1) DFT20 over n2 -> Z[k1 + 20 k2];
//   split:  Z[400 - k] from the partner lane (ds_bpermute), X[k] = (A + V_k B) / 2 with
//           A = Z_k + conj Z_{M-k}, B = Z_k - conj Z_{M-k}, V_k = -i W_800^k;
//   mel:    |X| into the wave's own slabs, lanes over (mel, frame) pairs with consecutive mels
//           (similar band widths) in one pass; weights transposed [j][m] in LDS.
// Every wave runs its rounds independently (no workgroup barrier before the peak), so the waves
// drift apart and hide each other's latency.  STFT, filterbank and |.| are homogeneous, so the
// chunk's peak division is applied to the mel energies at the end.  Measured (64 songs x 8 chunks):
// 0.181 ms (round 2: 8 waves at 224 VGPRs, per-lane divergent mel loop with weights contiguous)
// -> 0.122-0.127 ms.  LDS-bound (PMC: LDS active ~55 % of the kernel, VALU ~40 %).
// ===========================================================================
typedef float v2f __attribute__((ext_vector_type(2)));
// 12 waves (3 per SIMD; the LDS footprint holds one block per CU).  110 VGPRs since lanes 60-63
// duplicate lanes 0-3 (with active-lane branches: ~156 VGPRs, 0.124 ms -> 0.119 ms without); at 16
// waves the tables + mel tile exceed 160 KB of LDS
#ifndef LF_SPLIT_GROUP
#define LF_SPLIT_GROUP 5
#endif
#ifndef LF_MEL_UNROLL
#define LF_MEL_UNROLL 4
#endif
#ifndef LF_WIN_GROUP
#define LF_WIN_GROUP 4
#endif
// LF_PROFILE builds (scripts/logmel_phases.py only): per-wave clock cycles of each phase
#ifdef LF_PROFILE
__device__ unsigned long long lf_prof_buf[4096 * 12 * 8];
#define LF_T(i)                                                    \
  do {                                                             \
    __builtin_amdgcn_sched_barrier(0);                             \
    const unsigned long long t_ = __builtin_readcyclecounter();    \
    lf_acc[i] += t_ - lf_t;                                        \
    lf_t = t_;                                                     \
    __builtin_amdgcn_sched_barrier(0);                             \
  } while (0)
#else
#define LF_T(i) do {} while (0)
#endif
constexpr int LF_M = 400, LF_R = 20, LF_FPW = 3, LF_WAVES = 8, LF_THREADS = LF_WAVES * 64;
constexpr int LF_FPR = LF_WAVES * LF_FPW;   // frames per round
constexpr int LF_RS = 21;          // transpose row stride: 21 * q distinct mod 32 for q < 20
constexpr int LF_FS = 420;         // frame slab (== 4 mod 32: the three frames' pass-B reads are conflict-free)
// per-wave LDS: the 3 frames' slabs + a scratch slab for lanes 60-63 (LF_FPW + 1 slabs)
constexpr int LF_WB = (LF_FPW + 1) * LF_FS;
constexpr int LF_NBT = 16;         // band positions held transposed (wider bands read the rest from bw)
// magnitude row of frame f at slab offset LF_MOFF(f) (0, 11, 5): with the transposed weights and the
// padded mel tile, the mel stage's LDS accesses run at ~1.6 cycles per group instead of ~3
__device__ __forceinline__ int lf_moff(int f) { return f == 0 ? 0 : (f == 1 ? 11 : 5); }

// b (complex) from LDS tables: a * b
__device__ __forceinline__ cf cmulv(cf a, cf b) { return {fmaf(a.x, b.x, -(a.y * b.y)), fmaf(a.x, b.y, a.y * b.x)}; }

// 20-point DFT on float2 vectors (v_pk_{add,mul,fma}_f32: fewer VALU instructions than scalar
// complex code, which measured 2-3 % slower)
__device__ __forceinline__ v2f vfma(v2f a, v2f b, v2f c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ v2f vsplat(float s) { return (v2f){s, s}; }
__device__ __forceinline__ v2f vcmul(v2f a, v2f b) { return vfma(vsplat(a.y), (v2f){-b.y, b.x}, vsplat(a.x) * b); }
__device__ __forceinline__ v2f vnegi(v2f a) { return (v2f){a.y, -a.x}; }   // -i a
__device__ __forceinline__ void vbfly4(v2f& a0, v2f& a1, v2f& a2, v2f& a3) {
  const v2f t0 = a0 + a2, t1 = a0 - a2, t2 = a1 + a3, t3 = vnegi(a1 - a3);
  a0 = t0 + t2;
  a2 = t0 - t2;
  a1 = t1 + t3;
  a3 = t1 - t3;
}
__device__ __forceinline__ void vbfly5(v2f& a0, v2f& a1, v2f& a2, v2f& a3, v2f& a4) {
  const float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;
  const float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;
  const v2f b1 = a1 + a4, b2 = a2 + a3, d1 = a1 - a4, d2 = a2 - a3;
  const v2f r1 = vfma(vsplat(c2), b2, vfma(vsplat(c1), b1, a0));
  const v2f r2 = vfma(vsplat(c1), b2, vfma(vsplat(c2), b1, a0));
  const v2f q1 = vnegi(vfma(vsplat(s2), d2, vsplat(s1) * d1));
  const v2f q2 = vnegi(vfma(vsplat(-s1), d2, vsplat(s2) * d1));
  a0 = a0 + (b1 + b2);
  a1 = r1 + q1;
  a4 = r1 - q1;
  a2 = r2 + q2;
  a3 = r2 - q2;
}
// forward 20-point DFT in place, natural order in and out (n = 5 a + b, k = c + 4 d)
__device__ __forceinline__ void dft20(cf (&vc)[20]) {
  const v2f W[13] = {{1.0f, 0.0f},
                     {9.51056516295153531e-01f, -3.09016994374947396e-01f},
                     {8.09016994374947451e-01f, -5.87785252292473137e-01f},
                     {5.87785252292473137e-01f, -8.09016994374947451e-01f},
                     {3.09016994374947451e-01f, -9.51056516295153531e-01f},
                     {0.0f, -1.0f},
                     {-3.09016994374947340e-01f, -9.51056516295153642e-01f},
                     {-5.87785252292473026e-01f, -8.09016994374947451e-01f},
                     {-8.09016994374947340e-01f, -5.87785252292473248e-01f},
                     {-9.51056516295153531e-01f, -3.09016994374947507e-01f},
                     {-1.0f, 0.0f},
                     {-9.51056516295153753e-01f, 3.09016994374946896e-01f},
                     {-8.09016994374947562e-01f, 5.87785252292473026e-01f}};
  v2f v[20];
#pragma unroll
  for (int i = 0; i < 20; ++i) v[i] = (v2f){vc[i].x, vc[i].y};
#pragma unroll
  for (int b = 0; b < 5; ++b) {
    vbfly4(v[b], v[5 + b], v[10 + b], v[15 + b]);
#pragma unroll
    for (int c = 1; c < 4; ++c)
      if (b > 0) v[5 * c + b] = vcmul(v[5 * c + b], W[b * c]);
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    vbfly5(v[5 * c], v[5 * c + 1], v[5 * c + 2], v[5 * c + 3], v[5 * c + 4]);
#pragma unroll
    for (int d = 0; d < 5; ++d) vc[c + 4 * d] = {v[5 * c + d].x, v[5 * c + d].y};
  }
}

__global__ __launch_bounds__(LF_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void logmel800_kernel(LogmelArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  const int chunk = blockIdx.x;
#ifdef LF_PROFILE
  unsigned long long lf_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, lf_t = __builtin_readcyclecounter();
#endif
  const float* x = a.wav + (int64_t)(chunk / a.chunks_per_song) * a.song_stride +
                   (int64_t)(chunk % a.chunks_per_song) * a.chunk_hop;
  cf* tw = reinterpret_cast<cf*>(sm + a.o_tw);      // [k1][n2] = W_400^{n2 k1}
  cf* vtw = reinterpret_cast<cf*>(sm + a.o_ptw);    // V_k = -i W_800^k, k <= 400
  const float2* win2 = reinterpret_cast<const float2*>(sm + a.o_win);   // window pairs (w[2n], w[2n+1])
  int* blo = reinterpret_cast<int*>(sm + a.o_blo);
  int* bn = reinterpret_cast<int*>(sm + a.o_bn);
  int* boff = reinterpret_cast<int*>(sm + a.o_boff);
  float* bw = sm + a.o_bw;
  float* bwt = sm + a.o_bwt;                          // [j][m] at row stride n_mels + 1
  float* buf = sm + a.o_fft;                          // [16 waves][3 frames][420]: transposes, then |X|
  float* red = sm + a.o_red;

  LF_T(7);
  for (int j = tid; j < LF_M; j += LF_THREADS) {
    double s, c;
    const int e = ((j / LF_R) * (j % LF_R)) % LF_M;
    sincospi(2.0 * (double)e / (double)LF_M, &s, &c);
    tw[j] = {(float)c, (float)-s};
  }
  for (int k = tid; k <= LF_M; k += LF_THREADS) {
    double s, c;
    sincospi((double)k / (double)LF_M, &s, &c);      // W_800^k = (c, -s);  -i W = (-s, -c)
    vtw[k] = {(float)-s, (float)-c};
  }
  for (int i = tid; i < 800; i += LF_THREADS) sm[a.o_win + i] = a.window[i];
  for (int m = tid; m < a.n_mels; m += LF_THREADS) {
    blo[m] = a.band_lo[m];
    bn[m] = a.band_n[m];
    boff[m] = a.band_off[m];
  }
  for (int i = tid; i < a.nnz; i += LF_THREADS) bw[i] = a.band_w[i];
  for (int i = tid; i < LF_NBT * a.n_mels; i += LF_THREADS) {
    const int j = i / a.n_mels, m = i % a.n_mels;
    bwt[j * (a.n_mels + 1) + m] = (j < a.band_n[m]) ? a.band_w[a.band_off[m] + j] : 0.f;
  }
  __syncthreads();
  float* o = a.out + (size_t)chunk * a.n_mels * a.width;
  LF_T(0);

  // frame slot in the wave and n2 (pass A) / k1 (pass B).
  // lanes 60-63 run a 4th frame slot (q = 0-3) through their own scratch slab: no active-lane
  // branches, and at slab offset 3 * 420 = 12 (mod 32) their transpose reads share no bank with
  // frames 1 and 2 (as duplicates of lanes 0-3 they conflicted with lanes 32-35 on every read)
  const int fl = lane / LF_R, q = lane % LF_R;
  const int partner = fl * LF_R + (q == 0 ? 0 : LF_R - q);
  // float2 sample loads when every frame start is 8-byte aligned (even hop and an aligned chunk)
  const bool vec_ok = (a.hop & 1) == 0 && ((((uintptr_t)x) & 7) == 0);
  float* B = buf + w * LF_WB + fl * LF_FS;
  float pk = 0.f;
  for (int tb = 0; tb < a.width; tb += LF_FPR) {
    const int nfr = min(LF_FPR, a.width - tb);
    const int s = LF_FPW * w + fl;                    // frame slot in the round
    const bool fok = s < nfr;
    cf y[20];
    // ---- pass A ----
    {
      const int base = (a.frame0 + tb + (fok ? s : 0)) * a.hop - 400;
      const bool interior = base >= 0 && base + 800 <= a.L;
      if (__all(interior)) {
        if (vec_ok) {
          const float2* xp = reinterpret_cast<const float2*>(x + base) + q;
          float2 xv[LF_R];
#pragma unroll
          for (int n1 = 0; n1 < LF_R; ++n1) xv[n1] = xp[LF_R * n1];
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int n1 = 0; n1 < LF_R; ++n1) {
            pk = fmaxf(pk, fmaxf(fabsf(xv[n1].x), fabsf(xv[n1].y)));
            { const float2 wv = win2[LF_R * n1 + q]; y[n1] = {xv[n1].x * wv.x, xv[n1].y * wv.y}; }
            // window reads in groups of 4 (hoisting all 20 next to the 20 sample loads spills)
            if (n1 % LF_WIN_GROUP == LF_WIN_GROUP - 1) __builtin_amdgcn_sched_barrier(0);
          }
        } else {
          const float* xp = x + base + 2 * q;
#pragma unroll
          for (int n1 = 0; n1 < LF_R; ++n1) {
            const float x0 = xp[40 * n1], x1 = xp[40 * n1 + 1];
            pk = fmaxf(pk, fmaxf(fabsf(x0), fabsf(x1)));
            { const float2 wv = win2[LF_R * n1 + q]; y[n1] = {x0 * wv.x, x1 * wv.y}; }
          }
        }
      } else {
#pragma unroll
        for (int n1 = 0; n1 < LF_R; ++n1) {
          const int s0 = 40 * n1 + 2 * q;
          int j0 = base + s0, j1 = base + s0 + 1;
          j0 = j0 < 0 ? -j0 : j0;                        // reflect (torch pad_mode="reflect")
          j0 = j0 >= a.L ? 2 * (a.L - 1) - j0 : j0;
          j1 = j1 < 0 ? -j1 : j1;
          j1 = j1 >= a.L ? 2 * (a.L - 1) - j1 : j1;
          const float x0 = x[j0], x1 = x[j1];
          pk = fmaxf(pk, fmaxf(fabsf(x0), fabsf(x1)));
          { const float2 wv = win2[LF_R * n1 + q]; y[n1] = {x0 * wv.x, x1 * wv.y}; }
        }
      }
      LF_T(1);
      dft20(y);
#pragma unroll
      for (int k1 = 1; k1 < LF_R; ++k1) y[k1] = cmulv(y[k1], tw[k1 * LF_R + q]);
    }
    LF_T(2);
    // ---- transpose (real parts, then imaginary parts) ----
    cf v[20];
#pragma unroll
    for (int k1 = 0; k1 < LF_R; ++k1) B[k1 * LF_RS + q] = y[k1].x;
    wave_lds_sync();
#pragma unroll
    for (int n2 = 0; n2 < LF_R; ++n2) v[n2].x = B[q * LF_RS + n2];
    wave_lds_sync();
#pragma unroll
    for (int k1 = 0; k1 < LF_R; ++k1) B[k1 * LF_RS + q] = y[k1].y;
    wave_lds_sync();
#pragma unroll
    for (int n2 = 0; n2 < LF_R; ++n2) v[n2].y = B[q * LF_RS + n2];
    LF_T(3);
    // ---- pass B: Z[q + 20 k2] = v[k2] ----
    dft20(v);
    LF_T(4);
    // ---- real-input split + |X| straight into the frame's slab (its transpose reads are done:
    //      LDS ops of one wave stay in order) ----
#pragma unroll
    for (int k2 = 0; k2 < LF_R; ++k2) {
      const cf zp = {__shfl(v[LF_R - 1 - k2].x, partner, 64), __shfl(v[LF_R - 1 - k2].y, partner, 64)};
      const cf zr = (q == 0) ? v[(LF_R - k2) % LF_R] : zp;
      const cf zk = v[k2];
      const cf A = {zk.x + zr.x, zk.y - zr.y};
      const cf Bv = {zk.x - zr.x, zk.y + zr.y};
      const cf X2 = cadd(cmulv(Bv, vtw[q + LF_R * k2]), A);
      // v_sqrt_f32 (1 ulp; the correctly rounded sqrtf expands to ~10 instructions)
      B[lf_moff(fl) + q + LF_R * k2] = 0.5f * __builtin_amdgcn_sqrtf(X2.x * X2.x + X2.y * X2.y);
      // groups of 5 bins: the scheduler would otherwise hoist all 40 partner shuffles (and the V
      // reads) to the top and spill
      if (k2 % LF_SPLIT_GROUP == LF_SPLIT_GROUP - 1) __builtin_amdgcn_sched_barrier(0);
    }
    if (q == 0) B[lf_moff(fl) + LF_M] = fabsf(v[0].x - v[0].y);   // X[400] = Re Z0 - Im Z0
    wave_lds_sync();
    LF_T(5);
    // ---- mel filters: lane pair p = (mel p / 3, frame p % 3), consecutive mels (similar band
    //      widths) in one pass ----
    for (int p0 = 0; p0 < LF_FPW * a.n_mels; p0 += 64) {
      const int p = p0 + lane;
      const int m = p / LF_FPW, f = p % LF_FPW;
      const int t = tb + LF_FPW * w + f;
      const bool ok = p < LF_FPW * a.n_mels && t < a.width;
      const int mc = ok ? m : 0;
      const int lo = blo[mc], nb = ok ? bn[mc] : 0;
      const float* wm = bw + boff[mc];
      const float* mp = buf + w * LF_WB + f * LF_FS + lf_moff(f) + lo;
      const float* wt = bwt + mc;
      // the same sequential fma chain, its LDS reads issued LF_MEL_UNROLL at a time (past the
      // band: weight 0 and magnitude 0, acc + 0 * 0 == acc for the non-negative sums here)
      float acc = 0.f;
      for (int j0 = 0; j0 < nb; j0 += LF_MEL_UNROLL) {
        float wv[LF_MEL_UNROLL], mv[LF_MEL_UNROLL];
#pragma unroll
        for (int u = 0; u < LF_MEL_UNROLL; ++u) {
          const int j = j0 + u;
          const bool jok = j < nb;
          wv[u] = jok ? (j < LF_NBT ? wt[j * (a.n_mels + 1)] : wm[j]) : 0.f;
          mv[u] = jok ? mp[j] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < LF_MEL_UNROLL; ++u) acc = fmaf(wv[u], mv[u], acc);
      }
      if (ok) o[m * a.width + t] = acc;               // linear mel; log + peak scale below
    }
    wave_lds_sync();                                   // magnitudes consumed before the next round's transposes
    LF_T(6);
  }
  {
    const int c0 = max(0, a.frame0 * a.hop - 400);
    const int c1 = min(a.L, (a.frame0 + a.width - 1) * a.hop + 400);
    for (int i = tid; i < c0; i += LF_THREADS) pk = fmaxf(pk, fabsf(x[i]));
    for (int i = c1 + tid; i < a.L; i += LF_THREADS) pk = fmaxf(pk, fabsf(x[i]));
  }
  for (int off = 32; off > 0; off >>= 1) pk = fmaxf(pk, shfl_xor(pk, off));
  if (lane == 0) red[w] = pk;
  __syncthreads();   // the block's linear mel visible to all its waves (stores write through the CU's L1)
  float peak = red[0];
  for (int i = 1; i < LF_WAVES; ++i) peak = fmaxf(peak, red[i]);
  LF_T(7);
  // in place over the block's own output (just written, L2-resident): mel / peak as
  // mel * (1 / peak) (a power-of-two input scaling still cancels exactly) and log10 as
  // v_log_f32 * log10(2): 1-2 ulp instead of the ~40-instruction divide + log10f
  const float rscale = a.peak_norm ? 1.f / peak : 1.f;
  const int total = a.n_mels * a.width;
  auto fin = [&](float v) {
    float vv = __builtin_amdgcn_logf(fmaf(v, rscale, a.log_eps)) * 0.30102999566398120f;
    return a.do_clamp ? ((vv < a.clamp_min) ? a.clamp_min : vv) : vv;
  };
  if ((((uintptr_t)o) & 15) == 0 && (total & 3) == 0) {
    float4* o4 = reinterpret_cast<float4*>(o);
    constexpr int EU = 8;
    for (int i0 = 0; i0 < total / 4; i0 += EU * LF_THREADS) {
      float4 v[EU];
#pragma unroll
      for (int u = 0; u < EU; ++u) {
        const int i = i0 + u * LF_THREADS + tid;
        if (i < total / 4) v[u] = o4[i];
      }
#pragma unroll
      for (int u = 0; u < EU; ++u) {
        const int i = i0 + u * LF_THREADS + tid;
        if (i < total / 4) o4[i] = make_float4(fin(v[u].x), fin(v[u].y), fin(v[u].z), fin(v[u].w));
      }
    }
  } else {
    for (int i = tid; i < total; i += LF_THREADS) o[i] = fin(o[i]);
  }
#ifdef LF_PROFILE
  if (chunk < 4096) lf_prof_buf[((size_t)chunk * LF_WAVES + w) * 8 + (lane & 7)] = lf_acc[lane & 7];
#endif
}

int factor_radices(int M, int* r) {
  int n = 0;
  while (M % 4 == 0 && n < LM_MAX_STAGES) { r[n++] = 4; M /= 4; }
  while (M % 2 == 0 && n < LM_MAX_STAGES) { r[n++] = 2; M /= 2; }
  while (M % 3 == 0 && n < LM_MAX_STAGES) { r[n++] = 3; M /= 3; }
  while (M % 5 == 0 && n < LM_MAX_STAGES) { r[n++] = 5; M /= 5; }
  return M == 1 ? n : -1;
}

}  // namespace

#ifdef LF_PROFILE
extern "C" int drsa_amd_logmel_prof(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(lf_prof_buf), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -1;
}
#endif
extern "C" int drsa_amd_logmel_smem_bytes(int n_fft, int hop, int n_mels, int width, int band_nnz) {
  const int M = n_fft / 2;
  int off = 0;
  auto take = [&](int n) { int o = off; off += (n + 3) & ~3; return o; };
  take(2 * M);
  take(2 * (M + 1));
  take(n_fft);
  take(n_mels);
  take(n_mels);
  take(n_mels);
  take(band_nnz);
  take((LM_WAVES - 1) * hop + n_fft);
  take(LM_WAVES * 4 * M);
  take(n_mels * width);
  take(LM_WAVES);
  return off * 4;
}

extern "C" int drsa_amd_logmel(const float* wav, int64_t n_songs, int64_t song_stride, int chunks_per_song,
                               int64_t chunk_hop, int chunk_len, int n_fft, int hop, int n_mels, int width,
                               int frame0, const float* window, const int* band_lo, const int* band_n,
                               const int* band_off, const float* band_w, int band_nnz, int peak_norm, int clamp,
                               float clamp_min, float log_eps, float* out, void* stream) {
  DRSA_REQUIRE(wav && window && band_lo && band_n && band_off && band_w && out, "logmel: null pointer");
  DRSA_REQUIRE(n_songs >= 0 && chunks_per_song >= 1, "logmel: bad chunk counts");
  DRSA_REQUIRE(n_fft >= 8 && n_fft % 2 == 0, "logmel: n_fft must be even (got %d)", n_fft);
  DRSA_REQUIRE(hop >= 1 && n_mels >= 1 && width >= 1 && frame0 >= 0, "logmel: bad hop/n_mels/width/frame0");
  DRSA_REQUIRE(chunk_len > n_fft / 2, "logmel: reflect padding needs chunk_len > n_fft/2");
  DRSA_REQUIRE(frame0 + width <= 1 + chunk_len / hop, "logmel: frames %d..%d exceed the %d STFT frames", frame0,
               frame0 + width - 1, 1 + chunk_len / hop);
  DRSA_REQUIRE(band_nnz >= 0, "logmel: band_nnz < 0");
  LogmelArgs a{};
  a.n_stages = factor_radices(n_fft / 2, a.radix);
  DRSA_REQUIRE(a.n_stages > 0, "logmel: n_fft/2 = %d must factor into 2, 3, 5", n_fft / 2);
  if (n_songs == 0) return DRSA_OK;
  const int64_t n_chunks = n_songs * chunks_per_song;
  DRSA_REQUIRE(n_chunks < (1 << 30), "logmel: too many chunks");
  a.wav = wav;
  a.song_stride = song_stride;
  a.chunk_hop = chunk_hop;
  a.chunks_per_song = chunks_per_song;
  a.n_chunks = (int)n_chunks;
  a.L = chunk_len;
  a.nfft = n_fft;
  a.hop = hop;
  a.n_mels = n_mels;
  a.width = width;
  a.frame0 = frame0;
  a.window = window;
  a.band_lo = band_lo;
  a.band_n = band_n;
  a.band_off = band_off;
  a.band_w = band_w;
  a.nnz = band_nnz;
  a.peak_norm = peak_norm;
  a.do_clamp = clamp;
  a.clamp_min = clamp_min;
  a.log_eps = log_eps;
  a.out = out;
  const int M = n_fft / 2;
  auto carve = [&](bool fast) {
    int off = 0;
    auto take = [&](int n) { int o = off; off += (n + 3) & ~3; return o; };
    a.o_tw = take(2 * M);
    a.o_ptw = take(2 * (M + 1));
    a.o_win = take(n_fft);
    a.o_blo = take(n_mels);
    a.o_bn = take(n_mels);
    a.o_boff = take(n_mels);
    a.o_bw = take(band_nnz);
    a.o_samp = take(fast ? 0 : (LM_WAVES - 1) * hop + n_fft);
    a.o_fft = take(fast ? LF_WAVES * LF_WB : LM_WAVES * 4 * M);
    a.o_mel = take(fast ? 0 : n_mels * width);
    a.o_bwt = take(fast ? LF_NBT * (n_mels + 1) : 0);
    a.o_red = take(fast ? LF_WAVES : LM_WAVES);
    a.smem_floats = off;
    return (size_t)off * 4;
  };
  // the 16-wave n_fft = 800 kernel when its tables + mel tile fit in LDS, else the generic kernel
  bool fast = n_fft == 800 && carve(true) <= 160 * 1024;
  const size_t smem = carve(fast);
  DRSA_REQUIRE(smem <= 160 * 1024, "logmel: LDS footprint %zu B exceeds 160 KB (n_mels*width too large)", smem);
  const void* fn = fast ? (const void*)logmel800_kernel : (const void*)logmel_kernel;
  DRSA_SMEM(fn, smem);
  if (fast)
    hipLaunchKernelGGL(logmel800_kernel, dim3((unsigned)n_chunks), dim3(LF_THREADS), smem, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(logmel_kernel, dim3((unsigned)n_chunks), dim3(LM_THREADS), smem, (hipStream_t)stream, a);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}
