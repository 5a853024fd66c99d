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
// Fast path for n_fft = 800 (GTZAN, AUDIO_PARAMS['gtzan']): the 400-point complex FFT of a
// frame as 20 x 20 (n = 20 n1 + n2, k = k1 + 20 k2), each 20-point DFT in registers (4 x 5).
// Three frames per wave, one lane per (frame, n2) in pass A and per (frame, k1) in pass B
// (60 of 64 lanes busy): two LDS hand-offs per frame instead of the generic kernel's
// Stockham stages.  Samples come straight from global memory (frames overlap 55 %, served by
// L1/L2); one workgroup per chunk keeps the peak division and the coalesced output rows.
// ===========================================================================
constexpr int LF_M = 400, LF_R = 20, LF_FPW = 3;   // complex points, radix, frames per wave
// T layout: pass-A rows k1 at stride LF_RS = 21 (pass-B lanes k1 read a row each: 42-bank
// stride, conflict-free); frames at LF_FS = 421 complex
constexpr int LF_RS = 21, LF_FS = 421;
#ifndef LF_UNROLL_MEL
#define LF_UNROLL_MEL 0
#endif
#ifndef LF_VEC_LOADS
#define LF_VEC_LOADS 0
#endif
constexpr int LF_MAXB = 20;                          // unrolled mel band width (wider: loop)

__device__ __constant__ cf kW20[13] = {
    {1.0f, 0.0f},
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

// forward 20-point DFT in place: v[n] -> v[k] (4 x 5: n = 5 n1 + n2, k = k1 + 4 k2)
__device__ __forceinline__ void dft20(cf* v) {
  cf y[4][5];
#pragma unroll
  for (int n2 = 0; n2 < 5; ++n2) {
    cf t[4] = {v[n2], v[5 + n2], v[10 + n2], v[15 + n2]};
    bfly4(t);
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) y[k1][n2] = (n2 * k1 == 0) ? t[k1] : cmul(t[k1], kW20[n2 * k1]);
  }
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    bfly5(y[k1]);
#pragma unroll
    for (int k2 = 0; k2 < 5; ++k2) v[k1 + 4 * k2] = y[k1][k2];
  }
}

__global__ __launch_bounds__(LM_THREADS) void logmel800_kernel(LogmelArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  const int chunk = blockIdx.x;
  const float* x = a.wav + (int64_t)(chunk / a.chunks_per_song) * a.song_stride +
                   (int64_t)(chunk % a.chunks_per_song) * a.chunk_hop;
  cf* tw = reinterpret_cast<cf*>(sm + a.o_tw);      // [k1][n2] = W_400^{n2 k1} (lanes n2 adjacent)
  cf* ptw = reinterpret_cast<cf*>(sm + a.o_ptw);    // W_800^k, k <= 400
  float* win = sm + a.o_win;
  int* blo = reinterpret_cast<int*>(sm + a.o_blo);
  int* bn = reinterpret_cast<int*>(sm + a.o_bn);
  int* boff = reinterpret_cast<int*>(sm + a.o_boff);
  float* bw = sm + a.o_bw;
  cf* T = reinterpret_cast<cf*>(sm + a.o_fft) + (size_t)w * LF_FPW * LF_FS;  // [3][LF_FS] per wave
  float* mel = sm + a.o_mel;
  float* red = sm + a.o_red;

  for (int j = tid; j < LF_M; j += LM_THREADS) {
    double s, c;
    const int e = ((j / LF_R) * (j % LF_R)) % LF_M;
    sincospi(2.0 * (double)e / (double)LF_M, &s, &c);
    tw[j] = {(float)c, (float)-s};
  }
  for (int k = tid; k <= LF_M; k += LM_THREADS) {
    double s, c;
    sincospi((double)k / (double)LF_M, &s, &c);
    ptw[k] = {(float)c, (float)-s};
  }
  for (int i = tid; i < 800; i += LM_THREADS) win[i] = a.window[i];
  for (int m = tid; m < a.n_mels; m += LM_THREADS) {
    blo[m] = a.band_lo[m];
    bn[m] = a.band_n[m];
    boff[m] = a.band_off[m];
  }
  for (int i = tid; i < a.nnz; i += LM_THREADS) bw[i] = a.band_w[i];
  __syncthreads();

  const int fl = lane / LF_R, q = lane % LF_R;       // frame slot in the wave, n2 / k1
  const bool lact = lane < LF_FPW * LF_R;
  float pk = 0.f;
  constexpr int FPR = LM_WAVES * LF_FPW;             // frames per workgroup round
  for (int tb = 0; tb < a.width; tb += FPR) {
    const int fi = tb + w * LF_FPW + fl;             // frame slot index in [0, width)
    const bool fok = lact && fi < a.width;
    cf v[LF_R];
    // ---- pass A: lane (frame, n2) loads z[20 n1 + n2] = x[2n] w[2n] + i x[2n+1] w[2n+1] ----
    {
      const int base = (a.frame0 + (fok ? fi : 0)) * a.hop - 400;
      if (LF_VEC_LOADS && base >= 0 && base + 800 <= a.L && ((base + (int)((uintptr_t)x >> 2)) & 1) == 0) {
        // interior frame, 8-byte aligned pairs: one float2 load per n1
        const float2* xp = reinterpret_cast<const float2*>(x + base) + q;
#pragma unroll
        for (int n1 = 0; n1 < LF_R; ++n1) {
          const float2 xv = xp[20 * n1];
          const int s0 = 40 * n1 + 2 * q;
          pk = fok ? fmaxf(pk, fmaxf(fabsf(xv.x), fabsf(xv.y))) : pk;
          v[n1] = {xv.x * win[s0], xv.y * win[s0 + 1]};
        }
      } else {
#pragma unroll
        for (int n1 = 0; n1 < LF_R; ++n1) {
          const int s0 = 40 * n1 + 2 * q;
          int j0 = base + s0, j1 = base + s0 + 1;
          j0 = j0 < 0 ? -j0 : j0;
          j0 = j0 >= a.L ? 2 * (a.L - 1) - j0 : j0;
          j1 = j1 < 0 ? -j1 : j1;
          j1 = j1 >= a.L ? 2 * (a.L - 1) - j1 : j1;
          const float x0 = x[j0], x1 = x[j1];
          pk = fok ? fmaxf(pk, fmaxf(fabsf(x0), fabsf(x1))) : pk;
          v[n1] = {x0 * win[s0], x1 * win[s0 + 1]};
        }
      }
      dft20(v);
      // twiddle W_400^{n2 k1}, store T[k1][n2]
#pragma unroll
      for (int k1 = 0; k1 < LF_R; ++k1) {
        const cf t = (k1 == 0) ? v[0] : cmul(v[k1], tw[k1 * LF_R + q]);
        if (lact) T[fl * LF_FS + k1 * LF_RS + q] = t;
      }
    }
    wave_lds_sync();
    // ---- pass B: lane (frame, k1) reads T[k1][n2], DFT over n2 -> Z[k1 + 20 k2] ----
    if (lact) {
#pragma unroll
      for (int n2 = 0; n2 < LF_R; ++n2) v[n2] = T[fl * LF_FS + q * LF_RS + n2];
    }
    dft20(v);
    wave_lds_sync();
    if (lact) {
#pragma unroll
      for (int k2 = 0; k2 < LF_R; ++k2) T[fl * LF_FS + q + LF_R * k2] = v[k2];
    }
    wave_lds_sync();
    // ---- real split + |X|: 3 x 401 bins over the wave; magnitudes held in registers until
    //      every lane has read its Z pairs, then written over T (as floats) ----
    constexpr int NB = LF_FPW * (LF_M + 1);
    constexpr int NIT = (NB + 63) / 64;
    float mg[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int i = lane + 64 * it;
      const int f = i / (LF_M + 1), k = i % (LF_M + 1);
      float m = 0.f;
      if (i < NB) {
        const cf* Z = T + f * LF_FS;
        const cf zk = Z[k == LF_M ? 0 : k];
        const cf zr = Z[k == 0 ? 0 : LF_M - k];
        const cf zc = {zr.x, -zr.y};
        const cf e = cscale(cadd(zk, zc), 0.5f);
        const cf d = csub(zk, zc);
        const cf o = {0.5f * d.y, -0.5f * d.x};
        const cf X = cadd(e, cmul(ptw[k], o));
        m = sqrtf(X.x * X.x + X.y * X.y);
      }
      mg[it] = m;
    }
    wave_lds_sync();
    float* magb = reinterpret_cast<float*>(T);      // [3][401] floats
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int i = lane + 64 * it;
      if (i < NB) magb[i] = mg[it];
    }
    wave_lds_sync();
    // ---- banded mel filters, lanes over (frame, mel) ----
    for (int i = lane; i < LF_FPW * a.n_mels; i += 64) {
      const int f = i / a.n_mels, m = i % a.n_mels;
      const int t = tb + w * LF_FPW + f;
      if (t < a.width) {
        const float* wm = bw + boff[m];
        const float* mgp = magb + f * (LF_M + 1) + blo[m];
        const int nb = bn[m];
        float acc = 0.f;
        if (LF_UNROLL_MEL && nb <= LF_MAXB) {
          // all band reads issued together (masked, clamped), then the ordered chain
          float wv[LF_MAXB], mv[LF_MAXB];
#pragma unroll
          for (int qq = 0; qq < LF_MAXB; ++qq) {
            const int qc = qq < nb ? qq : 0;
            wv[qq] = wm[qc];
            mv[qq] = mgp[qc];
          }
#pragma unroll
          for (int qq = 0; qq < LF_MAXB; ++qq)
            if (qq < nb) acc += wv[qq] * mv[qq];
        } else {
          for (int qq = 0; qq < nb; ++qq) acc += wm[qq] * mgp[qq];
        }
        mel[m * a.width + t] = acc;
      }
    }
    wave_lds_sync();
  }
  {
    const int c0 = max(0, a.frame0 * a.hop - 400);
    const int c1 = min(a.L, (a.frame0 + a.width - 1) * a.hop + 400);
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
    float vv = log10f(mel[i] / inv_scale + a.log_eps);
    if (a.do_clamp) vv = (vv < a.clamp_min) ? a.clamp_min : vv;
    o[i] = vv;
  }
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
  static const int no_fast = getenv("DRSA_AMD_LOGMEL_GENERIC") ? atoi(getenv("DRSA_AMD_LOGMEL_GENERIC")) : 0;
  const bool fast = n_fft == 800 && !no_fast;
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
  a.o_fft = take(fast ? LM_WAVES * LF_FPW * 2 * LF_FS : LM_WAVES * 4 * M);
  a.o_mel = take(n_mels * width);
  a.o_red = take(LM_WAVES);
  a.smem_floats = off;
  const size_t smem = (size_t)off * 4;
  DRSA_REQUIRE(smem <= 160 * 1024, "logmel: LDS footprint %zu B exceeds 160 KB (n_mels*width too large)", smem);
  const void* fn = fast ? (const void*)logmel800_kernel : (const void*)logmel_kernel;
  DRSA_SMEM(fn, smem);
  if (fast)
    hipLaunchKernelGGL(logmel800_kernel, dim3((unsigned)n_chunks), dim3(LM_THREADS), smem, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(logmel_kernel, dim3((unsigned)n_chunks), dim3(LM_THREADS), smem, (hipStream_t)stream, a);
  DRSA_LAUNCH_CHECK();
  return DRSA_OK;
}
