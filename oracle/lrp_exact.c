/*
 * ORACLE — test infrastructure only.  Pinned-order fp32 primitives for oracle/lrp_ref.py's
 * mode="exact".  Each output element is ONE sequential fp32 fma chain in a documented order,
 * which is the order the HIP kernels accumulate in (f32 MFMA = k-ordered fma chain):
 *
 *   conv2d_exact            out[co][y][x] = (chain over ci, ky, kx of x*w) + b         ('same', zero pad)
 *   conv_transpose_exact    out[ci][y][x] = chain over co, ky', kx' of g[co][y+ky'-1][x+kx'-1]
 *                                                         * w[co][ci][2-ky'][2-kx']
 *   linear_exact            out[m][n] = (chain over k of x[m][k] * W[n][k]) + b[n]
 *   matmul_exact            out[m][n] = chain over k of A[m][k] * B[k][n]
 *   (heatmap sums are numpy's own float32 sum, the reference's: oracle/lrp_ref.py plane_sum)
 *
 * The algorithm these feed (the LRP rules) is restated in oracle/lrp_ref.py; only the
 * summation order inside dot products is fixed here.  Compiled by oracle/Makefile with
 * -ffp-contract=off so every a*b+c is written explicitly as fmaf() or as two roundings.
 */
#include <math.h>
#include <stdint.h>
#include <stddef.h>

void conv2d_exact(const float* x, const float* w, const float* b, float* out, int B, int Cin, int Cout,
                  int H, int W) {
#pragma omp parallel for collapse(2) schedule(static)
  for (int bb = 0; bb < B; ++bb)
    for (int co = 0; co < Cout; ++co)
      for (int y = 0; y < H; ++y)
        for (int xx = 0; xx < W; ++xx) {
          float acc = 0.f;
          for (int ci = 0; ci < Cin; ++ci)
            for (int ky = 0; ky < 3; ++ky)
              for (int kx = 0; kx < 3; ++kx) {
                const int yy = y + ky - 1, xi = xx + kx - 1;
                const float v = (yy >= 0 && yy < H && xi >= 0 && xi < W)
                                    ? x[(((size_t)bb * Cin + ci) * H + yy) * W + xi] : 0.f;
                acc = fmaf(v, w[(((size_t)co * Cin + ci) * 3 + ky) * 3 + kx], acc);
              }
          out[(((size_t)bb * Cout + co) * H + y) * W + xx] = b ? acc + b[co] : acc;
        }
}

void conv_transpose_exact(const float* g, const float* w, float* out, int B, int Cout, int Cin, int H, int W) {
#pragma omp parallel for collapse(2) schedule(static)
  for (int bb = 0; bb < B; ++bb)
    for (int ci = 0; ci < Cin; ++ci)
      for (int y = 0; y < H; ++y)
        for (int xx = 0; xx < W; ++xx) {
          float acc = 0.f;
          for (int co = 0; co < Cout; ++co)
            for (int kyp = 0; kyp < 3; ++kyp)
              for (int kxp = 0; kxp < 3; ++kxp) {
                const int yy = y + kyp - 1, xi = xx + kxp - 1;
                const float v = (yy >= 0 && yy < H && xi >= 0 && xi < W)
                                    ? g[(((size_t)bb * Cout + co) * H + yy) * W + xi] : 0.f;
                acc = fmaf(v, w[(((size_t)co * Cin + ci) * 3 + (2 - kyp)) * 3 + (2 - kxp)], acc);
              }
          out[(((size_t)bb * Cin + ci) * H + y) * W + xx] = acc;
        }
}

void linear_exact(const float* x, const float* Wt, const float* b, float* out, int M, int N, int K) {
#pragma omp parallel for schedule(static)
  for (int m = 0; m < M; ++m)
    for (int n = 0; n < N; ++n) {
      float acc = 0.f;
      for (int k = 0; k < K; ++k) acc = fmaf(x[(size_t)m * K + k], Wt[(size_t)n * K + k], acc);
      out[(size_t)m * N + n] = b ? acc + b[n] : acc;
    }
}

void matmul_exact(const float* A, const float* Bm, float* out, int M, int N, int K) {
#pragma omp parallel for schedule(static)
  for (int m = 0; m < M; ++m)
    for (int n = 0; n < N; ++n) {
      float acc = 0.f;
      for (int k = 0; k < K; ++k) acc = fmaf(A[(size_t)m * K + k], Bm[(size_t)k * N + n], acc);
      out[(size_t)m * N + n] = acc;
    }
}
