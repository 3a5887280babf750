// Encoder GEMM check + A/B: the launcher's choice (launch_gemm_tiles(..., 256): k_gemm_256
// from 256 tiles, else k_gemm_tile with 128 x 64 tiles below 256 tiles) against
// k_gemm_tile with 128 x 128 tiles (..., 129) on the large-v3 encoder shapes, uniform random [-1, 1) fp16
// operands (cdna_hip_programming.md §5.4 rule 25: never zero-filled).
//   * correctness: every output of both kernels against each other (max |diff| relative to
//     the output scale) and 4096 sampled outputs against an fp64 host dot product;
//   * timing: interleaved rounds in one process (rule 24), median of the per-round
//     averages, TFLOP/s = 2 M N K / time.
//   make -C whisper.coreml_amd tools/gemm_bench && ./whisper.coreml_amd/tools/gemm_bench [windows]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "wh_gemm.h"

using namespace wh;

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

struct Shape {
  const char* name;
  int M, N, K;
  int group_rows, group_pad;  // X rows in groups of group_rows with group_pad pad rows between
};

static double host_dot(const std::vector<half_t>& X, const std::vector<half_t>& W, const Shape& s, int ldx, int m,
                       int n) {
  const int gi = m / s.group_rows, ri = m % s.group_rows;
  const size_t xo = ((size_t)gi * (s.group_rows + s.group_pad) + ri) * ldx;
  double acc = 0;
  for (int k = 0; k < s.K; ++k) acc += (double)(float)X[xo + k] * (double)(float)W[(size_t)n * s.K + k];
  return acc;
}

int main(int argc, char** argv) {
  const int nwin = argc > 1 ? atoi(argv[1]) : 20;
  const int rounds = argc > 2 ? atoi(argv[2]) : 7;
  // the two launch_gemm_tiles selections compared (A, B): default 129 (k_gemm_tile 128x128)
  // against 256 (the launcher); 256 257 compares the 16x16x32 and 32x32x16 MFMA forms
  const int selA = argc > 3 ? atoi(argv[3]) : 129, selB = argc > 4 ? atoi(argv[4]) : 256;
  const int M = 1500 * nwin;
  const Shape shapes[] = {
      {"qkv", M, 3840, 1280, 1500, 0}, {"out", M, 1280, 1280, 1500, 0}, {"fc1", M, 5120, 1280, 1500, 0},
      {"fc2", M, 1280, 5120, 1500, 0}, {"grouped", M, 1280, 1280, 1500, 2},
      {"ragged", 1000 + 37, 1280, 1280, 1 << 30, 0}, {"one-window", 1500, 5120, 1280, 1500, 0},
      {"1w-out", 1500, 1280, 1280, 1500, 0}, {"1w-fc2", 1500, 1280, 5120, 1500, 0},
  };
  std::mt19937 rng(1234);
  std::uniform_real_distribution<float> uni(-1.f, 1.f);
  int fails = 0;
  for (const Shape& s : shapes) {
    const int ldx = s.K;
    const int ngroups = (s.M + s.group_rows - 1) / std::min(s.group_rows, s.M);
    const size_t xrows = s.group_rows >= s.M ? (size_t)s.M : (size_t)ngroups * (s.group_rows + s.group_pad);
    std::vector<half_t> hX(xrows * ldx), hW((size_t)s.N * s.K);
    std::vector<float> hb(s.N);
    for (auto& v : hX) v = (half_t)uni(rng);
    for (auto& v : hW) v = (half_t)uni(rng);
    for (auto& v : hb) v = uni(rng);
    half_t *X, *W, *Y0, *Y1;
    float* bias;
    CK(hipMalloc(&X, hX.size() * 2));
    CK(hipMalloc(&W, hW.size() * 2));
    CK(hipMalloc(&Y0, (size_t)s.M * s.N * 2));
    CK(hipMalloc(&Y1, (size_t)s.M * s.N * 2));
    CK(hipMalloc(&bias, s.N * 4));
    CK(hipMemcpy(X, hX.data(), hX.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(W, hW.data(), hW.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(bias, hb.data(), s.N * 4, hipMemcpyHostToDevice));
    GemmArgs a;
    a.X = X;
    a.W = W;
    a.bias = bias;
    a.M = s.M;
    a.N = s.N;
    a.K = s.K;
    a.ldx = ldx;
    a.x_group_rows = std::min(s.group_rows, s.M);
    a.x_group_stride = (int64_t)(s.group_rows + s.group_pad) * ldx;
    a.ldo = s.N;
    a.out_group_stride = (int64_t)a.x_group_rows * s.N;
    GemmArgs a0 = a, a1 = a;
    a0.out = Y0;
    a1.out = Y1;
    CK(hipMemset(Y0, 0, (size_t)s.M * s.N * 2));
    CK(hipMemset(Y1, 0, (size_t)s.M * s.N * 2));
    if (launch_gemm_tiles<half_t>(a0, EPI_STORE, selA, 0) || launch_gemm_tiles<half_t>(a1, EPI_STORE, selB, 0)) {
      printf("%s: launch refused\n", s.name);
      return 1;
    }
    CK(hipDeviceSynchronize());
    std::vector<half_t> h0((size_t)s.M * s.N), h1((size_t)s.M * s.N);
    CK(hipMemcpy(h0.data(), Y0, h0.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h1.data(), Y1, h1.size() * 2, hipMemcpyDeviceToHost));
    double dmax = 0, ymax = 0;
    for (size_t i = 0; i < h0.size(); ++i) {
      dmax = std::max(dmax, (double)std::fabs((float)h0[i] - (float)h1[i]));
      ymax = std::max(ymax, (double)std::fabs((float)h1[i]));
    }
    double emax = 0;
    std::uniform_int_distribution<int> rm(0, s.M - 1), rn(0, s.N - 1);
    for (int t = 0; t < 4096; ++t) {
      const int m = t < 64 ? s.M - 1 - t : rm(rng), n = rn(rng);
      const double ref = host_dot(hX, hW, s, ldx, m, n) + hb[n];
      emax = std::max(emax, std::fabs(ref - (double)(float)h1[(size_t)m * s.N + n]) / ymax);
    }
    // fp16 output rounding of values up to ymax: 2^-11 relative
    const bool ok = dmax / ymax < 2e-3 && emax < 2e-3;
    fails += !ok;
    // timing: interleaved rounds, 10 launches each
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> t128, t256;
    for (int rd = 0; rd < rounds; ++rd) {
      for (int v = 0; v < 2; ++v) {
        const int tile = v ? selB : selA;
        GemmArgs& av = v ? a1 : a0;
        launch_gemm_tiles<half_t>(av, EPI_STORE, tile, 0);
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < 10; ++i) launch_gemm_tiles<half_t>(av, EPI_STORE, tile, 0);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        (v ? t256 : t128).push_back(ms / 10);
      }
    }
    std::sort(t128.begin(), t128.end());
    std::sort(t256.begin(), t256.end());
    const double fl = 2.0 * s.M * s.N * s.K;
    const float m128 = t128[t128.size() / 2], m256 = t256[t256.size() / 2];
    printf("%-10s M=%6d N=%5d K=%5d  %d: %.4f ms %6.1f TF | %d: %.4f ms %6.1f TF (min %.4f)  x%.2f | "
           "max|B-A|/max|y| %.2e, max|B-fp64|/max|y| %.2e %s\n",
           s.name, s.M, s.N, s.K, selA, m128, fl / m128 / 1e9, selB, m256, fl / m256 / 1e9, t256[0], m128 / m256, dmax / ymax,
           emax, ok ? "ok" : "FAIL");
    fflush(stdout);
    CK(hipFree(X));
    CK(hipFree(W));
    CK(hipFree(Y0));
    CK(hipFree(Y1));
    CK(hipFree(bias));
  }
  printf("%s\n", fails ? "FAILED" : "all shapes ok");
  return fails ? 1 : 0;
}
