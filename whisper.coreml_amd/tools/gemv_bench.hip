// Microbenchmark of the decoder-step projection GEMVs (k_gemv_x / k_gemv_rows via
// launch_gemm) at decode batch sizes: for every (shape, rows, split-K, row-block)
// variant, the average launch time over 32 distinct weight copies (so weights stream
// from HBM as in a 32-layer step, not from the 256 MB Infinity Cache).
//   make -C whisper.coreml_amd tools/gemv_bench && ./whisper.coreml_amd/tools/gemv_bench [rows]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
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

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 100;
  const int n = 1280, L = 32, iters = 5;
  struct Shape { const char* name; int N, K; };
  const Shape shapes[] = {{"qkv", 3 * n, n}, {"out", n, n}, {"fc1", 4 * n, n}, {"fc2", n, 4 * n}};
  // weights: L copies of the largest (4n x n) matrix
  const size_t wsz = (size_t)4 * n * n;
  half_t* W;
  CK(hipMalloc(&W, wsz * L * sizeof(half_t)));
  CK(hipMemset(W, 0, wsz * L * sizeof(half_t)));
  half_t *X, *Y;
  CK(hipMalloc(&X, (size_t)M * 4 * n * sizeof(half_t)));
  CK(hipMemset(X, 0, (size_t)M * 4 * n * sizeof(half_t)));
  CK(hipMalloc(&Y, (size_t)M * 4 * n * sizeof(half_t)));
  float* part;
  CK(hipMalloc(&part, (size_t)16 * M * 4 * n * sizeof(float)));
  float* bias;
  CK(hipMalloc(&bias, 4 * n * sizeof(float)));
  CK(hipMemset(bias, 0, 4 * n * sizeof(float)));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  printf("rows=%d\n%-5s %5s %3s %3s %6s %9s %9s\n", M, "shape", "epi", "z", "mtb", "wgs", "us", "GB/s(W)");
  for (const auto& sh : shapes) {
    const int mts[] = {0, 4};
    for (int mtb : mts) {
      for (int z = 0; z <= 16; ++z) {
        // z == 0: direct store epilogue (bias [+gelu]) without split-K
        if (z > 0 && z != 1 && z != 2 && z != 3 && z != 4 && z != 5 && z != 6 && z != 8 && z != 10 && z != 12 &&
            z != 16)
          continue;
        GemmArgs g;
        g.M = M; g.N = sh.N; g.K = sh.K;
        g.ldx = sh.K; g.mt_block = mtb;
        int epi;
        if (z == 0) {
          epi = EPI_STORE_GELU; g.out = Y; g.ldo = sh.N; g.bias = bias;
        } else {
          epi = EPI_PARTIAL; g.out_f32 = part; g.ldo = sh.N; g.ksplit = z;
        }
        auto run = [&](int l) {
          g.X = X;
          g.W = W + (size_t)l * wsz;
          return launch_gemm<half_t>(g, epi, st);
        };
        if (run(0) != 0) continue;
        for (int l = 0; l < L; ++l) run(l);
        CK(hipEventRecord(a, st));
        for (int i = 0; i < iters; ++i)
          for (int l = 0; l < L; ++l) run(l);
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        const double us = ms * 1e3 / (iters * L);
        const int mt = (M + 15) / 16;
        const int rp = mtb ? (mtb < mt ? mtb : mt) : (mt >= 8 ? 8 : mt);
        const int wgs = (mt >= 3 ? (sh.N + 63) / 64 : (sh.N + 15) / 16) * ((M + 16 * rp - 1) / (16 * rp)) * (z ? z : 1);
        printf("%-5s %5s %3d %3d %6d %9.2f %9.1f\n", sh.name, z ? "part" : "gelu", z, mtb, wgs, us,
               (double)sh.N * sh.K * 2 / (us * 1e-6) / 1e9);
      }
    }
  }
  CK(hipGetLastError());
  return 0;
}
