// Microbenchmark of the decoder step's vocabulary projection at decode batch sizes
// (launch_gemm EPI_F32_COLS, N = 51866, K = 1280, fp16): the average launch time over
// three weight copies (400 MB, so weights stream from HBM as in the step, not from the
// 256 MB Infinity Cache), for row counts that select k_vocab_small (<= 32) and
// k_vocab_2p (33..112); with and without the x_rows gather.
//   make -C whisper.coreml_amd tools/vocab_bench && ./whisper.coreml_amd/tools/vocab_bench [rows,...]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "wh_gemm.h"

using namespace wh;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

int main(int argc, char** argv) {
  std::vector<int> rows = {16, 32, 33, 48, 64, 80, 96, 100, 112};
  if (argc > 1) {
    rows.clear();
    for (char* t = strtok(argv[1], ","); t; t = strtok(nullptr, ",")) rows.push_back(atoi(t));
  }
  const int N = 51866, K = 1280, C = 3, iters = 30;
  const size_t wsz = (size_t)N * K;
  half_t* W;
  CK(hipMalloc(&W, wsz * C * sizeof(half_t)));
  CK(hipMemset(W, 0, wsz * C * sizeof(half_t)));
  half_t* X;
  CK(hipMalloc(&X, (size_t)128 * K * sizeof(half_t)));
  CK(hipMemset(X, 0, (size_t)128 * K * sizeof(half_t)));
  float* Y;
  CK(hipMalloc(&Y, (size_t)128 * N * sizeof(float)));
  int* xr;
  CK(hipMalloc(&xr, 128 * sizeof(int)));
  std::vector<int> h(128);
  for (int i = 0; i < 128; ++i) h[i] = 127 - i;
  CK(hipMemcpy(xr, h.data(), 128 * sizeof(int), hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int M : rows)
    for (int gather = 0; gather < 2; ++gather) {
      auto run = [&](int i) {
        GemmArgs a;
        a.X = X; a.W = W + (size_t)(i % C) * wsz; a.M = M; a.N = N; a.K = K; a.ldx = K;
        a.x_group_rows = M; a.out_f32 = Y; a.ldo = N;
        if (gather) a.x_rows = xr;
        return launch_gemm<half_t>(a, EPI_F32_COLS, st);
      };
      for (int i = 0; i < 6; ++i)
        if (run(i)) { printf("rows %d: launch_gemm failed\n", M); return 1; }
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < iters; ++i) run(i);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / iters;
      printf("rows %3d %s: %7.2f us per launch, %5.2f TB/s of weights\n", M, gather ? "x_rows" : "plain ", us,
             wsz * 2 / us / 1e6);
    }
  return 0;
}
