// Microbenchmark of k_proj (wh_proj.h) variants at decode batch sizes against the
// split-K k_gemv_x + fixed-order reduce pair, per projection shape of a large-v3
// decoder layer.  Every timing averages over 32 distinct weight copies so weights
// stream from HBM as in a 32-layer step (not from the 256 MB Infinity Cache).
//   make -C whisper.coreml_amd tools/proj_bench && ./whisper.coreml_amd/tools/proj_bench [rows [copies]]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "wh_kernels.h"
#include "wh_proj.h"

using namespace wh;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef void (*KFn)(GemmArgs);

__global__ void k_empty(int* p) {
  if (p && threadIdx.x == 1023) p[0] = 1;
}
// stream `bytes` with every load of a thread issued before any use (U float4 per thread)
template <int U>
__global__ __launch_bounds__(256) void k_stream(const float4_t* __restrict__ src, int64_t n4, float* out) {
  float4_t v[U];
  const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + 256 * u;
    v[u] = i < n4 ? src[i] : (float4_t){0.f, 0.f, 0.f, 0.f};
  }
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) s += v[u][0] + v[u][1] + v[u][2] + v[u][3];
  if (s == 123.f) out[0] = s;
}

struct Var { int mt, nsub, kw, nstep, lds; KFn part, gelu; };

template <int MT, int NSUB, int KW, int NSTEP>
static Var var() {
  return {MT, NSUB, KW, NSTEP, ProjShape<half_t, MT, NSUB, KW, NSTEP>::LDS,
          &k_proj<half_t, MT, NSUB, KW, NSTEP, EPI_PARTIAL>, &k_proj<half_t, MT, NSUB, KW, NSTEP, EPI_STORE_GELU>};
}

#define V3(MT, NSUB, KW) var<MT, NSUB, KW, 5>(), var<MT, NSUB, KW, 10>(), var<MT, NSUB, KW, 20>()
#define V6(MT, NSUB) V3(MT, NSUB, 1), V3(MT, NSUB, 2)
#define V18(MT) V6(MT, 4), V6(MT, 5), V6(MT, 8)
static const Var VARS[] = {V18(4), V18(7), V3(2, 4, 1), V3(2, 4, 2)};

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 100;
  // argv[2] = distinct weight copies (32: HBM-cold as in a step; 1: Infinity-Cache warm)
  const int n = 1280, L = argc > 2 ? atoi(argv[2]) : 32, iters = 128 / L;
  struct Shape { const char* name; int N, K; };
  const Shape shapes[] = {{"qkv", 3 * n, n}, {"out", n, n}, {"fc1", 4 * n, n}, {"fc2", n, 4 * n}};
  const size_t wsz = (size_t)4 * n * n;
  half_t* W;
  CK(hipMalloc(&W, wsz * L * sizeof(half_t)));
  CK(hipMemset(W, 0, wsz * L * sizeof(half_t)));
  half_t *X, *Y;
  CK(hipMalloc(&X, (size_t)M * 4 * n * sizeof(half_t)));
  CK(hipMemset(X, 0, (size_t)M * 4 * n * sizeof(half_t)));
  CK(hipMalloc(&Y, (size_t)M * 4 * n * sizeof(half_t)));
  float *part, *xf, *bias, *lg, *lb;
  CK(hipMalloc(&part, (size_t)16 * M * 4 * n * sizeof(float)));
  CK(hipMalloc(&xf, (size_t)M * 4 * n * sizeof(float)));
  CK(hipMemset(xf, 0, (size_t)M * 4 * n * sizeof(float)));
  CK(hipMalloc(&bias, 4 * n * sizeof(float)));
  CK(hipMemset(bias, 0, 4 * n * sizeof(float)));
  CK(hipMalloc(&lg, n * sizeof(float)));
  CK(hipMalloc(&lb, n * sizeof(float)));
  CK(hipMemset(lg, 0, n * sizeof(float)));
  CK(hipMemset(lb, 0, n * sizeof(float)));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));

  auto timeit = [&](auto&& run) {
    for (int l = 0; l < L; ++l) run(l);
    CK(hipEventRecord(a, st));
    for (int i = 0; i < iters; ++i)
      for (int l = 0; l < L; ++l) run(l);
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    CK(hipGetLastError());
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1e3 / (iters * L);
  };

  printf("rows=%d\n%-5s %-14s %3s %3s %3s %6s %8s %8s\n", M, "shape", "variant", "mt", "ct", "z", "wgs", "us",
         "GB/s(W)");
  for (const auto& sh : shapes) {
    const double wbytes = (double)sh.N * sh.K * 2;
    // baseline: split-K k_gemv_x + the reduce that consumes its slabs
    {
      GemmArgs g;
      g.M = M; g.N = sh.N; g.K = sh.K; g.ldx = sh.K; g.X = X;
      g.out_f32 = part; g.ldo = sh.N; g.ksplit = gemv_ksplit(M, sh.N, sh.K, 16);
      const double us = timeit([&](int l) {
        g.W = W + (size_t)l * wsz;
        launch_gemm<half_t>(g, EPI_PARTIAL, st);
      });
      const double us2 = timeit([&](int l) {
        g.W = W + (size_t)l * wsz;
        launch_gemm<half_t>(g, EPI_PARTIAL, st);
        if (sh.N == n)
          launch_resid_ln<half_t>(xf, part, g.ksplit, (int64_t)M * sh.N, bias, Y, lg, lb, M, n, 1e-5f, st);
        else
          launch_reduce_store<half_t>(part, g.ksplit, (int64_t)M * sh.N, bias, Y, sh.N, M, sh.N, 1, st);
      });
      printf("%-5s %-14s %3s %3d %3d %6s %8.2f %8.1f\n", sh.name, "gemv_x", "-", 64, g.ksplit, "-", us,
             wbytes / (us * 1e-6) / 1e9);
      printf("%-5s %-14s %3s %3d %3d %6s %8.2f %8.1f\n", sh.name, "gemv_x+reduce", "-", 64, g.ksplit, "-", us2,
             wbytes / (us2 * 1e-6) / 1e9);
    }
    for (const Var& v : VARS) {
      const int kw = v.kw, kc = kw * v.nstep * 32;
      if (sh.K % kc) continue;
      const int z = sh.K / kc;
      if (v.lds > 160 * 1024) continue;
      const int nct = (sh.N + 16 * v.nsub - 1) / (16 * v.nsub), nmg = (M + 16 * v.mt - 1) / (16 * v.mt);
      const int wgs = nct * nmg * z;
      if (wgs < 64 || wgs > 1100) continue;
      KFn f = z == 1 ? v.gelu : v.part;
      CK(hipFuncSetAttribute(reinterpret_cast<const void*>(f), hipFuncAttributeMaxDynamicSharedMemorySize, v.lds));
      GemmArgs g;
      g.M = M; g.N = sh.N; g.K = sh.K; g.ldx = sh.K; g.X = X;
      g.bias = bias; g.out = Y; g.ldo = sh.N; g.out_f32 = part; g.ksplit = z;
      const double us = timeit([&](int l) {
        g.W = W + (size_t)l * wsz;
        hipLaunchKernelGGL(f, dim3(wgs), dim3(64 * v.nsub * v.kw), v.lds, st, g);
      });
      printf("%-5s %-14s %3d %3d %3d %6d %8.2f %8.1f  nstep=%d kw=%d\n", sh.name, "proj", v.mt, 16 * v.nsub, z, wgs,
             us, wbytes / (us * 1e-6) / 1e9, v.nstep, v.kw);
    }
    fflush(stdout);
  }
  CK(hipGetLastError());
  return 0;
}
