// Probe (round 5): what a kernel's first kernel-argument load costs.  Every step kernel
// starts by loading its arguments (s_load from the kernarg segment) and can issue no
// address-dependent load before they land; the chain traces show 2-4 us from a launch's
// first workgroup start to its first data phase.  This kernel times, with s_memrealtime
// (100 MHz) around each s_load + s_waitcnt in inline asm (so nothing the compiler hoists
// touches the segment first): (1) the first load of the segment, (2) a load from another
// 64-B line of it, (3) a scalar load from a device global the previous kernel wrote, (4)
// the same line again (a K$ hit).  Launch forms: eager stream launches, one hipGraph of the
// same launches, and both with a 256 MB streaming kernel between the probes (cold caches).
//   hipcc --offload-arch=gfx950 -O3 -o tools/kernarg_probe tools/kernarg_probe.hip && tools/kernarg_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));             \
      return 1;                                                                            \
    }                                                                                      \
  } while (0)

struct KArgs {  // 256 B, like the step kernels' GemmArgs
  int idx;
  int pad[63];
};

constexpr int NP = 64;
__device__ unsigned long long g_t[NP * 4][4];
__device__ int g_flag[64];

__global__ __launch_bounds__(64) void k_karg(KArgs) {
  const auto kp = __builtin_amdgcn_kernarg_segment_ptr();
  const int* fp = g_flag;
  unsigned long long t0, t1, t2, t3, t4;
  int idx, v1, v2, v3;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0));
  asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(idx) : "s"(kp));
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1));
  asm volatile("s_load_dword %0, %1, 0xc0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v1) : "s"(kp));
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t2));
  asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v2) : "s"(fp));
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t3));
  asm volatile("s_load_dword %0, %1, 0x4\n\ts_waitcnt lgkmcnt(0)" : "=s"(v3) : "s"(kp));
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t4));
  if (threadIdx.x == 0) {
    const int i = idx & (NP * 4 - 1);
    g_t[i][0] = t1 - t0;
    g_t[i][1] = t2 - t1;
    g_t[i][2] = t3 - t2;
    g_t[i][3] = t4 - t3 + 0 * (v1 + v2 + v3);
    g_flag[0] = idx;  // vector store: the next probe's scalar load of it misses
  }
}

// 256 MB streamed by every CU (evicts L2 / MALL lines, as a step's weight stream does)
__global__ __launch_bounds__(256) void k_stream(const float4* p, size_t n, float* sink) {
  float4 acc = make_float4(0, 0, 0, 0);
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const float4 v = p[i];
    acc.x += v.x;
  }
  if (acc.x == 1234.5f) sink[0] = acc.x;
}

static int run(const char* name, bool graph, bool cold, const float4* buf, size_t n, float* sink, hipStream_t st) {
  KArgs a{};
  std::vector<unsigned long long> h(NP * 4 * 4);
  auto body = [&]() {
    for (int i = 0; i < NP; ++i) {
      if (cold) k_stream<<<1024, 256, 0, st>>>(buf, n, sink);
      a.idx = i;
      k_karg<<<1, 64, 0, st>>>(a);
    }
  };
  hipGraphExec_t ge = nullptr;
  if (graph) {
    hipGraph_t g;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    body();
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphDestroy(g));
  }
  for (int rep = 0; rep < 3; ++rep) {
    if (graph)
      CK(hipGraphLaunch(ge, st));
    else
      body();
    CK(hipStreamSynchronize(st));
  }
  CK(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_t), h.size() * 8));
  const char* what[4] = {"first kernarg line", "second kernarg line", "device global (written by the last probe)",
                         "kernarg line again (K$ hit)"};
  for (int k = 0; k < 4; ++k) {
    std::vector<double> v;
    for (int i = 1; i < NP; ++i) v.push_back(h[i * 4 + k] * 0.01);
    std::sort(v.begin(), v.end());
    printf("%-34s %-44s median %6.2f us  p10 %6.2f  p90 %6.2f\n", name, what[k], v[v.size() / 2], v[v.size() / 10],
           v[v.size() * 9 / 10]);
  }
  if (ge) CK(hipGraphExecDestroy(ge));
  return 0;
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const size_t bytes = (size_t)256 << 20, n = bytes / 16;
  float4* buf;
  float* sink;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 0, bytes));
  CK(hipDeviceSynchronize());
  if (run("eager, back to back", false, false, buf, n, sink, st)) return 1;
  if (run("hipGraph, back to back", true, false, buf, n, sink, st)) return 1;
  if (run("eager, 256 MB stream between", false, true, buf, n, sink, st)) return 1;
  if (run("hipGraph, 256 MB stream between", true, true, buf, n, sink, st)) return 1;
  printf("done\n");
  return 0;
}
