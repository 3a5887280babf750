// Probe (round 5): does a captured hipGraph run two independent branches at the same time?
// The step's cross-attention streams 154 MB of cross-K/V that do not depend on the
// cross-q projection before it — only its query does.  If a graph branch could start the
// cross-attention beside the (latency-bound, HBM-light) projection, its stream would overlap
// the projection.  Captured here: stream A runs a 256-workgroup kernel that spins ~50 us;
// a fork (event) lets stream B run a 200-workgroup mark kernel with no dependency on it;
// both join before the next node.  Printed: when B's workgroups started relative to A's
// first and last workgroup start / end, for (1) the fork captured before A's launch, (2)
// after it, and (3) the same two-stream pattern eagerly (no graph).
//   hipcc --offload-arch=gfx950 -O3 -o tools/graph_branch_probe tools/graph_branch_probe.hip && tools/graph_branch_probe
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

__global__ __launch_bounds__(256) void k_spin(unsigned long long* ts, int ticks) {
  if (threadIdx.x == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    ts[2 * blockIdx.x] = t0;
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)ticks) __builtin_amdgcn_s_sleep(2);
    ts[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
  }
}
__global__ __launch_bounds__(512) void k_mark(unsigned long long* ts) {
  if (threadIdx.x == 0) ts[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
}
__global__ void k_nop(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 1000000) p[0] = 1;
}

static int report(const char* name, unsigned long long* dA, unsigned long long* dB) {
  std::vector<unsigned long long> a(512), b(200);
  CK(hipMemcpy(a.data(), dA, 512 * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), dB, 200 * 8, hipMemcpyDeviceToHost));
  unsigned long long a0 = ~0ull, a1 = 0, aend = 0, b0 = ~0ull, b1 = 0;
  for (int i = 0; i < 256; ++i) {
    a0 = std::min(a0, a[2 * i]);
    a1 = std::max(a1, a[2 * i]);
    aend = std::max(aend, a[2 * i + 1]);
  }
  for (int i = 0; i < 200; ++i) {
    b0 = std::min(b0, b[i]);
    b1 = std::max(b1, b[i]);
  }
  auto us = [&](unsigned long long t) { return ((double)t - (double)a0) * 0.01; };
  printf("%-40s A starts 0.00 .. %.2f, A ends %.2f; B starts %.2f .. %.2f us -> %s\n", name, us(a1), us(aend), us(b0),
         us(b1), b1 < aend ? "CONCURRENT" : "serialised");
  return 0;
}

int main() {
  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  hipEvent_t fork, join;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  unsigned long long *dA, *dB;
  CK(hipMalloc(&dA, 512 * 8));
  CK(hipMalloc(&dB, 200 * 8));
  const int ticks = 5000;  // 50 us
  for (int order = 0; order < 2; ++order) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(sa, hipStreamCaptureModeGlobal));
    k_nop<<<1, 64, 0, sa>>>(nullptr);
    if (order == 0) {
      CK(hipEventRecord(fork, sa));
      CK(hipStreamWaitEvent(sb, fork, 0));
      k_spin<<<256, 256, 0, sa>>>(dA, ticks);
      k_mark<<<200, 512, 0, sb>>>(dB);
    } else {
      CK(hipEventRecord(fork, sa));
      k_spin<<<256, 256, 0, sa>>>(dA, ticks);
      CK(hipStreamWaitEvent(sb, fork, 0));
      k_mark<<<200, 512, 0, sb>>>(dB);
    }
    CK(hipEventRecord(join, sb));
    CK(hipStreamWaitEvent(sa, join, 0));
    k_nop<<<1, 64, 0, sa>>>(nullptr);
    CK(hipStreamEndCapture(sa, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int rep = 0; rep < 3; ++rep) CK(hipGraphLaunch(ge, sa));
    CK(hipStreamSynchronize(sa));
    if (report(order == 0 ? "graph, branch B forked before A's launch" : "graph, branch B captured after A", dA, dB))
      return 1;
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  // eager two streams
  for (int rep = 0; rep < 3; ++rep) {
    k_nop<<<1, 64, 0, sa>>>(nullptr);
    CK(hipEventRecord(fork, sa));
    CK(hipStreamWaitEvent(sb, fork, 0));
    k_spin<<<256, 256, 0, sa>>>(dA, ticks);
    k_mark<<<200, 512, 0, sb>>>(dB);
    CK(hipDeviceSynchronize());
  }
  if (report("eager, two streams", dA, dB)) return 1;
  printf("done\n");
  return 0;
}
