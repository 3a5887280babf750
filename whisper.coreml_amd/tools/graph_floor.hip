// Per-node wall time of a captured hipGraph chain (what a decoder step's ~390 dependent
// kernels pay beyond their own work): N nodes of one kernel kind, replayed R times,
// hipEvents around the replays.  Kinds: 0 = 1 workgroup doing nothing, 1 = 256
// workgroups doing nothing, 2 = 256 workgroups of 256 threads each loading 16 KB (one
// 16 B load per lane x 4, a distinct slice per node so it streams) and storing 1 KB,
// 3 = kind 2 with 512-thread workgroups and 32 KB.  A 256-byte by-value argument as
// the step's GemmArgs.
//   make -C whisper.coreml_amd tools/graph_floor && ./whisper.coreml_amd/tools/graph_floor
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

struct Arg {
  const float4* src;
  float4* dst;
  int per;  // float4 loads per lane
  int pad[58];
};

__global__ void k_nop(Arg a) {
  if (a.per < 0) a.dst[threadIdx.x] = make_float4(0, 0, 0, 0);
}

__global__ void k_stream(Arg a) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x, n = gridDim.x * blockDim.x;
  float4 s = make_float4(0, 0, 0, 0);
  for (int i = 0; i < a.per; ++i) {
    const float4 v = a.src[t + (size_t)i * n];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  if (threadIdx.x < 64) a.dst[blockIdx.x * 64 + threadIdx.x] = s;
}

int main(int argc, char** argv) {
  const int nodes = argc > 1 ? atoi(argv[1]) : 384, reps = argc > 2 ? atoi(argv[2]) : 20;
  const size_t slice = (size_t)32 * 1024 * 256;  // bytes per node for kind 3
  float4 *src, *dst;
  CK(hipMalloc(&src, slice * nodes));
  CK(hipMemset(src, 0, slice * nodes));
  CK(hipMalloc(&dst, 256 * 64 * sizeof(float4)));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[] = {"1 wg nop", "256 wg nop", "256 wg x 256 thr, 16 KB/wg load", "256 wg x 512 thr, 32 KB/wg load"};
  for (int kind = 0; kind < 4; ++kind) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < nodes; ++i) {
      Arg a{};
      a.src = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(src) + slice * i);
      a.dst = dst;
      a.per = kind >= 2 ? 4 : 0;
      if (kind == 0) k_nop<<<1, 64, 0, st>>>(a);
      else if (kind == 1) k_nop<<<256, 256, 0, st>>>(a);
      else if (kind == 2) k_stream<<<256, 256, 0, st>>>(a);
      else k_stream<<<256, 512, 0, st>>>(a);
    }
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-36s %d nodes: %.2f us per node\n", names[kind], nodes, ms * 1e3 / (reps * nodes));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
