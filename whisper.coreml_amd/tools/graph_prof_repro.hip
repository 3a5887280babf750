// Minimal reproducer for the rocprofv3 --kernel-trace segfault seen when the decoder
// step is replayed as a hipGraph.  Captures a chain of `nodes` kernel
// launches whose by-value argument is `argb` bytes (the step's kernels take 100-400 B
// structs), instantiates, replays it `reps` times.  Usage: graph_prof_repro nodes argb reps
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int B>
struct Arg { float* p; char pad[B - 8]; };

template <int B>
__global__ void k_touch(Arg<B> a) {
  if (threadIdx.x == 0 && blockIdx.x == 0) a.p[0] += (float)a.pad[B - 9];
}

template <int B>
int run(int nodes, int reps) {
  float* d = nullptr;
  if (hipMalloc(&d, 4) != hipSuccess) return 1;
  hipMemset(d, 0, 4);
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  Arg<B> a{};
  a.p = d;
  a.pad[B - 9] = 1;
  hipGraph_t g;
  hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
  for (int i = 0; i < nodes; ++i) k_touch<B><<<1, 64, 0, st>>>(a);
  if (hipStreamEndCapture(st, &g) != hipSuccess) return 2;
  hipGraphExec_t ge;
  if (hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) != hipSuccess) return 3;
  for (int r = 0; r < reps; ++r) hipGraphLaunch(ge, st);
  hipStreamSynchronize(st);
  float h = 0;
  hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  printf("nodes %d argb %d reps %d -> %.0f (want %d)\n", nodes, B, reps, h, nodes * reps);
  return h == (float)(nodes * reps) ? 0 : 4;
}

int main(int argc, char** argv) {
  const int nodes = argc > 1 ? atoi(argv[1]) : 400, argb = argc > 2 ? atoi(argv[2]) : 256,
            reps = argc > 3 ? atoi(argv[3]) : 50;
  switch (argb) {
    case 64: return run<64>(nodes, reps);
    case 256: return run<256>(nodes, reps);
    case 1024: return run<1024>(nodes, reps);
    default: return run<2048>(nodes, reps);
  }
}
