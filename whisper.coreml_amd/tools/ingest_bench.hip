// Per-node wall time of a captured chain of "projection-shaped" kernels: what one
// dependent launch costs as a function of the bytes each workgroup must ingest.  Each
// workgroup loads H bytes of a streamed (HBM, distinct per node and workgroup) buffer and
// S bytes of a shared buffer (the same S-byte slice is read by every workgroup of a
// group of `share` consecutive workgroups: L2 / Infinity-Cache resident after its first
// read, as a projection's activation rows are), 16 B per lane per load, `ilp` loads in
// flight per lane per batch, then stores 1 KB per workgroup.  Used to price the
// row-tiled full-K decoder projections against the split-K + reduction chain
// (DESIGN.md round 4).
//   make -C whisper.coreml_amd tools/ingest_bench && ./whisper.coreml_amd/tools/ingest_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef float float4_t __attribute__((ext_vector_type(4)));

struct Arg {
  const float4_t* hbm;     // this node's streamed buffer
  const float4_t* shared;  // shared slices
  float4_t* dst;
  int h16;    // float4 per workgroup from hbm
  int s16;    // float4 per workgroup from shared
  int share;  // workgroups per shared slice
};

template <int ILP>
__global__ __launch_bounds__(512) void k_ingest(Arg a) {
  const int t = threadIdx.x, nt = blockDim.x;
  const float4_t* h = a.hbm + (size_t)blockIdx.x * a.h16;
  const float4_t* s = a.shared + (size_t)(blockIdx.x / a.share) * a.s16;
  float4_t acc = {0.f, 0.f, 0.f, 0.f};
  // shared first (the activation rows), then the streamed bytes, ILP loads per batch
  for (int base = t; base < a.s16; base += nt * ILP) {
    float4_t v[ILP];
#pragma unroll
    for (int i = 0; i < ILP; ++i) v[i] = base + i * nt < a.s16 ? s[base + i * nt] : (float4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < ILP; ++i) acc += v[i];
  }
  for (int base = t; base < a.h16; base += nt * ILP) {
    float4_t v[ILP];
#pragma unroll
    for (int i = 0; i < ILP; ++i) v[i] = base + i * nt < a.h16 ? h[base + i * nt] : (float4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < ILP; ++i) acc += v[i];
  }
  if (t < 64) a.dst[blockIdx.x * 64 + t] = acc;
}

int main(int argc, char** argv) {
  const int nodes = argc > 1 ? atoi(argv[1]) : 96, reps = argc > 2 ? atoi(argv[2]) : 10;
  // (hbm KB, shared KB, workgroups, share, threads)
  struct C { int hk, sk, wgs, share, thr; const char* what; } cs[] = {
      {20, 35, 160, 20, 256, "k_proj out/cross (z=8): W 20 KB + X slice 35 KB"},
      {51, 72, 256, 64, 320, "k_proj fc1 (z=4): W 51 KB + X slice 72 KB"},
      {0, 0, 256, 1, 256, "nop"},
      {16, 0, 256, 1, 256, "16 KB hbm only"},
      {40, 80, 160, 40, 512, "rowtile 32x32 full K=1280 fp16 X: W 80 + X 80"},
      {80, 160, 160, 40, 512, "rowtile 32x32 K=1280 fp32 X (LN): W 80 + X 160"},
      {80, 80, 160, 40, 512, "rowtile 32x32 K=1280 fp16 X: W 80 + X 80 (2)"},
      {160, 160, 240, 60, 512, "rowtile 32x64 qkv K=1280 fp32 X: W 160 + X 160"},
      {160, 160, 320, 80, 512, "rowtile 32x64 fc1 K=1280 fp32 X: W 160 + X 160"},
      {327, 327, 160, 40, 512, "rowtile 32x32 fc2 K=5120 fp16 X: W 327 + X 327"},
      {164, 164, 320, 40, 512, "rowtile 32x32 fc2 K/2: W 164 + X 164"},
      {164, 327, 320, 80, 512, "rowtile 32x16 fc2 K=5120: W 164 + X 327"},
  };
  const int ncs = sizeof(cs) / sizeof(cs[0]);
  size_t hmax = 0, smax = 0;
  for (auto& c : cs) {
    hmax = std::max(hmax, (size_t)c.hk * 1024 * c.wgs);
    smax = std::max(smax, (size_t)c.sk * 1024 * (c.wgs / c.share + 1));
  }
  // distinct streamed bytes per node: nodes x hmax (cap at ~8 GB)
  const int nbuf = (int)std::min<size_t>(nodes, ((size_t)8 << 30) / std::max<size_t>(hmax, 1));
  char *hbm, *shared;
  float4_t* dst;
  CK(hipMalloc(&hbm, hmax * nbuf));
  CK(hipMemset(hbm, 0, hmax * nbuf));
  CK(hipMalloc(&shared, smax));
  CK(hipMemset(shared, 0, smax));
  CK(hipMalloc(&dst, 2048 * 64 * sizeof(float4_t)));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int ci = 0; ci < ncs; ++ci) {
    const C& c = cs[ci];
    for (int ilp : {8, 16}) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
      for (int i = 0; i < nodes; ++i) {
        Arg a{};
        a.hbm = reinterpret_cast<const float4_t*>(hbm + hmax * (i % nbuf));
        a.shared = reinterpret_cast<const float4_t*>(shared);
        a.dst = dst;
        a.h16 = c.hk * 1024 / 16;
        a.s16 = c.sk * 1024 / 16;
        a.share = c.share;
        if (ilp == 8) k_ingest<8><<<c.wgs, c.thr, 0, st>>>(a);
        else k_ingest<16><<<c.wgs, c.thr, 0, st>>>(a);
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
      printf("%-58s wgs %4d thr %3d ilp %2d: %6.2f us per node\n", c.what, c.wgs, c.thr, ilp,
             ms * 1e3 / (reps * nodes));
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
