// What an all-to-all activation hand-off ("edge") costs inside ONE persistent launch
// against the same dependency cut as a kernel boundary in a captured hipGraph chain —
// the question behind a batch-1 weight-streaming decode engine (MI355X_MICROARCH.md
// "engine-vs-launches"): a decoder layer at one window is 8 dependent phases whose every
// input is the WHOLE previous output (5 rows x 1280: 12.8 KB fp16 / 25.6 KB fp32; fc1's
// 51 KB), so each phase boundary is an all-gather to every CU.
//
// Edge e (E of them): every workgroup (256, one per CU) stores its slice of payload[e]
// (B / 256 bytes) write-through (sc1), drains it (vmcnt(0)), adds 1 to cnt[e] (relaxed
// agent atomic, lane 0); the next phase waits for cnt[e] == 256 (lane-0 poll with s_sleep,
// bounded: a timeout sets err and the loop still ends), then every thread reads the whole
// payload[e] with sc1 loads; its sum seeds the slice of edge e + 1 (a real data
// dependency, checked on the host).  Optional weight stream: W bytes per workgroup per
// phase from a buffer far larger than the Infinity Cache; the persistent kernel issues the
// NEXT phase's weight loads before it waits (what an engine's loader buys), the chain
// kernel can only issue them at its own start.
//   make -C whisper.coreml_amd tools/edge_bench && ./whisper.coreml_amd/tools/edge_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef float float4_t __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int NWG = 256, NT = 256, NC = NT - 64;  // NC: engine consumer threads
constexpr int MAXL = 16;  // payload float4 per thread (B <= 48 KB)
constexpr int WMAX = 8;   // weight float4 per thread per phase (W <= 32 KB)

struct Args {
  float* pay;        // [E][B / 4] floats
  int* cnt;          // [E]
  const float4_t* w; // weight stream
  int64_t wstride;   // float4 between consecutive phases' weight blocks
  int E, B, W;
  int* err;
  int xcd;  // engine hand-off: 0 flat counter, 1 per-XCD counters + top counter
};

__device__ __forceinline__ float slice_value(int e, int wg) { return (float)((e * 7 + wg) % 13); }

// sum of payload[e] read by this thread (n4 float4 in all, thread-strided)
template <bool SC1>
__device__ __forceinline__ float read_payload(const Args& a, int e) {
  const int n4 = a.B / 16;
  const float* base = a.pay + (int64_t)e * (a.B / 4);
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
  float4_t v[MAXL];
#pragma unroll
  for (int i = 0; i < MAXL; ++i) {
    const int c = threadIdx.x + (SC1 ? NC : NT) * i;
    if (SC1)
      v[i] = c < n4 ? __builtin_bit_cast(float4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, c * 16, 0, 16))
                    : (float4_t){0.f, 0.f, 0.f, 0.f};
    else
      v[i] = c < n4 ? reinterpret_cast<const float4_t*>(base)[c] : (float4_t){0.f, 0.f, 0.f, 0.f};
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXL; ++i) s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
  return s;
}

// this workgroup's slice of payload[e]: B / 256 bytes = B / 1024 floats... stored by the
// first B / (256 * 16) threads, one float4 each, value slice_value(e, wg) + 0 * seed
template <bool SC1>
__device__ __forceinline__ void write_slice(const Args& a, int e, float seed) {
  const int per = a.B / (NWG * 16);  // float4 per workgroup
  float* base = a.pay + (int64_t)e * (a.B / 4) + (int64_t)blockIdx.x * per * 4;
  if ((int)threadIdx.x < per) {
    const float v = slice_value(e, blockIdx.x) + (seed == -1.f ? 1.f : 0.f);
    const float4_t q = (float4_t){v, v, v, v};
    if (SC1) {
      const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, q), rs, threadIdx.x * 16, 0, 16);
    } else {
      reinterpret_cast<float4_t*>(base)[threadIdx.x] = q;
    }
  }
}

__device__ __forceinline__ float a_expect(const Args& a, int e) {
  // the whole payload of edge e summed: every workgroup's slice holds per*4 copies
  float s = 0.f;
  for (int wg = 0; wg < NWG; ++wg) s += slice_value(e, wg);
  return s * (float)(a.B / (NWG * 16) * 4);
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}

// waves 0-2 consume (slice store, hand-off, payload read); wave 3 is the weight loader:
// it moves the NEXT phase's W bytes into an LDS double buffer by LDS-DMA while the others
// run the hand-off (on CDNA one wave's vmcnt covers all its memory ops, so a poller that
// also prefetched would wait for its own prefetch), and retires them with its own vmcnt
// before the barrier that opens that phase.  Raw s_barriers: a __syncthreads() would make
// the loader drain its DMA at every barrier.
__global__ __launch_bounds__(NT) void k_engine(Args a) {
  __shared__ float red[NT / 64];
  __shared__ __attribute__((aligned(16))) char wbuf[2][32768];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const bool loader = wave == 3;
  const int wk = a.W / 1024;  // 1 KB LDS-DMA instructions per phase
  auto wload = [&](int e) {
    const char* src = reinterpret_cast<const char*>(a.w + (int64_t)e * a.wstride) + (int64_t)blockIdx.x * a.W + lane * 16;
    for (int i = 0; i < wk; ++i)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src + i * 1024),
                                       (__attribute__((address_space(3))) void*)(wbuf[e & 1] + i * 1024), 16, 0, 0);
  };
  int bad = 0;
  if (loader) {
    wload(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  raw_barrier();
  for (int e = 0; e < a.E; ++e) {
    // this phase's weights (landed before the barrier above) feed the slice
    const float ws = a.W ? reinterpret_cast<const float*>(wbuf[e & 1])[tid] : 0.f;
    if (loader) {
      if (e + 1 < a.E) wload(e + 1);  // next phase's weights in flight across the hand-off
    } else {
      write_slice<true>(a, e, ws * 0.f);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    raw_barrier();
    if (tid == 0) {
      // flat: 256 arrivals on cnt[e]; per-XCD (a.xcd): 32 arrivals on the group counter
      // cnt[E + 8e + g] (g = blockIdx % 8: the round-robin XCD, speed only), whose last
      // arriver adds 1 to cnt[e]; the wait is for cnt[e] == 256 resp. 8
      int target = NWG;
      if (a.xcd) {
        const int g = blockIdx.x & 7;
        target = 8;
        if (__hip_atomic_fetch_add(a.cnt + a.E + 8 * e + g, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == NWG / 8 - 1)
          __hip_atomic_fetch_add(a.cnt + e, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        __hip_atomic_fetch_add(a.cnt + e, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      int it = 0;
      while (__hip_atomic_load(a.cnt + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++it > (1 << 22)) { atomicExch(a.err, 1); break; }
      }
    }
    raw_barrier();
    if (!loader) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      float s = read_payload<true>(a, e);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      if (lane == 0) red[wave] = s;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // next phase's weights landed
    }
    raw_barrier();
    if (tid == 0) {
      const float tot = red[0] + red[1] + red[2];
      bad |= tot != a_expect(a, e);
    }
  }
  if (tid == 0 && bad) atomicAdd(a.err + 1, 1);
}

// one phase of the chain: read payload[e - 1] whole (plain loads: the boundary made it
// visible), this phase's weights issued at the start, store the slice of payload[e]
__global__ __launch_bounds__(NT) void k_chain(Args a, int e) {
  __shared__ float red[NT / 64];
  const int tid = threadIdx.x, wn = a.W / (NT * 16);
  float4_t wv[WMAX];
  const float4_t* wp = a.w + (int64_t)e * a.wstride + (int64_t)blockIdx.x * (a.W / 16) + tid;
#pragma unroll
  for (int i = 0; i < WMAX; ++i) wv[i] = i < wn ? wp[NT * i] : (float4_t){0.f, 0.f, 0.f, 0.f};
  float tot = 0.f, ok = 0.f;
  if (e > 0) {
    float s = read_payload<false>(a, e - 1);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((tid & 63) == 0) red[tid >> 6] = s;
    __syncthreads();
    for (int k = 0; k < NT / 64; ++k) tot += red[k];
    ok = tot == a_expect(a, e - 1) ? 0.f : -1.f;
    if (tid == 0 && ok != 0.f) atomicAdd(a.err + 1, 1);
  }
  float ws = 0.f;
#pragma unroll
  for (int i = 0; i < WMAX; ++i) ws += wv[i][0];
  write_slice<false>(a, e, ok + ws * 0.f);
}

int main(int argc, char** argv) {
  const int E = argc > 1 ? atoi(argv[1]) : 64, reps = argc > 2 ? atoi(argv[2]) : 20;
  const int Bs[] = {12288, 24576, 49152};  // multiples of 256 x 16 B
  const int Ws[] = {0, 16384, 32768};
  int dev;
  CK(hipGetDevice(&dev));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, dev));
  if (prop.multiProcessorCount < NWG) {
    printf("needs %d CUs (have %d): a persistent grid of %d would not be co-resident\n", NWG, prop.multiProcessorCount, NWG);
    return 1;
  }
  float* pay;
  int *cnt, *err;
  CK(hipMalloc(&pay, (size_t)E * 65536));
  CK(hipMalloc(&cnt, 9 * E * sizeof(int)));
  CK(hipMalloc(&err, 2 * sizeof(int)));
  // weights: E phases x 256 workgroups x W, spread over > 1 GB so a replay streams from HBM
  const int64_t wstride4 = (int64_t)NWG * 32768 / 16 * 3;  // float4 between phases (3x the max)
  float4_t* w;
  CK(hipMalloc(&w, (size_t)E * wstride4 * 16));
  CK(hipMemset(w, 0, (size_t)E * wstride4 * 16));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("E = %d dependent phases, 256 workgroups x 256 threads, %d reps\n", E, reps);
  printf("%8s %8s %6s %14s %14s %10s\n", "payload", "W/wg", "xcd", "engine us/edge", "chain us/phase", "errors");
  for (int B : Bs)
    for (int W : Ws)
     for (int xcd = 0; xcd < 2; ++xcd) {
      Args a{pay, cnt, w, wstride4, E, B, W, err, xcd};
      CK(hipMemset(err, 0, 2 * sizeof(int)));
      // engine: counters zeroed before every replay (memset node + kernel in one graph)
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
      CK(hipMemsetAsync(cnt, 0, 9 * E * sizeof(int), st));
      k_engine<<<NWG, NT, 0, st>>>(a);
      CK(hipStreamEndCapture(st, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      hipGraph_t gz;
      hipGraphExec_t gze;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
      CK(hipMemsetAsync(cnt, 0, 9 * E * sizeof(int), st));
      CK(hipStreamEndCapture(st, &gz));
      CK(hipGraphInstantiate(&gze, gz, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, st));
      CK(hipStreamSynchronize(st));
      int herr[2];
      CK(hipMemcpy(herr, err, sizeof(herr), hipMemcpyDeviceToHost));
      if (herr[0]) {
        printf("engine wait timed out (payload %d) - stopping\n", B);
        return 2;
      }
      float ms_e = 0.f, ms_z = 0.f, ms;
      CK(hipEventRecord(e0, st));
      for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms_e, e0, e1));
      CK(hipEventRecord(e0, st));
      for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(gze, st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms_z, e0, e1));
      // chain
      hipGraph_t gc;
      hipGraphExec_t gce;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
      for (int e = 0; e < E; ++e) k_chain<<<NWG, NT, 0, st>>>(a, e);
      CK(hipStreamEndCapture(st, &gc));
      CK(hipGraphInstantiate(&gce, gc, nullptr, nullptr, 0));
      CK(hipGraphLaunch(gce, st));
      CK(hipStreamSynchronize(st));
      CK(hipEventRecord(e0, st));
      for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(gce, st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      CK(hipMemcpy(herr, err, sizeof(herr), hipMemcpyDeviceToHost));
      printf("%8d %8d %6d %14.2f %14.2f %4d/%d\n", B, W, xcd, 1e3f * (ms_e - ms_z) / reps / E, 1e3f * ms / reps / E, herr[0],
             herr[1]);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
      CK(hipGraphExecDestroy(gze));
      CK(hipGraphDestroy(gz));
      CK(hipGraphExecDestroy(gce));
      CK(hipGraphDestroy(gc));
    }
  return 0;
}
