// AQL-level probe (round 5): can a kernel of the decoder-step chain START before its
// producer ends, so that its launch and its weight round trip overlap the producer?
//
// HIP stream semantics set the AQL barrier bit on every kernel packet (a packet launches
// only after every earlier packet of the queue has completed), and hip_ext.h documents
// hipExtAnyOrderLaunch as unsupported on gfx9.  Here the packets are written directly into
// an HSA queue of our own, with the barrier bit chosen per packet:
//   T0  HIP eager, hipExtAnyOrderLaunch: does the flag do anything on gfx950?
//   T1  barrier = 0 after a 256-workgroup spinning producer: when does the consumer start?
//   T2  dispatch order: a 4096-workgroup producer (two rounds of residency) followed by a
//       barrier-0 consumer: does any consumer workgroup start before the producer's last
//       workgroup started (i.e. is a grid fully dispatched before the next one begins)?
//   T3  chain of N dependent trivial kernels, barrier = 1 (HSA queue) vs a captured
//       hipGraph of the same kernels: the cost of one boundary per node
//   T4  chain of N trivial kernels, barrier = 0, each waiting on its predecessor's
//       arrival counter (256 arrivals, sharded per XCD) before adding to its own
//   T5  chain of N streaming nodes (weights W per workgroup from HBM, X slice written by
//       the predecessor, 1 KB output per workgroup, write-through): (a) barrier form,
//       one round trip for X and W; (b) overlapped form, barrier 0, W prefetched into
//       registers, wait on the counter, then X with sc1 loads
// Build: hipcc --offload-arch=gfx950 -O3 tools/aql_probe.hip -lhsa-runtime64 -o tools/aql_probe
//        hipcc --offload-arch=gfx950 -O3 --genco tools/aql_probe.hip -o tools/aql_probe.hsaco
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- device side
__device__ __forceinline__ unsigned long long rt_now() { return __builtin_amdgcn_s_memrealtime(); }

extern "C" __global__ __launch_bounds__(256) void p_spin(unsigned long long* ts, int ticks) {
  if (threadIdx.x == 0) {
    const unsigned long long t0 = rt_now();
    ts[2 * blockIdx.x] = t0;
    while (rt_now() - t0 < (unsigned long long)ticks) __builtin_amdgcn_s_sleep(2);
    ts[2 * blockIdx.x + 1] = rt_now();
  }
}

extern "C" __global__ __launch_bounds__(256) void p_mark(unsigned long long* ts) {
  if (threadIdx.x == 0) ts[blockIdx.x] = rt_now();
}

__device__ __forceinline__ unsigned ld_sc1(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wait until the 8 per-XCD shards of `cnt` sum to >= target (lanes 0..7 of wave 0 poll one
// shard each, 64 B apart); bounded: ~20 ms then err
__device__ __forceinline__ void wait_cnt(const unsigned* cnt, unsigned target, int* err) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const unsigned long long t0 = rt_now();
    while (true) {
      unsigned v = lane < 8 ? ld_sc1(cnt + 32 * lane) : 0u;
#pragma unroll
      for (int o = 4; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      v = __shfl(v, 0, 64);
      if (v >= target) break;
      if (rt_now() - t0 > 2000000ull) {
        if (lane == 0) atomicAdd(err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void arrive(unsigned* cnt) {
  // every storing wave drained its stores before the barrier; one lane adds to its XCD's shard
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    __hip_atomic_fetch_add(cnt + 32 * (xcc & 7), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

extern "C" __global__ __launch_bounds__(256) void p_node(const unsigned* prev, unsigned target, unsigned* own,
                                                          int* err) {
  if (prev) wait_cnt(prev, target, err);
  arrive(own);
}

extern "C" __global__ __launch_bounds__(256) void p_empty(int* dummy) {
  if (dummy && threadIdx.x == 0 && blockIdx.x == 100000) dummy[0] = 1;
}

// streaming node: W slice of WB x 16 B per thread (weights), X slice of 16 KB per workgroup
// (4 x 16 B per thread, sc1 when overlapped), 1 KB of output per workgroup written through.
template <int WB>
__device__ __forceinline__ void stream_body(const u32x4* W, const float* X, float* Y, const unsigned* prev,
                                            unsigned target, unsigned* own, int* err, int overlapped,
                                            int wstride16) {
  const int t = threadIdx.x, b = blockIdx.x;
  u32x4 w[WB];
  const u32x4* wp = W + (size_t)b * WB * 256 + t;
  // X: the workgroup's 16 KB slice of the predecessor's 256 KB output (slices shared by
  // the workgroups of equal b % 16)
  const int xoff = (b & 15) * 1024 + t;  // in 16-B units
  u32x4 x[4];
  if (overlapped) {
#pragma unroll
    for (int i = 0; i < WB; ++i) w[i] = wp[i * 256];
    wait_cnt(prev, target, err);
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)X, 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (xoff + 256 * i) * 16, 0, 16);
  } else {
    const u32x4* xp = reinterpret_cast<const u32x4*>(X) + xoff;
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = xp[256 * i];
#pragma unroll
    for (int i = 0; i < WB; ++i) w[i] = wp[i * 256];
  }
  const u32x4 x0 = x[0] ^ x[2], x1 = x[1] ^ x[3];
  unsigned s = x0.x ^ x1.y;
#pragma unroll
  for (int i = 0; i < WB; ++i) s += w[i].x ^ w[i].y ^ w[i].z ^ w[i].w;
  // 1 KB per workgroup: threads 0..63 store 16 B each, write-through
  if (t < 64) {
    const float4 v = make_float4((float)s, (float)x0.z, (float)x1.w, 1.0f);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v),
                                           __builtin_amdgcn_make_buffer_rsrc(Y, 0, 0x7fffffff, 0x00020000),
                                           (b * 64 + t) * 16, 0, 16);
  }
  (void)wstride16;
  if (own) arrive(own);
}

// hand-off through replicated ready flags: producers add to ONE counter; the workgroup whose
// add completes it writes `epoch` into 16 flag replicas (one line each); a consumer
// workgroup polls replica b % 16 from one lane with a longer sleep
__device__ __forceinline__ void arrive_ready(unsigned* cnt, unsigned target, unsigned* ready) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < 64) {
    unsigned old = 0;
    if (threadIdx.x == 0) old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __shfl(old, 0, 64);
    if (old == target - 1 && threadIdx.x < 16)
      __hip_atomic_store(ready + 32 * threadIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
__device__ __forceinline__ void wait_ready(const unsigned* ready, int* err, int sleep) {
  if (threadIdx.x == 0) {
    const unsigned* f = ready + 32 * (blockIdx.x & 15);
    const unsigned long long t0 = rt_now();
    while (ld_sc1(f) == 0u) {
      if (rt_now() - t0 > 2000000ull) { atomicAdd(err, 1); break; }
      if (sleep) __builtin_amdgcn_s_sleep(4); else __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}
extern "C" __global__ __launch_bounds__(256) void p_stream8r(const u32x4* W, const float* X, float* Y,
                                                              const unsigned* prev_ready, unsigned* own_cnt,
                                                              unsigned* own_ready, int* err, int sleep) {
  const int t = threadIdx.x, b = blockIdx.x;
  constexpr int WB = 8;
  u32x4 w[WB];
  const u32x4* wp = W + (size_t)b * WB * 256 + t;
  const int xoff = (b & 15) * 1024 + t;
  u32x4 x[4];
#pragma unroll
  for (int i = 0; i < WB; ++i) w[i] = wp[i * 256];
  if (prev_ready) wait_ready(prev_ready, err, sleep);
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)X, 0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int i = 0; i < 4; ++i) x[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (xoff + 256 * i) * 16, 0, 16);
  const u32x4 x0 = x[0] ^ x[2], x1 = x[1] ^ x[3];
  unsigned s = x0.x ^ x1.y;
#pragma unroll
  for (int i = 0; i < WB; ++i) s += w[i].x ^ w[i].y ^ w[i].z ^ w[i].w;
  if (t < 64) {
    const float4 v = make_float4((float)s, (float)x0.z, (float)x1.w, 1.0f);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v),
                                           __builtin_amdgcn_make_buffer_rsrc(Y, 0, 0x7fffffff, 0x00020000),
                                           (b * 64 + t) * 16, 0, 16);
  }
  arrive_ready(own_cnt, 256u, own_ready);
}

extern "C" __global__ __launch_bounds__(256) void p_stream8(const u32x4* W, const float* X, float* Y,
                                                             const unsigned* prev, unsigned target, unsigned* own,
                                                             int* err, int overlapped) {
  stream_body<8>(W, X, Y, prev, target, own, err, overlapped, 0);
}
extern "C" __global__ __launch_bounds__(256) void p_stream2(const u32x4* W, const float* X, float* Y,
                                                             const unsigned* prev, unsigned target, unsigned* own,
                                                             int* err, int overlapped) {
  stream_body<2>(W, X, Y, prev, target, own, err, overlapped, 0);
}

// ---------------------------------------------------------------- host side
#define HC(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)
#define SC(x)                                                                  \
  do {                                                                         \
    hsa_status_t s_ = (x);                                                     \
    if (s_ != HSA_STATUS_SUCCESS) {                                            \
      const char* m_ = nullptr;                                                \
      hsa_status_string(s_, &m_);                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, m_ ? m_ : "?"); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

static hsa_agent_t g_gpu;
static hsa_status_t find_gpu(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU) {
    g_gpu = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

struct Kern {
  uint64_t obj = 0;
  uint32_t kargs = 0, group = 0, priv = 0;
};

struct Aql {
  hsa_queue_t* q = nullptr;
  hsa_queue_t* qs[4] = {};
  hsa_executable_t exe{};
  hsa_signal_t done{};
  char* kbuf = nullptr;  // device kernarg arena
  size_t kcap = 0, kused = 0;
  std::vector<char> hk;  // host image of the kernarg arena
  Kern get(const char* name) {
    hsa_executable_symbol_t s;
    SC(hsa_executable_get_symbol_by_name(exe, (std::string(name) + ".kd").c_str(), &g_gpu, &s));
    Kern k;
    SC(hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.obj));
    SC(hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k.kargs));
    SC(hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.group));
    SC(hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.priv));
    return k;
  }
  void init(const char* hsaco) {
    SC(hsa_init());
    hsa_iterate_agents(find_gpu, nullptr);
    FILE* f = fopen(hsaco, "rb");
    if (!f) { fprintf(stderr, "cannot open %s\n", hsaco); exit(1); }
    std::vector<char> co;
    char buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) co.insert(co.end(), buf, buf + n);
    fclose(f);
    hsa_code_object_reader_t rd;
    SC(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &rd));
    SC(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe));
    SC(hsa_executable_load_agent_code_object(exe, g_gpu, rd, nullptr, nullptr));
    SC(hsa_executable_freeze(exe, nullptr));
    for (int i = 0; i < 4; ++i)
      SC(hsa_queue_create(g_gpu, 8192, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &qs[i]));
    q = qs[0];
    SC(hsa_signal_create(1, 0, nullptr, &done));
    kcap = 8 << 20;
    HC(hipMalloc(&kbuf, kcap));
    hk.assign(kcap, 0);
  }
  // stage a kernarg block; returns its device address
  void* karg(const void* a, size_t n, const Kern& k) {
    const size_t sz = std::max<size_t>(n, k.kargs);
    kused = (kused + 63) & ~(size_t)63;
    if (kused + sz > kcap) { fprintf(stderr, "kernarg arena full\n"); exit(1); }
    memcpy(hk.data() + kused, a, n);
    memset(hk.data() + kused + n, 0, sz - n);
    void* d = kbuf + kused;
    kused += sz;
    return d;
  }
  void upload() { HC(hipMemcpy(kbuf, hk.data(), kused, hipMemcpyHostToDevice)); }
  void reset() { kused = 0; }
  // write one dispatch packet
  int acq_scope = HSA_FENCE_SCOPE_AGENT, rel_scope = HSA_FENCE_SCOPE_AGENT;
  void dispatch(const Kern& k, void* kargs, int nwg, bool barrier, bool last, int qi = 0) {
    hsa_queue_t* q = qs[qi];
    const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
    while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {}
    hsa_kernel_dispatch_packet_t* p =
        reinterpret_cast<hsa_kernel_dispatch_packet_t*>(q->base_address) + (idx & (q->size - 1));
    memset(reinterpret_cast<char*>(p) + 4, 0, sizeof(*p) - 4);
    p->workgroup_size_x = 256;
    p->workgroup_size_y = 1;
    p->workgroup_size_z = 1;
    p->grid_size_x = (uint32_t)nwg * 256;
    p->grid_size_y = 1;
    p->grid_size_z = 1;
    p->private_segment_size = k.priv;
    p->group_segment_size = k.group;
    p->kernel_object = k.obj;
    p->kernarg_address = kargs;
    if (last) {
      hsa_signal_store_relaxed(done, 1);
      p->completion_signal = done;
    } else {
      p->completion_signal.handle = 0;
    }
    uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                      ((barrier ? 1 : 0) << HSA_PACKET_HEADER_BARRIER) |
                      (acq_scope << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                      ((last ? HSA_FENCE_SCOPE_SYSTEM : rel_scope) << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
    const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
    __atomic_store_n(reinterpret_cast<uint32_t*>(p), (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
    hsa_signal_store_screlease(q->doorbell_signal, idx);
  }
  void wait() {
    while (hsa_signal_wait_scacquire(done, HSA_SIGNAL_CONDITION_LT, 1, 5000000000ull, HSA_WAIT_STATE_ACTIVE) >= 1) {
      fprintf(stderr, "AQL wait timed out\n");
      exit(2);
    }
  }
};

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const char* hsaco = argc > 1 ? argv[1] : "tools/aql_probe.hsaco";
  HC(hipSetDevice(0));
  Aql A;
  A.init(hsaco);
  const Kern kspin = A.get("p_spin"), kmark = A.get("p_mark"), knode = A.get("p_node"), kempty = A.get("p_empty"),
             ks8 = A.get("p_stream8"), ks2 = A.get("p_stream2"), ks8r = A.get("p_stream8r");
  printf("kernarg sizes: spin %u mark %u node %u stream %u; group %u priv %u\n", kspin.kargs, kmark.kargs, knode.kargs,
         ks8.kargs, ks8.group, ks8.priv);

  unsigned long long *ts_a, *ts_b;
  HC(hipMalloc(&ts_a, 2 * 8192 * 8));
  HC(hipMalloc(&ts_b, 8192 * 8));
  int* err;
  HC(hipMalloc(&err, 4));
  HC(hipMemset(err, 0, 4));
  std::vector<unsigned long long> ha(2 * 8192), hb(8192);

  auto report_overlap = [&](const char* tag, int nspin, int nmark) {
    HC(hipMemcpy(ha.data(), ts_a, 2 * nspin * 8, hipMemcpyDeviceToHost));
    HC(hipMemcpy(hb.data(), ts_b, nmark * 8, hipMemcpyDeviceToHost));
    unsigned long long s_min = ~0ull, s_last_start = 0, s_end = 0, m_min = ~0ull, m_max = 0;
    for (int i = 0; i < nspin; ++i) {
      s_min = std::min(s_min, ha[2 * i]);
      s_last_start = std::max(s_last_start, ha[2 * i]);
      s_end = std::max(s_end, ha[2 * i + 1]);
    }
    for (int i = 0; i < nmark; ++i) { m_min = std::min(m_min, hb[i]); m_max = std::max(m_max, hb[i]); }
    printf("%s: producer [%0.2f .. last start %0.2f .. end %0.2f] us; consumer first %0.2f last %0.2f us "
           "(relative to producer first start) -> %s\n",
           tag, 0.0, (s_last_start - s_min) / 100.0, (s_end - s_min) / 100.0, ((double)m_min - s_min) / 100.0,
           ((double)m_max - s_min) / 100.0, m_min < s_end ? "OVERLAP" : "serialised");
  };

  // ---- T0: HIP eager + hipExtAnyOrderLaunch
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(p_spin, dim3(256), dim3(256), 0, 0, ts_a, 5000);
    hipExtLaunchKernelGGL(p_mark, dim3(256), dim3(256), 0, 0, nullptr, nullptr, hipExtAnyOrderLaunch, ts_b);
    HC(hipDeviceSynchronize());
    if (rep == 2) report_overlap("T0 HIP hipExtAnyOrderLaunch", 256, 256);
  }

  // ---- T1: HSA barrier 0 after a 256-WG spinner (50 us)
  for (int barrier = 1; barrier >= 0; --barrier)
    for (int rep = 0; rep < 3; ++rep) {
      A.reset();
      struct { unsigned long long* ts; int ticks; } a1 = {ts_a, 5000};
      struct { unsigned long long* ts; } a2 = {ts_b};
      void* k1 = A.karg(&a1, sizeof a1, kspin);
      void* k2 = A.karg(&a2, sizeof a2, kmark);
      A.upload();
      A.dispatch(kspin, k1, 256, true, false);
      A.dispatch(kmark, k2, 256, barrier != 0, true);
      A.wait();
      if (rep == 2) report_overlap(barrier ? "T1 HSA barrier=1" : "T1 HSA barrier=0", 256, 256);
    }

  // ---- T2: dispatch order with a 4096-WG producer (20 us each)
  for (int rep = 0; rep < 3; ++rep) {
    A.reset();
    struct { unsigned long long* ts; int ticks; } a1 = {ts_a, 2000};
    struct { unsigned long long* ts; } a2 = {ts_b};
    void* k1 = A.karg(&a1, sizeof a1, kspin);
    void* k2 = A.karg(&a2, sizeof a2, kmark);
    A.upload();
    A.dispatch(kspin, k1, 4096, true, false);
    A.dispatch(kmark, k2, 256, false, true);
    A.wait();
    if (rep == 2) {
      report_overlap("T2 HSA 4096-WG producer, consumer barrier=0", 4096, 256);
      HC(hipMemcpy(ha.data(), ts_a, 2 * 4096 * 8, hipMemcpyDeviceToHost));
      HC(hipMemcpy(hb.data(), ts_b, 256 * 8, hipMemcpyDeviceToHost));
      unsigned long long last_start = 0, m_min = ~0ull;
      for (int i = 0; i < 4096; ++i) last_start = std::max(last_start, ha[2 * i]);
      for (int i = 0; i < 256; ++i) m_min = std::min(m_min, hb[i]);
      int early = 0;
      for (int i = 0; i < 4096; ++i) early += ha[2 * i] > m_min;
      printf("T2 producer workgroups that started after the consumer's first: %d of 4096 (%s)\n", early,
             early ? "grids interleave" : "in-order grid dispatch");
    }
  }

  // ---- T3: chain of N trivial dependent kernels
  const int N = 384;
  unsigned* cnt;
  const size_t cnt_words = (size_t)(N + 1) * 256;
  HC(hipMalloc(&cnt, cnt_words * 4));
  for (int rep = 0; rep < 3; ++rep) {
    A.reset();
    struct { int* d; } ae = {nullptr};
    void* ke = A.karg(&ae, sizeof ae, kempty);
    A.upload();
    const double t0 = now_us();
    for (int i = 0; i < N; ++i) A.dispatch(kempty, ke, 256, true, i == N - 1);
    A.wait();
    const double t1 = now_us();
    if (rep == 2) printf("T3 HSA barrier chain of %d empty kernels: %.2f us per node\n", N, (t1 - t0) / N);
  }
  {
    hipStream_t s;
    HC(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipGraph_t g;
    hipGraphExec_t ge;
    HC(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(p_empty, dim3(256), dim3(256), 0, s, (int*)nullptr);
    HC(hipStreamEndCapture(s, &g));
    HC(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int rep = 0; rep < 3; ++rep) {
      const double t0 = now_us();
      HC(hipGraphLaunch(ge, s));
      HC(hipStreamSynchronize(s));
      const double t1 = now_us();
      if (rep == 2) printf("T3 hipGraph chain of %d empty kernels: %.2f us per node\n", N, (t1 - t0) / N);
    }
    HC(hipGraphExecDestroy(ge));
    HC(hipGraphDestroy(g));
    HC(hipStreamDestroy(s));
  }

  // ---- T4: counter chain, barrier 0
  for (int rep = 0; rep < 3; ++rep) {
    HC(hipMemset(cnt, 0, cnt_words * 4));
    A.reset();
    std::vector<void*> ka(N);
    for (int i = 0; i < N; ++i) {
      struct { const unsigned* prev; unsigned target; unsigned* own; int* err; } a = {
          i ? cnt + (size_t)(i - 1) * 256 : nullptr, 256u, cnt + (size_t)i * 256, err};
      ka[i] = A.karg(&a, sizeof a, knode);
    }
    A.upload();
    const double t0 = now_us();
    for (int i = 0; i < N; ++i) A.dispatch(knode, ka[i], 256, i == 0, i == N - 1);
    A.wait();
    const double t1 = now_us();
    int herr = 0;
    HC(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    if (rep == 2) printf("T4 HSA barrier-0 counter chain of %d: %.2f us per node (poll timeouts %d)\n", N,
                         (t1 - t0) / N, herr);
  }

  // ---- T5: streaming chain
  const size_t wmax = (size_t)N * 256 * 256 * 8 * 16;  // N nodes x 256 WGs x 256 thr x 8 x 16 B = 3.2 GB at N=384
  const int NS = 192;
  const size_t wbytes = (size_t)NS * 256 * 256 * 8 * 16;
  (void)wmax;
  char* W;
  HC(hipMalloc(&W, wbytes));
  unsigned* rdyb;
  HC(hipMalloc(&rdyb, (size_t)(NS + 1) * 512 * 4));
  HC(hipMemset(rdyb, 0, (size_t)(NS + 1) * 512 * 4));
  HC(hipMemset(W, 1, wbytes));
  float* act;  // NS + 1 activation buffers of 256 KB (only the first 32 KB x 8 slices are read)
  HC(hipMalloc(&act, (size_t)(NS + 1) * 65536 * 4));
  HC(hipMemset(act, 0, (size_t)(NS + 1) * 65536 * 4));
  for (int wb : {8, 2}) {
    const Kern& ks = wb == 8 ? ks8 : ks2;
    for (int mode = 0; mode < 2; ++mode)
      for (int rep = 0; rep < 4; ++rep) {
        HC(hipMemset(cnt, 0, cnt_words * 4));
        HC(hipMemset(err, 0, 4));
        A.reset();
        std::vector<void*> ka(NS);
        for (int i = 0; i < NS; ++i) {
          struct { const void* W; const float* X; float* Y; const unsigned* prev; unsigned target; unsigned* own;
                   int* err; int ov; } a = {
              W + (size_t)i * 256 * 256 * wb * 16, act + (size_t)i * 65536, act + (size_t)(i + 1) * 65536,
              mode && i ? cnt + (size_t)(i - 1) * 256 : nullptr, 256u, mode ? cnt + (size_t)i * 256 : nullptr, err,
              mode && i ? 1 : 0};
          ka[i] = A.karg(&a, sizeof a, ks);
        }
        A.upload();
        const double t0 = now_us();
        for (int i = 0; i < NS; ++i) A.dispatch(ks, ka[i], 256, mode == 0 || i == 0, i == NS - 1);
        A.wait();
        const double t1 = now_us();
        int herr = 0;
        HC(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
        if (rep == 3)
          printf("T5 stream chain (W %d KB/WG, X 16 KB/WG, Y 1 KB/WG) %s: %.2f us per node (poll timeouts %d)\n",
                 wb * 4, mode ? "barrier-0 + prefetch + counter" : "barrier-1 one round trip", (t1 - t0) / NS, herr);
      }
  }
  // ---- T6: two queues: producer spinning on queue 0, consumer on queue 1
  for (int rep = 0; rep < 3; ++rep) {
    A.reset();
    struct { unsigned long long* ts; int ticks; } a1 = {ts_a, 5000};
    struct { unsigned long long* ts; } a2 = {ts_b};
    void* k1 = A.karg(&a1, sizeof a1, kspin);
    void* k2 = A.karg(&a2, sizeof a2, kmark);
    A.upload();
    A.dispatch(kspin, k1, 256, true, false, 0);
    A.dispatch(kmark, k2, 256, true, false, 1);
    HC(hipDeviceSynchronize());
    // wait for both: poll the queues' read indices is not enough; sleep generously
    const double t0 = now_us();
    while (now_us() - t0 < 2000) {}
    if (rep == 2) report_overlap("T6 two queues (spin on q0, mark on q1)", 256, 256);
  }
  // ---- T7: counter chain alternating over NQ queues
  for (int nq : {2, 3, 4})
    for (int rep = 0; rep < 3; ++rep) {
      HC(hipMemset(cnt, 0, cnt_words * 4));
      HC(hipMemset(err, 0, 4));
      A.reset();
      std::vector<void*> ka(N);
      for (int i = 0; i < N; ++i) {
        struct { const unsigned* prev; unsigned target; unsigned* own; int* err; } a = {
            i ? cnt + (size_t)(i - 1) * 256 : nullptr, 256u, cnt + (size_t)i * 256, err};
        ka[i] = A.karg(&a, sizeof a, knode);
      }
      A.upload();
      const double t0 = now_us();
      for (int i = 0; i < N; ++i) A.dispatch(knode, ka[i], 256, true, i == N - 1, i % nq);
      A.wait();
      const double t1 = now_us();
      int herr = 0;
      HC(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
      if (rep == 2) printf("T7 counter chain over %d queues: %.2f us per node (poll timeouts %d)\n", nq, (t1 - t0) / N, herr);
    }
  // ---- T8: streaming chain alternating over NQ queues
  for (int wb : {8, 2}) {
    const Kern& ks = wb == 8 ? ks8 : ks2;
    for (int nq : {2, 3})
      for (int rep = 0; rep < 4; ++rep) {
        HC(hipMemset(cnt, 0, cnt_words * 4));
        HC(hipMemset(err, 0, 4));
        A.reset();
        std::vector<void*> ka(NS);
        for (int i = 0; i < NS; ++i) {
          struct { const void* W; const float* X; float* Y; const unsigned* prev; unsigned target; unsigned* own;
                   int* err; int ov; } a = {
              W + (size_t)i * 256 * 256 * wb * 16, act + (size_t)i * 65536, act + (size_t)(i + 1) * 65536,
              i ? cnt + (size_t)(i - 1) * 256 : nullptr, 256u, cnt + (size_t)i * 256, err, i ? 1 : 0};
          ka[i] = A.karg(&a, sizeof a, ks);
        }
        A.upload();
        const double t0 = now_us();
        for (int i = 0; i < NS; ++i) A.dispatch(ks, ka[i], 256, true, i == NS - 1, i % nq);
        A.wait();
        const double t1 = now_us();
        int herr = 0;
        HC(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
        if (rep == 3)
          printf("T8 stream chain (W %d KB/WG) over %d queues, prefetch + counter: %.2f us per node (poll timeouts %d)\n",
                 wb * 4, nq, (t1 - t0) / NS, herr);
      }
  }
  // ---- T9: fence scopes on a barrier chain (empty kernels and streaming nodes)
  {
    const int scopes[][2] = {{HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_AGENT}, {HSA_FENCE_SCOPE_NONE, HSA_FENCE_SCOPE_NONE},
                             {HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_NONE}, {HSA_FENCE_SCOPE_NONE, HSA_FENCE_SCOPE_AGENT},
                             {HSA_FENCE_SCOPE_SYSTEM, HSA_FENCE_SCOPE_SYSTEM}};
    for (auto& sc : scopes) {
      A.acq_scope = sc[0];
      A.rel_scope = sc[1];
      double te = 0, tsn = 0;
      for (int rep = 0; rep < 3; ++rep) {
        A.reset();
        struct { int* d; } ae = {nullptr};
        void* ke = A.karg(&ae, sizeof ae, kempty);
        A.upload();
        const double t0 = now_us();
        for (int i = 0; i < N; ++i) A.dispatch(kempty, ke, 256, true, i == N - 1);
        A.wait();
        te = (now_us() - t0) / N;
      }
      for (int rep = 0; rep < 3; ++rep) {
        A.reset();
        std::vector<void*> ka(NS);
        for (int i = 0; i < NS; ++i) {
          struct { const void* W; const float* X; float* Y; const unsigned* prev; unsigned target; unsigned* own;
                   int* err; int ov; } a = {W + (size_t)i * 256 * 256 * 8 * 16, act + (size_t)i * 65536,
                                            act + (size_t)(i + 1) * 65536, nullptr, 256u, nullptr, err, 0};
          ka[i] = A.karg(&a, sizeof a, ks8);
        }
        A.upload();
        const double t0 = now_us();
        for (int i = 0; i < NS; ++i) A.dispatch(ks8, ka[i], 256, true, i == NS - 1);
        A.wait();
        tsn = (now_us() - t0) / NS;
      }
      printf("T9 fences acquire %d release %d: empty chain %.2f us/node, stream chain (32 KB W) %.2f us/node\n", sc[0],
             sc[1], te, tsn);
    }
    A.acq_scope = HSA_FENCE_SCOPE_AGENT;
    A.rel_scope = HSA_FENCE_SCOPE_AGENT;
  }
  // ---- T10: two-queue streaming chain with replicated ready flags
  for (int sl = 0; sl < 2; ++sl)
    for (int rep = 0; rep < 4; ++rep) {
      HC(hipMemset(cnt, 0, cnt_words * 4));
      HC(hipMemset(err, 0, 4));
      A.reset();
      // counter i at cnt + i*256, ready flags of i at cnt + (N + 1 + ...) -> use a second region
      std::vector<void*> ka(NS);
      for (int i = 0; i < NS; ++i) {
        unsigned* rdy = cnt + (size_t)i * 256 + 32;  // 16 replicas x 32 words would overlap: use 8 words stride
        (void)rdy;
        struct { const void* W; const float* X; float* Y; const unsigned* prev_ready; unsigned* own_cnt;
                 unsigned* own_ready; int* err; int sleep; } a = {
            W + (size_t)i * 256 * 256 * 8 * 16, act + (size_t)i * 65536, act + (size_t)(i + 1) * 65536,
            i ? rdyb + (size_t)(i - 1) * 512 : nullptr, cnt + (size_t)i * 256, rdyb + (size_t)i * 512, err, sl};
        ka[i] = A.karg(&a, sizeof a, ks8r);
      }
      A.upload();
      const double t0 = now_us();
      for (int i = 0; i < NS; ++i) A.dispatch(ks8r, ka[i], 256, true, i == NS - 1, i % 2);
      A.wait();
      const double t1 = now_us();
      int herr = 0;
      HC(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
      if (rep == 3)
        printf("T10 stream chain (W 32 KB/WG) over 2 queues, ready replicas, sleep %d: %.2f us per node (poll timeouts %d)\n",
               sl ? 4 : 1, (t1 - t0) / NS, herr);
      HC(hipMemset(rdyb, 0, (size_t)(NS + 1) * 512 * 4));
    }
  printf("done\n");
  return 0;
}
