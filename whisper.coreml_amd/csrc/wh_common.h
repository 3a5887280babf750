// Common device/host helpers for libwhisper_hip (gfx950 / CDNA4 only).
//
// Element types: the hot path is templated on T in {float, half_t}.  half_t is
// the fp16 production path (weights + activations fp16, fp32 accumulate, fp32
// residual stream); float is the parity path that matches the reference CPU
// fp32 model token-for-token.
//
// MFMA fragment convention used by every GEMM / attention kernel here
// (16x16 output tiles, wave64):
//   lane l, row index r = l & 15, k-group g = l >> 4
//   a "k-step" covers 32 consecutive k; lane (r, g) holds the 8 elements
//   k = 32*s + 8*g + j (j = 0..7) of its row.
//   * half_t : one v_mfma_f32_16x16x32_f16 per k-step
//   * float  : eight v_mfma_f32_16x16x4_f32 per k-step, step j feeding k = 8g + j
//     (the k order inside a step is permuted identically for A and B, so the
//     sum is the same contraction).
//   D layout (both): lane holds D[row = 4*g + j][col = r], j = 0..3.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef _Float16 half_t;
typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
typedef float float4_t __attribute__((ext_vector_type(4)));
typedef float float8_t __attribute__((ext_vector_type(8)));

#define WH_DEV __device__ __forceinline__
#define WH_DEV_HOST __host__ __device__ __forceinline__

// Tuning switches (WHISPER_HIP_* environment variables that select measured-but-not-
// adopted kernel variants for A/B runs) are read only by the tuning build
// (`make tune` -> lib/libwhisper_hip_tune.so, loaded with WHISPER_HIP_LIB).  The shipped
// library ignores the environment: every variant it can run is the tested default.
#ifndef WH_TUNING
#define WH_TUNING 0
#endif
#include <stdlib.h>
static inline const char* tune_env(const char* name) {
#if WH_TUNING
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

// ---------------------------------------------------------------- launch attribution
// Every kernel launch site is `kernel<<<...>>>(...), wh_launched("kernel");`: the name of
// the thread's last launch is kept, so a launch error that surfaces later (the entry
// points check hipGetLastError() once, after their launches) names the launch before it.
// The tuning build also checks hipGetLastError() after EVERY launch and keeps the first
// failing launch's name and error (wh_first_launch_error), so the error is attributed to
// the launch that raised it, not to the entry point that noticed.
#include <string>
inline const char*& wh_last_launch() {
  static thread_local const char* name = "(none)";
  return name;
}
inline std::string& wh_first_launch_error() {
  static thread_local std::string err;
  return err;
}
inline void wh_launched(const char* name) {
  wh_last_launch() = name;
#if WH_TUNING
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess && wh_first_launch_error().empty())
    wh_first_launch_error() = std::string("launch of ") + name + ": " + hipGetErrorString(e);
#endif
}
// a launcher that refuses its operands records why (surfaces at the entry point's check)
inline void wh_set_launch_error(const char* msg) {
  if (wh_first_launch_error().empty()) wh_first_launch_error() = msg;
}

// Chain trace (tuning build only, profiles/chain_trace.py): per-workgroup wall-clock marks
// (s_memrealtime, 100 MHz) of the decoder-step kernels, one slot per kernel role; every
// launch of a role overwrites its slot, so after one step a slot holds that role's LAST
// launch (layer 31's).  Mark 0 = workgroup start, 1 / 2 = kernel-specific phase ends,
// 3 = thread 0 done (its stores drained).  Each translation unit has its own copy of the
// array (static) and reader (WH_CT_READER); the slots of one role live in one unit.
constexpr int CT_SLOTS = 12, CT_WG = 2048;
enum { CT_PROJ_QKV = 0, CT_PROJ_NN = 1, CT_PROJ_FC1 = 2, CT_PROJ_FC2 = 3, CT_RESID_LN = 4, CT_REDUCE = 5,
       CT_SELF_ATTN = 6, CT_XATTN = 7, CT_VOCAB = 8, CT_LOGIT = 9, CT_MERGE = 10,
       CT_LOGIT_SLICE = 11 };  // k_logit_part slice phases: 0 loads landed, 1 top-k, 2 record stored, 3 arrived
#if WH_TUNING
static __device__ unsigned long long g_ct_trace[CT_SLOTS][CT_WG][4];
#define CT_MARK(slot, k)                                                                 \
  do {                                                                                   \
    const unsigned ct_b_ = blockIdx.x + blockIdx.y * gridDim.x;                          \
    if (threadIdx.x == 0 && ct_b_ < (unsigned)CT_WG)                                     \
      g_ct_trace[slot][ct_b_][k] = __builtin_amdgcn_s_memrealtime();                     \
  } while (0)
#define CT_END(slot)                                       \
  do {                                                     \
    if (threadIdx.x == 0) {                                \
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     \
      CT_MARK(slot, 3);                                    \
    }                                                      \
  } while (0)
#define WH_CT_READER(name)                                                                        \
  extern "C" int wh_tune_ct_trace_##name(unsigned long long* out) {                              \
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ct_trace), sizeof(g_ct_trace)) == hipSuccess ? 0 : -1; \
  }                                                                                               \
  extern "C" int wh_tune_ct_clear_##name() {                                                      \
    static unsigned long long z[CT_SLOTS][CT_WG][4];                                              \
    return hipMemcpyToSymbol(HIP_SYMBOL(g_ct_trace), z, sizeof(z)) == hipSuccess ? 0 : -1;        \
  }
#else
#define CT_MARK(slot, k) \
  do {                   \
  } while (0)
#define CT_END(slot) \
  do {               \
  } while (0)
#define WH_CT_READER(name)
#endif

// cross-V (V^T) of a (window, head) is TILE-MAJOR: [TKP / 64 tiles][64 d][64 keys, 32-key permutation],
// so one 64-key tile's V^T is 8 KB contiguous (one stream, like K's [TKP][64] rows); element (d, t)
// sits at xv_index(d, t).
// 2^x as the bare v_exp_f32 (exp2f adds a denormal-range rescale: 5 more instructions per
// call).  Softmax uses only: a result below 2^-126 is flushed instead of kept denormal,
// which leaves every fp16 probability (min subnormal 2^-24) and every fp32 sum that
// includes the row maximum's 1 unchanged.
WH_DEV float hw_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
// workgroup barrier for LDS data only: waits for this wave's LDS operations, never for its
// global loads / stores in flight.  (__syncthreads is a workgroup-scope release + acquire;
// hipcc decides per site whether that needs a vmcnt wait — in k_resid_ln it emits none,
// in the fused selection it emitted some; this form does not depend on that choice.)
WH_DEV void wh_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// floor(b * n / nb) of a contiguous range split (workgroup b of nb takes [split(b), split(b + 1))),
// in 32-bit unsigned arithmetic: b * n < 2^32 at every call site (<= 256 workgroups x
// < 2^24 units).  The int64 form is a ~140-instruction scalar divide ahead of the first load.
WH_DEV int range_split(int b, int n, int nb) { return (int)(((unsigned)b * (unsigned)n) / (unsigned)nb); }
typedef float f32x2_t __attribute__((ext_vector_type(2)));  // packed fp32 (v_pk_add_f32 / v_pk_mul_f32)

WH_DEV_HOST int xv_perm(int t) {
  const int q = t & 31;
  return (t & ~31) + 8 * ((q & 15) >> 2) + 4 * (q >> 4) + (q & 3);
}
WH_DEV_HOST int64_t xv_index(int d, int t) { return ((int64_t)(t >> 6) * 64 + d) * 64 + xv_perm(t & 63); }

// ---------------------------------------------------------------- fragments
template <typename T> struct Frag;
template <> struct Frag<half_t> { half8_t v; };
template <> struct Frag<float> { float8_t v; };

// load 8 consecutive elements (16 B for half, 32 B for float)
WH_DEV void frag_load(Frag<half_t>& f, const half_t* p) { f.v = *reinterpret_cast<const half8_t*>(p); }
WH_DEV void frag_load(Frag<float>& f, const float* p) {
  const float4_t* q = reinterpret_cast<const float4_t*>(p);
  float4_t a = q[0], b = q[1];
  f.v = (float8_t){a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// once-read streams (decode weights, cross-K/V): nontemporal loads when built with
// WH_NT=1 (MI355X_MICROARCH.md "nt-weights")
#ifndef WH_NT
#define WH_NT 0
#endif
WH_DEV void frag_load_stream(Frag<half_t>& f, const half_t* p) {
#if WH_NT
  f.v = __builtin_nontemporal_load(reinterpret_cast<const half8_t*>(p));
#else
  frag_load(f, p);
#endif
}
WH_DEV void frag_load_stream(Frag<float>& f, const float* p) {
#if WH_NT
  const float4_t* q = reinterpret_cast<const float4_t*>(p);
  float4_t a = __builtin_nontemporal_load(q), b = __builtin_nontemporal_load(q + 1);
  f.v = (float8_t){a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
#else
  frag_load(f, p);
#endif
}

// 8 consecutive elements at byte offset `off` (< 2^31) of a buffer resource (wt_rsrc):
// 32-bit address arithmetic instead of a 64-bit multiply chain per load
template <typename R>
WH_DEV void frag_load_buf(Frag<half_t>& f, R rs, int off) {
  f.v = __builtin_bit_cast(half8_t, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
}
template <typename R>
WH_DEV void frag_load_buf(Frag<float>& f, R rs, int off) {
  const float4_t a = __builtin_bit_cast(float4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
  const float4_t b = __builtin_bit_cast(float4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 0));
  f.v = (float8_t){a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// two groups of 4 consecutive elements (8 B each for half, 16 B for float)
WH_DEV void load4x2(Frag<half_t>& f, const half_t* p0, const half_t* p1) {
  const half4_t a = *reinterpret_cast<const half4_t*>(p0), b = *reinterpret_cast<const half4_t*>(p1);
  f.v = (half8_t){a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}
WH_DEV void load4x2(Frag<float>& f, const float* p0, const float* p1) {
  const float4_t a = *reinterpret_cast<const float4_t*>(p0), b = *reinterpret_cast<const float4_t*>(p1);
  f.v = (float8_t){a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

WH_DEV void mfma_step(float4_t& acc, const Frag<half_t>& a, const Frag<half_t>& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a.v, b.v, acc, 0, 0, 0);
}
WH_DEV void mfma_step(float4_t& acc, const Frag<float>& a, const Frag<float>& b) {
#pragma unroll
  for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[j], b.v[j], acc, 0, 0, 0);
}

// ---------------------------------------------------------------- write-through stores
// Outputs the NEXT launch reads (split-K slabs, logits) are stored write-through (sc1):
// the kernel-end release then has no dirty L2 lines to write back, which otherwise
// lengthens the boundary by ~bytes / 6 TB/s (MI355X_MICROARCH.md price list,
// "boundary"; 100-row step: 3.68 -> 3.55 ms with the k_proj slabs write-through).
// base must be wave-uniform (a kernel argument); offsets in bytes, < 2^31.
#ifndef WH_WT
#define WH_WT 1
#endif
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
WH_DEV auto wt_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
template <typename R>
WH_DEV void wt_store1(R rs, int off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rs, off, 0, 16);
}
template <typename R>
WH_DEV void wt_store4(R rs, int off, float4_t v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rs, off, 0, 16);
}

// ---------------------------------------------------------------- conversions
template <typename T> WH_DEV T from_f32(float x);
template <> WH_DEV float from_f32<float>(float x) { return x; }
template <> WH_DEV half_t from_f32<half_t>(float x) { return (half_t)x; }
WH_DEV float to_f32(float x) { return x; }
WH_DEV float to_f32(half_t x) { return (float)x; }

// store 4 consecutive elements
WH_DEV void store4(float* p, float a, float b, float c, float d) {
  *reinterpret_cast<float4_t*>(p) = (float4_t){a, b, c, d};
}
WH_DEV void store4(half_t* p, float a, float b, float c, float d) {
  *reinterpret_cast<half4_t*>(p) = (half4_t){(half_t)a, (half_t)b, (half_t)c, (half_t)d};
}
WH_DEV float4_t load4f(const float* p) { return *reinterpret_cast<const float4_t*>(p); }
WH_DEV float4_t load4f(const half_t* p) {
  half4_t h = *reinterpret_cast<const half4_t*>(p);
  return (float4_t){(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
}

// exact-erf GELU (nn.GELU() default), evaluated in fp32
WH_DEV float gelu_f(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f)); }

// ---------------------------------------------------------------- wave reductions (wave64)
// The xor butterfly (partner lane i ^ 32, ^ 16, ^ 8, ^ 4, ^ 2, ^ 1) without LDS: the
// permlane swaps give every lane its i ^ 32 and i ^ 16 partner (v_permlane32_swap /
// v_permlane16_swap on two copies: one copy ends with the lower half / even rows, the
// other with the upper half / odd rows), then DPP row rotations by 8, 4, 2, 1 — after the
// earlier steps lanes i and i ^ 8 (then ^ 4, ^ 2) hold bit-equal values, so lane
// (i + k) mod 16 stands in for i ^ k.  Every lane adds the same two operands as in the
// __shfl_xor form (IEEE addition is commutative): bit-identical results, without the six
// dependent ds_bpermute round trips through the LDS crossbar.  Full-wave execution only
// (every caller is in wave-uniform control flow).
template <typename V>
WH_DEV void perm32_pair(V& a, V& b) {  // a, b = copies of v -> (lower half, upper half) values
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
template <typename V>
WH_DEV void perm16_pair(V& a, V& b) {  // a, b = copies of v -> (even rows, odd rows) values
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
template <int CTRL>
WH_DEV float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, true));
}
template <int CTRL>
WH_DEV int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, true);
}
constexpr int DPP_ROR8 = 0x128, DPP_ROR4 = 0x124, DPP_ROR2 = 0x122, DPP_ROR1 = 0x121;
WH_DEV float wave_sum(float v) {
  float a = v, b = v;
  perm32_pair(a, b);
  v = a + b;
  a = v; b = v;
  perm16_pair(a, b);
  v = a + b;
  v += dpp_f<DPP_ROR8>(v);
  v += dpp_f<DPP_ROR4>(v);
  v += dpp_f<DPP_ROR2>(v);
  v += dpp_f<DPP_ROR1>(v);
  return v;
}
WH_DEV float wave_max(float v) {
  // fmaxf(own, partner) as the butterfly orders it (the sign of a max of +-0 follows the
  // operand order)
  const int lane = __lane_id();
  float a = v, b = v;
  perm32_pair(a, b);
  v = (lane & 32) ? fmaxf(b, a) : fmaxf(a, b);
  a = v; b = v;
  perm16_pair(a, b);
  v = (lane & 16) ? fmaxf(b, a) : fmaxf(a, b);
  v = fmaxf(v, dpp_f<DPP_ROR8>(v));
  v = fmaxf(v, dpp_f<DPP_ROR4>(v));
  v = fmaxf(v, dpp_f<DPP_ROR2>(v));
  v = fmaxf(v, dpp_f<DPP_ROR1>(v));
  return v;
}
// single butterfly steps (partner lane i ^ 8 / ^ 16 / ^ 32), same operand order as
// `v op __shfl_xor(v, k)`: own value first
WH_DEV float xor8_sum(float v) { return v + dpp_f<DPP_ROR8>(v); }  // (i + 8) mod 16 == i ^ 8
WH_DEV float xor16_sum(float v) {
  float a = v, b = v;
  perm16_pair(a, b);
  return (__lane_id() & 16) ? b + a : a + b;
}
WH_DEV float xor32_sum(float v) {
  float a = v, b = v;
  perm32_pair(a, b);
  return (__lane_id() & 32) ? b + a : a + b;
}
WH_DEV float xor16_max(float v) {
  float a = v, b = v;
  perm16_pair(a, b);
  return (__lane_id() & 16) ? fmaxf(b, a) : fmaxf(a, b);
}
WH_DEV float xor32_max(float v) {
  float a = v, b = v;
  perm32_pair(a, b);
  return (__lane_id() & 32) ? fmaxf(b, a) : fmaxf(a, b);
}
// the __shfl_xor forms, for the equality test (tools/wave_reduce_check.hip)
WH_DEV float wave_sum_xor(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
WH_DEV float wave_max_xor(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ordered float <-> uint for atomicMax over signed floats
WH_DEV unsigned f2ord(float f) {
  unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
WH_DEV float ord2f(unsigned u) { return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u); }

// XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): blocks dealt round-robin over 8 XCDs get contiguous tile ranges.
WH_DEV int xcd_remap(int bid, int nwg) {
  if (nwg < 16) return bid;
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8, idx = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}
