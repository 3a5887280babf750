// Checks that the LDS-free wave reductions of wh_common.h (permlane swaps + DPP row
// rotations) return exactly the bits of the __shfl_xor butterfly they replace, on every
// lane, for random, tied, signed-zero, infinite and denormal inputs; and that the
// argbest (value desc, index asc) of wh_decode.hip's form matches a host scan.
//   make -C whisper.coreml_amd tools/wave_reduce_check && whisper.coreml_amd/tools/wave_reduce_check
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "wh_common.h"



__device__ __forceinline__ bool better_t(float a, int ia, float b, int ib) { return a > b || (a == b && ia < ib); }

__device__ void argbest_new(float& v, int& idx) {
  {
    float a = v, b = v;
    int ia = idx, ib = idx;
    perm32_pair(a, b);
    perm32_pair(ia, ib);
    const bool t = (b > a) | ((b == a) & (ib < ia));  // better(b, a) without a branch: full EXEC below
    v = t ? b : a;
    idx = t ? ib : ia;
  }
  {
    float a = v, b = v;
    int ia = idx, ib = idx;
    perm16_pair(a, b);
    perm16_pair(ia, ib);
    const bool t = (b > a) | ((b == a) & (ib < ia));  // better(b, a) without a branch: full EXEC below
    v = t ? b : a;
    idx = t ? ib : ia;
  }
  auto step = [&](float ov, int oi) {
    const bool t = (ov > v) | ((ov == v) & (oi < idx));
    v = t ? ov : v;
    idx = t ? oi : idx;
  };
  step(dpp_f<DPP_ROR8>(v), dpp_i<DPP_ROR8>(idx));
  step(dpp_f<DPP_ROR4>(v), dpp_i<DPP_ROR4>(idx));
  step(dpp_f<DPP_ROR2>(v), dpp_i<DPP_ROR2>(idx));
  step(dpp_f<DPP_ROR1>(v), dpp_i<DPP_ROR1>(idx));
}

__device__ void argbest_xor(float& v, int& idx) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(idx, o, 64);
    if (better_t(ov, oi, v, idx)) { v = ov; idx = oi; }
  }
}

// out[4 * i + 0..3]: sum_new, sum_xor, max_new, max_xor per lane; ai: argbest value / index
__global__ void k_check(const float* in, const int* ix, float* out, float* av, int* ai, float* av2, int* ai2) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  const float x = in[i];
  out[4 * i + 0] = wave_sum(x);
  out[4 * i + 1] = wave_sum_xor(x);
  out[4 * i + 2] = wave_max(x);
  out[4 * i + 3] = wave_max_xor(x);
  float v = x;
  int id = ix[i];
  argbest_new(v, id);
  av[i] = v;
  ai[i] = id;
  v = x;
  id = ix[i];
  argbest_xor(v, id);
  av2[i] = v;
  ai2[i] = id;
}

// the single butterfly steps: out[10 * i + 2k] new form, out[10 * i + 2k + 1] __shfl_xor form
__global__ void k_steps(const float* in, float* out) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  const float x = in[i];
  float* o = out + 10 * i;
  o[0] = xor8_sum(x);  o[1] = x + __shfl_xor(x, 8, 64);
  o[2] = xor16_sum(x); o[3] = x + __shfl_xor(x, 16, 64);
  o[4] = xor32_sum(x); o[5] = x + __shfl_xor(x, 32, 64);
  o[6] = xor16_max(x); o[7] = fmaxf(x, __shfl_xor(x, 16, 64));
  o[8] = xor32_max(x); o[9] = fmaxf(x, __shfl_xor(x, 32, 64));
}

int main() {
  const int waves = 1 << 14, n = waves * 64;
  std::vector<float> h(n);
  std::vector<int> hi(n);
  std::mt19937 rng(7);
  std::normal_distribution<float> nd(0.f, 10.f);
  for (int w = 0; w < waves; ++w)
    for (int l = 0; l < 64; ++l) {
      float x = nd(rng);
      switch (w % 8) {
        case 1: x = std::round(x); break;                        // ties
        case 2: x = (l & 1) ? 0.f : -0.f; break;                 // signed zeros
        case 3: if (l == w % 64) x = -INFINITY; break;
        case 4: x = x * 1e-39f; break;                           // denormals
        case 5: x = (l % 7 == 0) ? -INFINITY : x; break;
        case 6: x = x * 1e30f; break;                            // overflow to inf in sums
        default: break;
      }
      h[w * 64 + l] = x;
      // distinct indices within a wave (vocabulary ids): in wave-order or shuffled
      hi[w * 64 + l] = (w % 3 == 0) ? l : (int)((l * 7919 + w * 131) % 1000003);
    }
  float *din, *dout, *dav, *dav2;
  int *dix, *dai, *dai2;
  (void)hipMalloc(&din, n * 4); (void)hipMalloc(&dix, n * 4); (void)hipMalloc(&dout, n * 16);
  (void)hipMalloc(&dav, n * 4); (void)hipMalloc(&dai, n * 4); (void)hipMalloc(&dav2, n * 4); (void)hipMalloc(&dai2, n * 4);
  (void)hipMemcpy(din, h.data(), n * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dix, hi.data(), n * 4, hipMemcpyHostToDevice);
  k_check<<<waves, 64>>>(din, dix, dout, dav, dai, dav2, dai2);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 2; }
  std::vector<float> o(n * 4), av(n), av2(n);
  std::vector<int> ai(n), ai2(n);
  (void)hipMemcpy(o.data(), dout, n * 16, hipMemcpyDeviceToHost);
  (void)hipMemcpy(av.data(), dav, n * 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(ai.data(), dai, n * 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(av2.data(), dav2, n * 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(ai2.data(), dai2, n * 4, hipMemcpyDeviceToHost);
  float* dst;
  (void)hipMalloc(&dst, (size_t)n * 40);
  k_steps<<<waves, 64>>>(din, dst);
  std::vector<float> so((size_t)n * 10);
  (void)hipMemcpy(so.data(), dst, (size_t)n * 40, hipMemcpyDeviceToHost);
  long bad_steps = 0;
  for (size_t i = 0; i < (size_t)n * 5; ++i)
    if (std::memcmp(&so[2 * i], &so[2 * i + 1], 4) && !(std::isnan(so[2 * i]) && std::isnan(so[2 * i + 1]))) ++bad_steps;
  long bad_vs_xor = 0;
  for (int i = 0; i < n; ++i)
    if (ai[i] != ai2[i] || std::memcmp(&av[i], &av2[i], 4)) ++bad_vs_xor;
  long bad_sum = 0, bad_max = 0, bad_arg = 0;
  for (int i = 0; i < n; ++i) {
    if (std::memcmp(&o[4 * i], &o[4 * i + 1], 4) && !(std::isnan(o[4 * i]) && std::isnan(o[4 * i + 1]))) ++bad_sum;
    if (std::memcmp(&o[4 * i + 2], &o[4 * i + 3], 4)) ++bad_max;
  }
  for (int w = 0; w < waves; ++w) {
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int l = 0; l < 64; ++l) {
      const float x = h[w * 64 + l];
      const int id = hi[w * 64 + l];
      if (x > bv || (x == bv && id < bi)) { bv = x; bi = id; }
    }
    for (int l = 0; l < 64; ++l)
      if (ai[w * 64 + l] != bi || std::memcmp(&av[w * 64 + l], &bv, 4)) { ++bad_arg; break; }
  }
  printf("%d waves: wave_sum mismatches %ld, wave_max mismatches %ld, argbest waves wrong %ld, argbest lanes != "
         "xor form %ld, single steps %ld\n", waves, bad_sum, bad_max, bad_arg, bad_vs_xor, bad_steps);
  return bad_sum || bad_max || bad_arg || bad_vs_xor || bad_steps ? 1 : 0;
}
