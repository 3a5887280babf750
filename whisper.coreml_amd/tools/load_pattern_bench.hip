// Streaming-read rate of the two 16-B-per-lane access shapes the decode kernels use,
// on a buffer far larger than the Infinity Cache:
//   rows64 : an MFMA fragment load of a row-major [rows][128 B] matrix: lane (r = l & 15,
//            g = l >> 4) reads 16 B at row r, byte 16 g (+ 64 B for the second half) —
//            16 rows x 64 B per wave instruction (k_proj weights, cross-K / V^T tiles);
//   flat1k : the same bytes pre-arranged so one wave instruction reads 1 KB contiguous.
// grid: `wgs` workgroups of 256 threads, each streaming its contiguous share, `depth`
// loads per lane in flight.  Usage: load_pattern_bench [MB] [wgs] [reps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float float4_t __attribute__((ext_vector_type(4)));

template <int PAT, int DEPTH>
__global__ __launch_bounds__(256) void k_stream(const char* __restrict__ buf, size_t per_wg, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const char* base = buf + (size_t)blockIdx.x * per_wg;
  // a "tile" = 16 rows x 128 B = 2 KB = two wave instructions
  const size_t ntile = per_wg / 2048;
  float4_t acc = {0, 0, 0, 0};
  for (size_t t0 = (size_t)wave * DEPTH; t0 < ntile; t0 += 4 * DEPTH) {
    float4_t v[DEPTH][2];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const size_t t = t0 + d < ntile ? t0 + d : t0;
      const char* tp = base + t * 2048;
      if (PAT == 0) {
        const int r = lane & 15, g = lane >> 4;
        v[d][0] = *reinterpret_cast<const float4_t*>(tp + r * 128 + g * 16);
        v[d][1] = *reinterpret_cast<const float4_t*>(tp + r * 128 + 64 + g * 16);
      } else {
        v[d][0] = *reinterpret_cast<const float4_t*>(tp + lane * 16);
        v[d][1] = *reinterpret_cast<const float4_t*>(tp + 1024 + lane * 16);
      }
    }
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) acc += v[d][0] + v[d][1];
  }
  if (acc[0] == 123.456f) out[0] = acc[1];
}

template <int PAT, int DEPTH>
float run(const char* buf, size_t bytes, int wgs, int reps, float* out) {
  const size_t per = bytes / wgs / 2048 * 2048;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k_stream<PAT, DEPTH><<<wgs, 256>>>(buf, per, out);
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) k_stream<PAT, DEPTH><<<wgs, 256>>>(buf, per, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return (float)(per * wgs) * reps / (ms * 1e-3f) / 1e9f;
}

int main(int argc, char** argv) {
  const size_t mb = argc > 1 ? atol(argv[1]) : 2048;
  const int reps = argc > 3 ? atoi(argv[3]) : 10;
  const size_t bytes = mb << 20;
  char* buf = nullptr;
  float* out = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  if (hipMemset(buf, 1, bytes) != hipSuccess) return 1;
  const int wlist[] = {256, 512, 1024, 2048};
  for (int wgs : wlist) {
    printf("wgs %4d  rows64 d4 %6.0f d8 %6.0f | flat1k d4 %6.0f d8 %6.0f GB/s\n", wgs,
           run<0, 4>(buf, bytes, wgs, reps, out), run<0, 8>(buf, bytes, wgs, reps, out),
           run<1, 4>(buf, bytes, wgs, reps, out), run<1, 8>(buf, bytes, wgs, reps, out));
  }
  return 0;
}
