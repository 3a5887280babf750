// Word-level timestamps on the GPU: the numeric half of find_alignment
// (reference whisper/timing.py:163-231) and its DTW (timing.py:57-105).
//
//   k_align_softmax  softmax over the first F = num_frames/2 audio frames of every
//                    alignment head's raw cross q.k row (qk_scale = 1, timing.py:198-199)
//   k_align_znorm    per (head, frame): (w - mean) / std over the token rows, biased
//                    std (torch.std_mean(..., unbiased=False), timing.py:200-201)
//   k_align_medmean  median of 7 (reflect padding, timing.py:19-54) along frames, then
//                    the mean over heads (timing.py:204), rows [n_sot, n-1) only
//                    (timing.py:205) -> matrix [N][F]
//   k_dtw            dtw_cpu (timing.py:82-105) on x = -matrix: one workgroup sweeps the
//                    anti-diagonals (cell (i,j) needs only diagonals d-1 and d-2, kept in
//                    LDS; thread i owns row i and prefetches its x 8 diagonals ahead; the
//                    trace is 2-bit packed in LDS); costs are float32 cells fed by a float64 add exactly as the
//                    reference's float32 `cost` array fed from x.double(); ties resolve as
//                    its if/elif/else (c0 < c1 && c0 < c2 -> 0, c1 < c0 && c1 < c2 -> 1,
//                    else 2); then one lane walks the backtrace (timing.py:57-79)
//   k_token_probs    softmax over [:eot] of the rows that predict each text token,
//                    evaluated at that token (timing.py:187-191)
#include "wh_align.h"

#include <algorithm>
#include <cmath>

namespace wh {

__device__ __forceinline__ float blk_max(float v, float* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
  for (int i = 1; i < nw; ++i) r = fmaxf(r, red[i]);
  return r;
}
__device__ __forceinline__ float blk_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += red[i];
  return r;
}

// qk element (head h, token row t, frame f) at qk[h * hs + t * Tk + f]
// grid (rows, heads), block 256: w[h][t][f] = softmax_f(qk[h][t][f]), f < F (in place)
__global__ __launch_bounds__(256) void k_align_softmax(float* __restrict__ qk, int64_t hs, int Tk, int F) {
  __shared__ float red[4];
  float* row = qk + (int64_t)blockIdx.y * hs + (int64_t)blockIdx.x * Tk;
  float m = -INFINITY;
  for (int f = threadIdx.x; f < F; f += 256) m = fmaxf(m, row[f]);
  m = blk_max(m, red);
  float s = 0.f;
  for (int f = threadIdx.x; f < F; f += 256) s += expf(row[f] - m);
  s = blk_sum(s, red);
  for (int f = threadIdx.x; f < F; f += 256) row[f] = expf(row[f] - m) / s;
}

// grid (ceil(F/64), heads), block 256: 64 frames per block, the 4 waves split the
// token rows; per-frame sums combined in LDS in wave order
__global__ __launch_bounds__(256) void k_align_znorm(float* __restrict__ w, int64_t hs, int rows, int Tk, int F) {
  __shared__ float red[2][4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int f = blockIdx.x * 64 + lane;
  const bool ok = f < F;
  float* col = w + (int64_t)blockIdx.y * hs + (ok ? f : 0);
  float s = 0.f;
  for (int t = wv; t < rows; t += 4) s += col[(int64_t)t * Tk];
  red[0][wv][lane] = s;
  __syncthreads();
  const float mean = (red[0][0][lane] + red[0][1][lane] + red[0][2][lane] + red[0][3][lane]) / (float)rows;
  float q = 0.f;
  for (int t = wv; t < rows; t += 4) {
    const float d = col[(int64_t)t * Tk] - mean;
    q += d * d;
  }
  red[1][wv][lane] = q;
  __syncthreads();
  const float sd = sqrtf((red[1][0][lane] + red[1][1][lane] + red[1][2][lane] + red[1][3][lane]) / (float)rows);
  if (!ok) return;
  for (int t = wv; t < rows; t += 4) col[(int64_t)t * Tk] = (col[(int64_t)t * Tk] - mean) / sd;
}

// grid (ceil(F/256), N), block 256: matrix[t - t0][f] = mean_h median7(w[h][t][f-3..f+3])
__global__ __launch_bounds__(256) void k_align_medmean(const float* __restrict__ w, int64_t hs, int Tk, int F, int heads,
                                                       int t0, int width, float* __restrict__ mat) {
  const int f = blockIdx.x * 256 + threadIdx.x;
  const int t = t0 + blockIdx.y;
  if (f >= F) return;
  const int pad = width / 2;
  float acc = 0.f;
  for (int h = 0; h < heads; ++h) {
    const float* row = w + (int64_t)h * hs + (int64_t)t * Tk;
    float med;
    if (F <= pad) {
      med = row[f];  // timing.py:23-25: no filtering when the row is too short
    } else {
      float v[15];
      for (int d = 0; d < width; ++d) {
        int g = f + d - pad;
        if (g < 0) g = -g;
        if (g >= F) g = 2 * (F - 1) - g;
        v[d] = row[g];
      }
      // insertion sort of <= 15 values; the median is the middle one
      for (int a = 1; a < width; ++a) {
        const float x = v[a];
        int b = a - 1;
        while (b >= 0 && v[b] > x) { v[b + 1] = v[b]; --b; }
        v[b + 1] = x;
      }
      med = v[pad];
    }
    acc += med;
  }
  mat[(int64_t)blockIdx.y * F + f] = acc / (float)heads;
}

// one workgroup: DTW of x = sign * mat [N][M] and its backtrace.  Lane i owns row
// i (cell (i, d - i) of every anti-diagonal d); the per-diagonal body is branch-free
// (selects, clamped addresses) so the compiler's wait counters stay exact, and each
// lane prefetches its x values PF diagonals ahead (register ring, loop unrolled by
// PF) — only LDS traffic sits between two barriers.  The trace is packed 2 bits per
// cell: in LDS when it fits (LDS_TRACE, the backtrace then walks LDS), otherwise in
// the global scratch.  path: [2][N+M] (text indices, then time indices).
constexpr int DTW_THREADS = 1024;
constexpr int DTW_MAXN = 1023;
constexpr int DTW_PF = 8;
template <bool LDS_TRACE>
__global__ __launch_bounds__(DTW_THREADS) void k_dtw(const DtwJob* __restrict__ jobs, float sign) {
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  typedef __attribute__((address_space(1))) const float gfloat;
  typedef __attribute__((address_space(3))) unsigned lword;
  typedef __attribute__((address_space(1))) unsigned gword;
  const DtwJob jb = jobs[blockIdx.x];
  const int N = jb.N, M = jb.M;
  const int tid = threadIdx.x, i = tid;  // row
  const int DS = blockDim.x + 2;         // diagonal buffer stride (every lane writes its slot)
  if (N >= (int)blockDim.x) return;      // launch guard (host sizes the block to N + 1 rows)
  float* dg = reinterpret_cast<float*>(dsm);  // [3][DS]
  lword* ltrace = (lword*)(reinterpret_cast<unsigned*>(dsm + 3 * DS * 4));
  gword* gtr = (gword*)jb.trace;
  const int WPR = (M + 1 + 15) / 16;  // trace words per row
  for (int k = tid; k < 3 * DS; k += blockDim.x) dg[k] = INFINITY;
  __syncthreads();
  if (tid == 0) dg[0] = 0.f;  // diagonal 0: cost[0][0]
  // x ring: q[k] = mat[i-1][j-1] for the diagonal d with (d - 1) % PF == k (raw; sign
  // applied at use).  Addresses are clamped into the matrix, so every lane loads.
  const int ic = min(max(i, 1), N);
  gfloat* xr = (gfloat*)(jb.mat + (int64_t)(ic - 1) * M);
  auto xat = [&](int d) -> float { return xr[min(max(d - i, 1), M) - 1]; };
  float q[DTW_PF];
#pragma unroll
  for (int k = 0; k < DTW_PF; ++k) q[k] = xat(1 + k);
  unsigned tw = 0;  // trace word being filled by this row
  const int im1 = i > 0 ? i - 1 : 0;
  __syncthreads();
  for (int d0 = 1; d0 <= N + M; d0 += DTW_PF) {
#pragma unroll
    for (int k = 0; k < DTW_PF; ++k) {
      const int d = d0 + k;
      float* cur = dg + (d % 3) * DS;
      const float* p1 = dg + ((d + 2) % 3) * DS;  // d - 1
      const float* p2 = dg + ((d + 1) % 3) * DS;  // d - 2
      const int j = d - i;
      const bool inner = d <= N + M && i >= 1 && i <= N && j >= 1 && j <= M;
      const float c0 = p2[im1], c1 = p1[im1], c2 = p1[i];
      const bool t0 = c0 < c1 && c0 < c2, t1 = !t0 && c1 < c0 && c1 < c2;
      const float c = t0 ? c0 : (t1 ? c1 : c2);
      const unsigned t = t0 ? 0u : (t1 ? 1u : 2u);
      const float cost = (float)((double)(sign * q[k]) + (double)c);
      if (d <= N + M) cur[i] = inner ? cost : INFINITY;
      const int sh = (j & 15) * 2;
      tw = inner ? ((tw & ~(3u << sh)) | (t << sh)) : tw;
      if (inner && ((j & 15) == 15 || j == M)) {
        if constexpr (LDS_TRACE) ltrace[i * WPR + (j >> 4)] = tw;
        else gtr[i * WPR + (j >> 4)] = tw;
      }
      q[k] = xat(d + DTW_PF);
      // LDS-only barrier: __syncthreads() would also wait for the x prefetches
      // (vmcnt(0)), putting a global-load latency on every diagonal
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  }
  __syncthreads();
  if (tid != 0) return;
  // backtrace (timing.py:57-79): trace[0][:] = 2, trace[:][0] = 1
  int* path = jb.path;
  int a = N, b = M, n = 0;
  while (a > 0 || b > 0) {
    path[n] = a - 1;
    path[(N + M) + n] = b - 1;
    ++n;
    unsigned w = 0;
    if (a > 0 && b > 0) {
      if constexpr (LDS_TRACE) w = ltrace[a * WPR + (b >> 4)];
      else w = gtr[a * WPR + (b >> 4)];
    }
    const int t = a == 0 ? 2 : (b == 0 ? 1 : (int)((w >> ((b & 15) * 2)) & 3u));
    if (t == 0) { --a; --b; }
    else if (t == 1) { --a; }
    else { --b; }
  }
  for (int u = 0, v = n - 1; u < v; ++u, --v) {
    int x = path[u]; path[u] = path[v]; path[v] = x;
    x = path[(N + M) + u]; path[(N + M) + u] = path[(N + M) + v]; path[(N + M) + v] = x;
  }
  *jb.plen = n;
}

size_t dtw_trace_bytes(int N, int M) { return (size_t)(N + 1) * ((M + 1 + 15) / 16) * 4; }

constexpr size_t DTW_LDS = 160 * 1024;
static int dtw_threads(int max_n) { return std::min(DTW_THREADS, (max_n + 1 + 63) / 64 * 64); }

int dtw_prepare(DtwJob* jobs, int n, size_t* lds) {
  int max_n = 0;
  size_t tmax = 0;
  for (int k = 0; k < n; ++k) {
    const DtwJob& j = jobs[k];
    if (j.N < 1 || j.M < 1 || j.N > DTW_MAXN) return -1;
    max_n = std::max(max_n, j.N);
    tmax = std::max(tmax, dtw_trace_bytes(j.N, j.M));
  }
  const size_t diag = (size_t)3 * (dtw_threads(max_n) + 2) * 4;
  const bool in_lds = diag + tmax <= DTW_LDS;
  for (int k = 0; k < n; ++k) jobs[k].in_lds = in_lds;
  *lds = in_lds ? diag + tmax : diag;
  return 0;
}

int launch_dtw_jobs(const DtwJob* d_jobs, int n, int max_n, int in_lds, size_t lds, float sign, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_dtw<true>), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)DTW_LDS) != hipSuccess)
      return -2;
    attr = true;
  }
  // one lane per row: the fewer waves, the cheaper each diagonal's barrier
  const int threads = dtw_threads(max_n);
  if (n <= 0) return 0;
  if (in_lds) k_dtw<true><<<n, threads, lds, st>>>(d_jobs, sign), wh_launched("k_dtw");
  else k_dtw<false><<<n, threads, lds, st>>>(d_jobs, sign), wh_launched("k_dtw");
  return 0;
}

// grid (rows), block 256: probs[k] = softmax(logits[k][:eot])[tok[k]]
__global__ __launch_bounds__(256) void k_token_probs(const float* __restrict__ logits, int64_t ld, int eot,
                                                     const int* __restrict__ tok, float* __restrict__ probs) {
  __shared__ float red[4];
  const float* row = logits + (int64_t)blockIdx.x * ld;
  float m = -INFINITY;
  for (int v = threadIdx.x; v < eot; v += 256) m = fmaxf(m, row[v]);
  m = blk_max(m, red);
  float s = 0.f;
  for (int v = threadIdx.x; v < eot; v += 256) s += expf(row[v] - m);
  s = blk_sum(s, red);
  if (threadIdx.x == 0) {
    const int t = tok[blockIdx.x];
    probs[blockIdx.x] = (t >= 0 && t < eot) ? expf(row[t] - m) / s : 0.f;
  }
}

void launch_align_matrix(float* qk, int64_t hs, int rows, int Tk, int F, int heads, int t0, int N, int width,
                         float* mat, hipStream_t st) {
  k_align_softmax<<<dim3(rows, heads), 256, 0, st>>>(qk, hs, Tk, F), wh_launched("k_align_softmax");
  k_align_znorm<<<dim3((F + 63) / 64, heads), 256, 0, st>>>(qk, hs, rows, Tk, F), wh_launched("k_align_znorm");
  k_align_medmean<<<dim3((F + 255) / 256, N), 256, 0, st>>>(qk, hs, Tk, F, heads, t0, width, mat), wh_launched("k_align_medmean");
}

void launch_token_probs(const float* logits, int64_t ld, int rows, int eot, const int* tok, float* probs,
                        hipStream_t st) {
  if (rows > 0) k_token_probs<<<rows, 256, 0, st>>>(logits, ld, eot, tok, probs), wh_launched("k_token_probs");
}

}  // namespace wh
