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
//                    LDS); costs are float32 cells fed by a float64 add exactly as the
//                    reference's float32 `cost` array fed from x.double(); ties resolve as
//                    its if/elif/else (c0 < c1 && c0 < c2 -> 0, c1 < c0 && c1 < c2 -> 1,
//                    else 2); then one lane walks the backtrace (timing.py:57-79)
//   k_token_probs    softmax over [:eot] of the rows that predict each text token,
//                    evaluated at that token (timing.py:187-191)
#include "wh_align.h"

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

// grid (rows, heads), block 256: w[h][t][f] = softmax_f(qk[h][t][f]), f < F (in place)
__global__ __launch_bounds__(256) void k_align_softmax(float* __restrict__ qk, int rows, int Tk, int F) {
  __shared__ float red[4];
  float* row = qk + ((int64_t)blockIdx.y * rows + blockIdx.x) * Tk;
  float m = -INFINITY;
  for (int f = threadIdx.x; f < F; f += 256) m = fmaxf(m, row[f]);
  m = blk_max(m, red);
  float s = 0.f;
  for (int f = threadIdx.x; f < F; f += 256) s += expf(row[f] - m);
  s = blk_sum(s, red);
  for (int f = threadIdx.x; f < F; f += 256) row[f] = expf(row[f] - m) / s;
}

// grid (ceil(F/64), heads), block 64: one lane per frame, loop over the token rows
__global__ __launch_bounds__(64) void k_align_znorm(float* __restrict__ w, int rows, int Tk, int F) {
  const int f = blockIdx.x * 64 + threadIdx.x;
  if (f >= F) return;
  float* col = w + (int64_t)blockIdx.y * rows * Tk + f;
  float s = 0.f;
  for (int t = 0; t < rows; ++t) s += col[(int64_t)t * Tk];
  const float mean = s / (float)rows;
  float q = 0.f;
  for (int t = 0; t < rows; ++t) {
    const float d = col[(int64_t)t * Tk] - mean;
    q += d * d;
  }
  const float sd = sqrtf(q / (float)rows);
  for (int t = 0; t < rows; ++t) col[(int64_t)t * Tk] = (col[(int64_t)t * Tk] - mean) / sd;
}

// grid (ceil(F/256), N), block 256: matrix[t - t0][f] = mean_h median7(w[h][t][f-3..f+3])
__global__ __launch_bounds__(256) void k_align_medmean(const float* __restrict__ w, int rows, int Tk, int F, int heads,
                                                       int t0, int width, float* __restrict__ mat) {
  const int f = blockIdx.x * 256 + threadIdx.x;
  const int t = t0 + blockIdx.y;
  if (f >= F) return;
  const int pad = width / 2;
  float acc = 0.f;
  for (int h = 0; h < heads; ++h) {
    const float* row = w + ((int64_t)h * rows + t) * Tk;
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

// one workgroup: DTW of x = sign * mat [N][M] and its backtrace.  trace: [N+1][M+1] int8
// scratch; path: [2][N+M] (text indices, then time indices), *plen = length.
constexpr int DTW_THREADS = 1024;
constexpr int DTW_MAXN = 1024;
__global__ __launch_bounds__(DTW_THREADS) void k_dtw(const float* __restrict__ mat, int N, int M, float sign,
                                                     signed char* __restrict__ trace, int* __restrict__ path,
                                                     int* __restrict__ plen) {
  __shared__ float dg[3][DTW_MAXN + 2];
  const int tid = threadIdx.x;
  const int64_t tw = M + 1;
  for (int i = tid; i <= N; i += DTW_THREADS) {
    dg[0][i] = INFINITY;
    dg[1][i] = INFINITY;
    dg[2][i] = INFINITY;
  }
  __syncthreads();
  if (tid == 0) dg[0][0] = 0.f;  // diagonal 0: cost[0][0]
  __syncthreads();
  for (int d = 1; d <= N + M; ++d) {
    float* cur = dg[d % 3];
    const float* p1 = dg[(d + 2) % 3];  // d - 1
    const float* p2 = dg[(d + 1) % 3];  // d - 2
    const int ilo = d - M > 0 ? d - M : 0, ihi = d < N ? d : N;
    for (int i = ilo + tid; i <= ihi; i += DTW_THREADS) {
      const int j = d - i;
      float cost;
      if (i == 0 || j == 0) {
        cost = INFINITY;
      } else {
        const float c0 = p2[i - 1], c1 = p1[i - 1], c2 = p1[i];
        float c;
        signed char t;
        if (c0 < c1 && c0 < c2) { c = c0; t = 0; }
        else if (c1 < c0 && c1 < c2) { c = c1; t = 1; }
        else { c = c2; t = 2; }
        const double x = (double)(sign * mat[(int64_t)(i - 1) * M + (j - 1)]);
        cost = (float)(x + (double)c);
        trace[i * tw + j] = t;
      }
      cur[i] = cost;
    }
    __syncthreads();
  }
  if (tid != 0) return;
  // backtrace (timing.py:57-79): trace[0][:] = 2, trace[:][0] = 1
  int i = N, j = M, n = 0;
  while (i > 0 || j > 0) {
    path[n] = i - 1;
    path[(N + M) + n] = j - 1;
    ++n;
    const int t = i == 0 ? 2 : (j == 0 ? 1 : trace[i * tw + j]);
    if (t == 0) { --i; --j; }
    else if (t == 1) { --i; }
    else { --j; }
  }
  // reverse in place
  for (int a = 0, b = n - 1; a < b; ++a, --b) {
    int x = path[a]; path[a] = path[b]; path[b] = x;
    x = path[(N + M) + a]; path[(N + M) + a] = path[(N + M) + b]; path[(N + M) + b] = x;
  }
  *plen = n;
}

// grid (T), block 256: probs[k] = softmax(logits[row0 + k][:eot])[tok[k]]
__global__ __launch_bounds__(256) void k_token_probs(const float* __restrict__ logits, int64_t ld, int row0, int eot,
                                                     const int* __restrict__ tok, float* __restrict__ probs) {
  __shared__ float red[4];
  const float* row = logits + (int64_t)(row0 + blockIdx.x) * ld;
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

void launch_align_matrix(float* qk, int rows, int Tk, int F, int heads, int t0, int N, int width, float* mat,
                         hipStream_t st) {
  k_align_softmax<<<dim3(rows, heads), 256, 0, st>>>(qk, rows, Tk, F);
  k_align_znorm<<<dim3((F + 63) / 64, heads), 64, 0, st>>>(qk, rows, Tk, F);
  k_align_medmean<<<dim3((F + 255) / 256, N), 256, 0, st>>>(qk, rows, Tk, F, heads, t0, width, mat);
}

int launch_dtw(const float* mat, int N, int M, float sign, signed char* trace, int* path, int* plen, hipStream_t st) {
  if (N < 1 || M < 1 || N > DTW_MAXN) return -1;
  k_dtw<<<1, DTW_THREADS, 0, st>>>(mat, N, M, sign, trace, path, plen);
  return 0;
}

void launch_token_probs(const float* logits, int64_t ld, int row0, int T, int eot, const int* tok, float* probs,
                        hipStream_t st) {
  if (T > 0) k_token_probs<<<T, 256, 0, st>>>(logits, ld, row0, eot, tok, probs);
}

}  // namespace wh
