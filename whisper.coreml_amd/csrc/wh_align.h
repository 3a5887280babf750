// Word-timestamp alignment kernels (wh_align.hip).
#pragma once
#include "wh_common.h"

namespace wh {

// qk: element (head h, token row t, frame f) at qk[h*hs + t*Tk + f], rows token rows
// (modified in place); mat: [N][F] = rows t0 .. t0+N-1 of the head-mean of the filtered
// weights (timing.py:196-205)
void launch_align_matrix(float* qk, int64_t hs, int rows, int Tk, int F, int heads, int t0, int N, int width,
                         float* mat, hipStream_t st);

// one DTW of x = sign * mat [N][M] (N <= 1023) + backtrace per workgroup; trace: global
// scratch of dtw_trace_bytes(N, M), used when the 2-bit packed trace does not fit LDS;
// path: [2][N+M] (text indices, then time indices), *plen valid entries of each
struct DtwJob {
  const float* mat;
  unsigned* trace;
  int* path;
  int* plen;
  int N, M, in_lds;
};
size_t dtw_trace_bytes(int N, int M);
// validates jobs, sets in_lds (one mode for the whole launch), returns the dynamic LDS
// bytes of the launch
int dtw_prepare(DtwJob* jobs, int n, size_t* lds);
// max_n: the largest N of the jobs (sizes the workgroup: one lane per row)
int launch_dtw_jobs(const DtwJob* d_jobs, int n, int max_n, int in_lds, size_t lds, float sign, hipStream_t st);
// probs[k] = softmax(logits[k][:eot])[tok[k]], k < rows (logits rows contiguous, stride ld)
void launch_token_probs(const float* logits, int64_t ld, int rows, int eot, const int* tok, float* probs,
                        hipStream_t st);

}  // namespace wh
