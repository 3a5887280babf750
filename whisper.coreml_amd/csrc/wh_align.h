// Word-timestamp alignment kernels (wh_align.hip).
#pragma once
#include "wh_common.h"

namespace wh {

// qk: [heads][rows][Tk] raw cross q.k of the alignment heads (modified in place);
// mat: [N][F] = rows t0 .. t0+N-1 of the head-mean of the filtered weights
void launch_align_matrix(float* qk, int rows, int Tk, int F, int heads, int t0, int N, int width, float* mat,
                         hipStream_t st);
// DTW of x = sign * mat [N][M] + backtrace; trace scratch [N+1][M+1]; path [2][N+M]
// (text indices, then time indices; the first *plen entries of each are valid)
int launch_dtw(const float* mat, int N, int M, float sign, signed char* trace, int* path, int* plen, hipStream_t st);
// probs[k] = softmax(logits[row0 + k][:eot])[tok[k]], k < T
void launch_token_probs(const float* logits, int64_t ld, int row0, int T, int eot, const int* tok, float* probs,
                        hipStream_t st);

}  // namespace wh
