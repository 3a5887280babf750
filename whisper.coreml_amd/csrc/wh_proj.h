// Decoder-step projections: weight-read-once skinny GEMM (device template;
// instantiated in wh_proj.hip).
//
//   Y[m][n] = sum_k X[m][k] * W[n][k]      (M = decode rows = windows x beams <= 128)
//
// A workgroup owns MT*16 rows x NSUB*16 columns x a K range of KC = KW*NSTEP*32
// (split-K z = K / KC over the grid).  The schedule is one straight line, so the
// whole workgroup's memory traffic is in flight at once (no sub-chunk loop):
//   1. every X chunk of the workgroup's [MT*16][KC] slice is loaded (L2-resident
//      activations) — first, so their wait does not wait on the weights;
//   2. every weight fragment of the wave (16 rows x NSTEP k-steps) is loaded (HBM);
//   3. X goes to LDS, one barrier, then NSTEP x MT MFMAs consume the weights in
//      load order (the compiler's vmcnt waits step down as they land).
// KW waves split the K range inside the workgroup; their tiles are summed in LDS in
// fixed order (deterministic, no atomics).  Workgroups that share a weight slice
// (different row groups) get consecutive logical ids, i.e. one XCD after the remap.
#pragma once
#include "wh_gemm.h"

#ifndef WH_PROJ_KZ_SLOW
#define WH_PROJ_KZ_SLOW 0
#endif

namespace wh {

template <typename T, int MT, int NSUB, int KW, int NSTEP>
struct ProjShape {
  static constexpr int CT = 16 * NSUB, MR = 16 * MT;
  static constexpr int KC = KW * NSTEP * 32;                  // K per workgroup
  static constexpr int XROW = KC * (int)sizeof(T) + 16;       // padded LDS row (bytes)
  static constexpr int CPR = KC * (int)sizeof(T) / 16;        // 16 B chunks per row
  static constexpr int NT = 64 * NSUB * KW;                   // threads
  static constexpr int XC = (MR * CPR + NT - 1) / NT;         // chunks per thread
  static constexpr int XBYTES = MR * XROW;
  static constexpr int RBYTES = (KW - 1) * NSUB * MT * 64 * 16;
  static constexpr int LDS = XBYTES > RBYTES ? XBYTES : RBYTES;
};

template <typename T, int MT, int NSUB, int KW, int NSTEP, int EPI>
__global__ __launch_bounds__(64 * NSUB * KW) void k_proj(GemmArgs a) {
  static_assert(NSUB * KW <= 16, "at most 16 waves");
  using P = ProjShape<T, MT, NSUB, KW, NSTEP>;
  constexpr int NT = 64 * NSUB * KW;
  extern __shared__ __attribute__((aligned(16))) char xs[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const int sub = wave % NSUB, kw = wave / NSUB;
  const int nct = (a.N + P::CT - 1) / P::CT, nmg = (a.M + P::MR - 1) / P::MR, z = a.K / P::KC;
  const int bid = xcd_remap(blockIdx.x, nct * nmg * z);
#if WH_PROJ_KZ_SLOW
  // column tiles vary fastest: an XCD's contiguous block of logical ids shares one or
  // two K ranges, so its X slices are fetched once into that XCD's L2 and re-read there
  const int mg = bid % nmg, t2 = bid / nmg, ct = t2 % nct, kz = t2 / nct;
#else
  const int mg = bid % nmg, t2 = bid / nmg, kz = t2 % z, ct = t2 / z;
#endif
  const int kb = kz * P::KC;
  const int n0 = ct * P::CT + sub * 16, m0 = mg * P::MR;

  // 1. X slice -> registers
  const char* X = reinterpret_cast<const char*>(a.X);
  // source row of each chunk (-1: padding row -> zeros); the optional gather is
  // resolved for every chunk before the first X load so no wait sits between them
  int xr[P::XC];
#pragma unroll
  for (int i = 0; i < P::XC; ++i) {
    const int c = tid + NT * i, m = m0 + c / P::CPR;
    xr[i] = (c < P::MR * P::CPR && m < a.M) ? m : -1;
  }
  if (a.x_rows) {
#pragma unroll
    for (int i = 0; i < P::XC; ++i)
      if (xr[i] >= 0) xr[i] = a.x_rows[xr[i]];
  }
  float4_t xv[P::XC];
#pragma unroll
  for (int i = 0; i < P::XC; ++i) {
    const int c = tid + NT * i, col = c % P::CPR;
    xv[i] = (float4_t){0.f, 0.f, 0.f, 0.f};
    if (xr[i] >= 0)
      xv[i] = *reinterpret_cast<const float4_t*>(X + ((int64_t)xr[i] * a.ldx + kb) * (int)sizeof(T) + col * 16);
  }
  // 2. the wave's weight fragments
  const T* wp = reinterpret_cast<const T*>(a.W) + (int64_t)min(n0 + r, a.N - 1) * a.K + kb + kw * NSTEP * 32 + 8 * g;
  Frag<T> wf[NSTEP];
#pragma unroll
  for (int s = 0; s < NSTEP; ++s) frag_load_stream(wf[s], wp + s * 32);
  // 3. X -> LDS
#pragma unroll
  for (int i = 0; i < P::XC; ++i) {
    const int c = tid + NT * i;
    if (c < P::MR * P::CPR) {
      const int row = c / P::CPR, col = c - row * P::CPR;
      *reinterpret_cast<float4_t*>(xs + row * P::XROW + col * 16) = xv[i];
    }
  }
  __syncthreads();

  float4_t acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = (float4_t){0.f, 0.f, 0.f, 0.f};
  const char* xl = xs + r * P::XROW + (kw * NSTEP * 32 + 8 * g) * (int)sizeof(T);
#pragma unroll
  for (int s = 0; s < NSTEP; ++s) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      Frag<T> xf;
      frag_load(xf, reinterpret_cast<const T*>(xl + mt * 16 * P::XROW + s * 32 * (int)sizeof(T)));
      mfma_step(acc[mt], wf[s], xf);
    }
  }

  // fixed-order reduction of the KW wave tiles
  if constexpr (KW > 1) {
    __syncthreads();
    float4_t* red = reinterpret_cast<float4_t*>(xs);  // [KW-1][NSUB][MT][64]
    if (kw > 0) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) red[(((kw - 1) * NSUB + sub) * MT + mt) * 64 + lane] = acc[mt];
    }
    __syncthreads();
    if (kw > 0) return;
#pragma unroll
    for (int q = 1; q < KW; ++q)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] += red[(((q - 1) * NSUB + sub) * MT + mt) * 64 + lane];
  }

  // epilogue: lane holds Y[m0 + mt*16 + r][n0 + 4g .. +3]
  const int n = n0 + 4 * g;
  if (n >= a.N) return;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = m0 + mt * 16 + r;
    if (m >= a.M) continue;
    float4_t v = acc[mt];
    if constexpr (EPI == EPI_PARTIAL) {
      store4(a.out_f32 + ((int64_t)kz * a.M + m) * a.ldo + n, v[0], v[1], v[2], v[3]);
    } else if constexpr (EPI == EPI_F32_COLS) {
      float* o = a.out_f32 + (int64_t)m * a.ldo;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (n + j < a.N) o[n + j] = v[j] + (a.bias ? a.bias[n + j] : 0.f);
    } else {
      if (a.bias) v += load4f(a.bias + n);
      epilogue_store<T, EPI>(a, m, 0, m, n, v);
    }
  }
}

}  // namespace wh
