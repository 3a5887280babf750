// Graph-chain prices of the 100-row decoder-step projection seams (round 4): N dependent
// nodes of one pattern captured in a hipGraph and replayed, hipEvents around the replays
// (what the step graph pays per node, launch gap included).  Weights rotate over 32
// copies so they stream from HBM as in a 32-layer step.  Patterns:
//   proj      k_proj out-projection tiling (N = K = 1280, 100 rows, z = 8 fp32 slabs)
//   rln       k_resid_ln of those 8 slabs (100 rows)
//   proj+rln  the seam as the step runs it
//   fc2 / fc2+rln   the fc2 tiling (K = 5120, z = 16) and its seam
//   variant knobs of a local copy of k_proj: no slab store, plain (not write-through) stores
//   ingest    a kernel that only loads the same bytes per workgroup (no LDS, no MFMA)
//   make -C whisper.coreml_amd tools/chain_bench && ./whisper.coreml_amd/tools/chain_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "wh_kernels.h"
#include "wh_proj.h"

using namespace wh;

namespace wh {
// ---- round-4 prototype, measured and NOT adopted: the residual
// seams folded into the split-K projections.  Kept here with its measurement.
// ------------------------------------------------------------ k_projx: the seams folded in
// The > 8-row decoder step ran every residual projection as k_proj (split-K slabs) +
// k_resid_ln (slab sum + bias + residual + LayerNorm) and fc1 as k_proj + k_reduce_store,
// 12 launches per layer.  k_projx folds both seams into the projections (8 launches):
//  * RX_RESID / RX_GELU: the z workgroups of a column tile meet in-launch.  Each stores its
//    fp32 slab write-through (sc1), drains it, and one lane adds to the tile's arrival
//    counter (relaxed agent atomic); one lane then polls the counter (relaxed agent loads,
//    s_sleep, bounded: 20 ms, then red_err) until all z have arrived, and the workgroup
//    reduces ITS share of the tile's rows — rows [kz RP, (kz + 1) RP), RP = ceil(M / z) —
//    with sc1 slab loads summed in slice order: x += (sum + bias) and the row's (sum, M2)
//    over the tile's columns (RX_RESID), or out = gelu(sum + bias) (RX_GELU).  Every
//    workgroup reduces, so the reduction is spread over the whole grid (a last-arriver form
//    would stream z x 25-36 KB through one CU).  MI355X_MICROARCH.md "Valid forms" row 1:
//    every slab store sc1 + every storing wave drained before the workgroup barrier and the
//    one counter add; every slab load sc1; the other loads (x, bias) read bytes no other
//    workgroup writes in the launch; one workgroup per CU (the launcher's LDS request).
//    All z workgroups of a tile must be resident together: grids <= 256 workgroups of one
//    per CU (launcher).
//  * PX_LN: the X slice is LayerNorm(x) computed here: the mean and variance of each row
//    come from the producer's per-tile (sum, M2), combined in tile order (Chan et al.'s
//    pairwise form: M2 = sum_t M2_t + n_t (mean_t - mean)^2), then x[row][kb .. kb + KC)
//    is normalised into the LDS tile.  Replaces k_resid_ln's LayerNorm.
// Arithmetic per row does not depend on the row count (batch invariance): the K split and
// the slice order come from the weight shape, the reduction share changes only which
// workgroup computes an element.
constexpr int PX_PLAIN = 0, PX_LN = 1;
constexpr int RX_SLABS = 0, RX_RESID = 1, RX_GELU = 2;
constexpr int PX_ST_MAX = 32;  // producer tiles per row the LayerNorm prologue combines
struct PxArgs : GemmArgs {
  float* red_slab = nullptr;
  int* red_cnt = nullptr;
  int* red_err = nullptr;
  float* st_out = nullptr;
  const float* st_in = nullptr;
  int st_tiles = 0, st_tw = 0, st_ld = 0;
};

template <typename T, int MT, int NSUB, int NSTEP, int PRO, int RED, int ZR>
__global__ __launch_bounds__(64 * NSUB) void k_projx(PxArgs a) {
  using P = ProjShape<T, MT, NSUB, 1, NSTEP>;
  constexpr int NT = 64 * NSUB, CT = P::CT, EPC = 16 / (int)sizeof(T);
  extern __shared__ __attribute__((aligned(16))) char xs[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const int R = a.M, nct = a.N / CT, z = a.K / P::KC;
  const int bid = xcd_remap(blockIdx.x, nct * z);
  const int kz = bid % z, ct = bid / z;
  const int kb = kz * P::KC;
  const int n0 = ct * CT + wave * 16;
  // LDS: the X tile [MR][XROW]; PX_LN: mean / rstd per row [MR][2], gamma / beta [2][KC],
  // the producer's statistics [MR][PX_ST_MAX] (float2)
  float* ln_mr = reinterpret_cast<float*>(xs + P::XBYTES);
  float* ln_gb = ln_mr + 2 * P::MR;
  float2* ln_st = reinterpret_cast<float2*>(ln_gb + 2 * P::KC);
  constexpr int SPT = PRO == PX_LN ? (P::MR * PX_ST_MAX + NT - 1) / NT : 1;  // statistics per thread

  // 1. every load of the workgroup before any wait: activations (L2), then weights (HBM)
  constexpr int F4 = PRO == PX_LN ? EPC / 4 : 1;  // fp32 float4 per 16-B chunk of T
  float4_t xv[P::XC][F4];
  float2 stv[SPT];
  float4_t gbv = (float4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < P::XC; ++i) {
    const int c = tid + NT * i, m = c / P::CPR, col = c - m * P::CPR;
#pragma unroll
    for (int f = 0; f < F4; ++f) xv[i][f] = (float4_t){0.f, 0.f, 0.f, 0.f};
    if (c < P::MR * P::CPR && m < R) {
      if constexpr (PRO == PX_LN) {
        const float* xp = a.xf32 + (int64_t)m * a.K + kb + col * EPC;
#pragma unroll
        for (int f = 0; f < F4; ++f) xv[i][f] = load4f(xp + 4 * f);
      } else {
        xv[i][0] = *reinterpret_cast<const float4_t*>(reinterpret_cast<const char*>(a.X) +
                                                      ((int64_t)m * a.ldx + kb) * (int)sizeof(T) + col * 16);
      }
    }
  }
  if constexpr (PRO == PX_LN) {
    // statistics of every (row, producer tile): staged through LDS (a per-row load would
    // hold PX_ST_MAX float2 in every thread)
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      const int e = tid + NT * j, m = e / a.st_tiles, t = e - m * a.st_tiles;
      stv[j] = m < R ? reinterpret_cast<const float2*>(a.st_in)[(int64_t)m * a.st_ld + t] : make_float2(0.f, 0.f);
    }
    // gamma / beta of this K range: KC / 4 float4 each
    if (tid < P::KC / 2) gbv = load4f((tid < P::KC / 4 ? a.ln_g : a.ln_b) + kb + 4 * (tid % (P::KC / 4)));
  }
  const T* wp = reinterpret_cast<const T*>(a.W) + (int64_t)(n0 + r) * a.K + kb + 8 * g;
  Frag<T> wf[NSTEP];
#pragma unroll
  for (int s = 0; s < NSTEP; ++s) frag_load_stream(wf[s], wp + s * 32);
  __builtin_amdgcn_sched_barrier(0);

  // 2. the X tile in LDS (PX_LN: normalised with the combined row statistics)
  if constexpr (PRO == PX_LN) {
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      const int e = tid + NT * j, m = e / a.st_tiles, t = e - m * a.st_tiles;
      if (m < R) ln_st[m * PX_ST_MAX + t] = stv[j];
    }
    if (tid < P::KC / 2) *reinterpret_cast<float4_t*>(ln_gb + 4 * tid) = gbv;
    __syncthreads();
    if (tid < R) {
      const float inv_n = 1.f / (float)a.K, tw = (float)a.st_tw;
      const float2* sr = ln_st + tid * PX_ST_MAX;
      float s = 0.f;
      for (int j = 0; j < a.st_tiles; ++j) s += sr[j].x;
      const float mean = s * inv_n;
      float m2 = 0.f;
      for (int j = 0; j < a.st_tiles; ++j) {
        const float d = sr[j].x / tw - mean;
        m2 += sr[j].y + tw * d * d;
      }
      ln_mr[2 * tid] = mean;
      ln_mr[2 * tid + 1] = rsqrtf(m2 * inv_n + a.ln_eps);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < P::XC; ++i) {
    const int c = tid + NT * i;
    if (c < P::MR * P::CPR) {
      const int m = c / P::CPR, col = c - m * P::CPR;
      if constexpr (PRO == PX_LN) {
        const float mean = ln_mr[2 * m], rstd = ln_mr[2 * m + 1];
        T* dst = reinterpret_cast<T*>(xs + m * P::XROW) + col * EPC;
#pragma unroll
        for (int f = 0; f < F4; ++f) {
          const int k = col * EPC + 4 * f;
          const float4_t gm = *reinterpret_cast<const float4_t*>(ln_gb + k);
          const float4_t bt = *reinterpret_cast<const float4_t*>(ln_gb + P::KC + k);
          const float4_t v = xv[i][f];
          // rows past M stay zero (their MFMA results are never stored)
          if (m < R)
            store4(dst + 4 * f, (v[0] - mean) * rstd * gm[0] + bt[0], (v[1] - mean) * rstd * gm[1] + bt[1],
                   (v[2] - mean) * rstd * gm[2] + bt[2], (v[3] - mean) * rstd * gm[3] + bt[3]);
          else
            store4(dst + 4 * f, 0.f, 0.f, 0.f, 0.f);
        }
      } else {
        *reinterpret_cast<float4_t*>(xs + m * P::XROW + col * 16) = xv[i][0];
      }
    }
  }
  __syncthreads();

  // 3. MFMAs in load order
  float4_t acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = (float4_t){0.f, 0.f, 0.f, 0.f};
  const char* xl = xs + r * P::XROW + 8 * g * (int)sizeof(T);
#pragma unroll
  for (int s = 0; s < NSTEP; ++s)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      Frag<T> xf;
      frag_load(xf, reinterpret_cast<const T*>(xl + mt * 16 * P::XROW + s * 32 * (int)sizeof(T)));
      mfma_step(acc[mt], wf[s], xf);
    }

  // 4. slab: lane holds Y[mt*16 + r][n0 + 4g .. +3] of slice kz
  const int n = n0 + 4 * g;
  if constexpr (RED == RX_SLABS) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = mt * 16 + r;
      if (m < R) wt_store4(wt_rsrc(a.out_f32), (int)((((int64_t)kz * R + m) * a.ldo + n) * 4), acc[mt]);
    }
    return;
  } else {
    static_assert(ZR >= 2 && ZR <= 16, "reduction slices");
    const auto rs = wt_rsrc(a.red_slab);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = mt * 16 + r;
      if (m < R) wt_store4(rs, (int)((((int64_t)kz * R + m) * a.N + n) * 4), acc[mt]);
    }
    // 5. rendezvous of the tile's z workgroups (see the header comment)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its slab stores
    __syncthreads();
    int* const okw = reinterpret_cast<int*>(xs);  // LDS word (the X tile is dead)
    if (tid == 0) {
      const int t = __hip_atomic_fetch_add(a.red_cnt + ct, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int target = (t / ZR + 1) * ZR;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
      int ok = 1;
      while (__hip_atomic_load(a.red_cnt + ct, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000ull) {  // 20 ms: a tile member never ran
          __hip_atomic_store(a.red_err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
      }
      *okw = ok;
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below
    if (!*okw) return;
    // 6. this workgroup's share of the tile: rows [r0, r1) x CT columns, one float4 per item
    constexpr int C4 = CT / 4;
    const int RP = (R + ZR - 1) / ZR, r0 = kz * RP, r1 = min(R, r0 + RP), items = max(0, r1 - r0) * C4;
    float* red = reinterpret_cast<float*>(xs) + 4;  // [RP][C4] row partials (RX_RESID)
    float* tmean = red + RP * C4;                   // [RP]
    constexpr int IPT = RED == RX_RESID ? 1 : 4;    // items per thread (RX_RESID: the launcher checks RP*C4 <= NT)
    float4_t nv[IPT];
#pragma unroll
    for (int ii = 0; ii < IPT; ++ii) {
      const int it = tid + NT * ii;
      if (it >= items) continue;
      const int row = r0 + it / C4, c = ct * CT + 4 * (it % C4);
      float4_t pv[ZR];
#pragma unroll
      for (int s = 0; s < ZR; ++s)
        pv[s] = __builtin_bit_cast(float4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                 rs, (int)((((int64_t)s * R + row) * a.N + c) * 4), 0, 16));
      const float4_t bv = load4f(a.bias + c);
      float4_t xo = (float4_t){0.f, 0.f, 0.f, 0.f};
      if constexpr (RED == RX_RESID) xo = load4f(a.out_f32 + (int64_t)row * a.ldo + c);
      float4_t t = pv[0];
#pragma unroll
      for (int s = 1; s < ZR; ++s) t += pv[s];
      t += bv;
      if constexpr (RED == RX_RESID) {
        xo += t;
        store4(a.out_f32 + (int64_t)row * a.ldo + c, xo[0], xo[1], xo[2], xo[3]);
        nv[ii] = xo;
      } else {
        store4(reinterpret_cast<T*>(a.out) + (int64_t)row * a.ldo + c, gelu_f(t[0]), gelu_f(t[1]), gelu_f(t[2]),
               gelu_f(t[3]));
      }
    }
    if constexpr (RED == RX_RESID) {
      // 7. per-row (sum, M2) over the tile's CT columns, in column order
      const bool has = tid < items;
      const int lr = tid / C4, c4 = tid % C4;
      if (has) red[lr * C4 + c4] = (nv[0][0] + nv[0][1]) + (nv[0][2] + nv[0][3]);
      __syncthreads();
      if (tid < r1 - r0) {
        float s = 0.f;
        for (int j = 0; j < C4; ++j) s += red[tid * C4 + j];
        tmean[tid] = s;
      }
      __syncthreads();
      float q = 0.f;
      if (has) {
        const float mu = tmean[lr] / (float)CT;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = nv[0][e] - mu;
          q += d * d;
        }
      }
      __syncthreads();  // every tmean read before red is rewritten
      if (has) red[lr * C4 + c4] = q;
      __syncthreads();
      if (tid < r1 - r0) {
        float m2 = 0.f;
        for (int j = 0; j < C4; ++j) m2 += red[tid * C4 + j];
        reinterpret_cast<float2*>(a.st_out)[(int64_t)(r0 + tid) * a.st_ld + ct] = make_float2(tmean[tid], m2);
      }
    }
  }
}

}  // namespace wh

// the three tilings the 1280-wide step selects (wh_proj.hip CFGS 0, 1, 2) and their z
struct PxCfg { int nsub, nstep; };
constexpr PxCfg PXC[] = {{4, 5}, {4, 10}, {5, 10}};
template <int MT, int C, int PRO, int RED, int ZR>
int px_go(const PxArgs& a, int wgs, hipStream_t st) {
  constexpr PxCfg c = PXC[C];
  using PS = ProjShape<half_t, MT, c.nsub, 1, c.nstep>;
  void (*f)(PxArgs) = &k_projx<half_t, MT, c.nsub, c.nstep, PRO, RED, ZR>;
  int lds = PS::XBYTES + (PRO == PX_LN ? (2 * PS::MR + 2 * PS::KC) * 4 + PS::MR * PX_ST_MAX * 8 : 0);
  if (RED != RX_SLABS) lds = std::max(lds, 81 * 1024);  // one workgroup per CU
  static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(f), hipFuncAttributeMaxDynamicSharedMemorySize,
                                         160 * 1024) == hipSuccess;
  if (!attr) return -2;
  hipLaunchKernelGGL(f, dim3(wgs), dim3(64 * c.nsub), lds, st, a);
  return 0;
}
// 100 rows: MT 7.  c: 0 = n x n (z 8, 160 workgroups), 1 = qkv (z 4, 240), 2 = fc1 (z 4, 256) / fc2 (z 16, 256)
int launch_projx(const PxArgs& a, int pro, int red, hipStream_t st) {
  const int c = a.N == 3 * 1280 ? 1 : (a.N == 4 * 1280 || a.K == 4 * 1280) ? 2 : 0;
  const int ct = 16 * PXC[c].nsub, z = a.K / (32 * PXC[c].nstep), wgs = a.N / ct * z;
  if (c == 0 && pro == PX_PLAIN && red == RX_RESID) return px_go<7, 0, PX_PLAIN, RX_RESID, 8>(a, wgs, st);
  if (c == 0 && pro == PX_LN && red == RX_SLABS) return px_go<7, 0, PX_LN, RX_SLABS, 1>(a, wgs, st);
  if (c == 1 && pro == PX_LN && red == RX_SLABS) return px_go<7, 1, PX_LN, RX_SLABS, 1>(a, wgs, st);
  if (c == 2 && pro == PX_LN && red == RX_GELU) return px_go<7, 2, PX_LN, RX_GELU, 4>(a, wgs, st);
  if (c == 2 && pro == PX_PLAIN && red == RX_RESID) return px_go<7, 2, PX_PLAIN, RX_RESID, 16>(a, wgs, st);
  return -1;
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

// local k_proj copy with knobs: bit 0 = no epilogue store, bit 1 = plain stores
template <int MT, int NSUB, int NSTEP, int MODE>
__global__ __launch_bounds__(64 * NSUB) void k_projv(GemmArgs a) {
  using T = half_t;
  using P = ProjShape<T, MT, NSUB, 1, NSTEP>;
  constexpr int NT = 64 * NSUB;
  extern __shared__ __attribute__((aligned(16))) char xs[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const int sub = wave;
  const int nct = (a.N + P::CT - 1) / P::CT, z = a.K / P::KC;
  const int bid = xcd_remap(blockIdx.x, nct * z);
  const int kz = bid % z, ct = bid / z;
  const int kb = kz * P::KC;
  const int n0 = ct * P::CT + sub * 16;
  const char* X = reinterpret_cast<const char*>(a.X);
  float4_t xv[P::XC];
#pragma unroll
  for (int i = 0; i < P::XC; ++i) {
    const int c = tid + NT * i, col = c % P::CPR, m = c / P::CPR;
    xv[i] = (float4_t){0.f, 0.f, 0.f, 0.f};
    if (c < P::MR * P::CPR && m < a.M)
      xv[i] = *reinterpret_cast<const float4_t*>(X + ((int64_t)m * a.ldx + kb) * (int)sizeof(T) + col * 16);
  }
  const T* wp = reinterpret_cast<const T*>(a.W) + (int64_t)(n0 + r) * a.K + kb + 8 * g;
  Frag<T> wf[NSTEP];
#pragma unroll
  for (int s = 0; s < NSTEP; ++s) frag_load_stream(wf[s], wp + s * 32);
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
  const char* xl = xs + r * P::XROW + 8 * g * (int)sizeof(T);
#pragma unroll
  for (int s = 0; s < NSTEP; ++s)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      Frag<T> xf;
      frag_load(xf, reinterpret_cast<const T*>(xl + mt * 16 * P::XROW + s * 32 * (int)sizeof(T)));
      mfma_step(acc[mt], wf[s], xf);
    }
  const int n = n0 + 4 * g;
  if constexpr (MODE & 1) {
    float s = 0.f;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) s += acc[mt][0] + acc[mt][1] + acc[mt][2] + acc[mt][3];
    if (s == 1234.5f) a.out_f32[0] = s;
    return;
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mt * 16 + r;
    if (m >= a.M) continue;
    if constexpr (MODE & 4) {  // fp16 slabs, write-through (8 B per lane)
      const half4_t h = (half4_t){(half_t)acc[mt][0], (half_t)acc[mt][1], (half_t)acc[mt][2], (half_t)acc[mt][3]};
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(unsigned __attribute__((ext_vector_type(2))), h), wt_rsrc(a.out_f32),
                                            (int)((((int64_t)kz * a.M + m) * a.ldo + n) * 2), 0, 16);
    } else if constexpr (MODE & 2) store4(a.out_f32 + ((int64_t)kz * a.M + m) * a.ldo + n, acc[mt][0], acc[mt][1], acc[mt][2],
                                   acc[mt][3]);
    else wt_store4(wt_rsrc(a.out_f32), (int)((((int64_t)kz * a.M + m) * a.ldo + n) * 4), acc[mt]);
  }
}

// k_resid_ln (wh_kernels.hip) reading fp16 slabs: one float4 of the row per thread
template <int NS>
__global__ __launch_bounds__(512) void k_rln16(float* __restrict__ x, const half_t* __restrict__ part, int64_t pstride,
                                               const float* __restrict__ bias, half_t* __restrict__ y,
                                               const float* __restrict__ gamma, const float* __restrict__ beta, int n,
                                               float eps) {
  __shared__ float red[2][8];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nwv = blockDim.x >> 6;
  float* xr = x + (int64_t)row * n;
  const int c = tid;
  const float4_t gm = load4f(gamma + 4 * c), bt = load4f(beta + 4 * c);
  float4_t a = load4f(xr + 4 * c);
  float4_t pp[NS];
#pragma unroll
  for (int sp = 0; sp < NS; ++sp) pp[sp] = load4f(part + sp * pstride + (int64_t)row * n + 4 * c);
  a += load4f(bias + 4 * c);
#pragma unroll
  for (int sp = 0; sp < NS; ++sp) a += pp[sp];
  store4(xr + 4 * c, a[0], a[1], a[2], a[3]);
  float s = wave_sum(a[0] + a[1] + a[2] + a[3]);
  if (lane == 0) red[0][wv] = s;
  __syncthreads();
  float tot = 0.f;
  for (int k = 0; k < nwv; ++k) tot += red[0][k];
  const float mean = tot / (float)n;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) q += (a[j] - mean) * (a[j] - mean);
  q = wave_sum(q);
  if (lane == 0) red[1][wv] = q;
  __syncthreads();
  float qt = 0.f;
  for (int k = 0; k < nwv; ++k) qt += red[1][k];
  const float rstd = rsqrtf(qt / (float)n + eps);
  store4(y + (int64_t)row * n + 4 * c, (a[0] - mean) * rstd * gm[0] + bt[0], (a[1] - mean) * rstd * gm[1] + bt[1],
         (a[2] - mean) * rstd * gm[2] + bt[2], (a[3] - mean) * rstd * gm[3] + bt[3]);
}

__global__ __launch_bounds__(256) void k_ingest(const float4_t* __restrict__ h, const float4_t* __restrict__ s, int h16,
                                                int s16, int share, float* out) {
  const int t = threadIdx.x;
  const float4_t* hp = h + (size_t)blockIdx.x * h16;
  const float4_t* sp = s + (size_t)(blockIdx.x / share) * s16;
  float4_t v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int j = t + 256 * i;
    v[i] = j < s16 ? sp[j] : (j - s16 < h16 && j >= s16 ? hp[j - s16] : (float4_t){0.f, 0.f, 0.f, 0.f});
  }
  float a = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) a += v[i][0] + v[i][1] + v[i][2] + v[i][3];
  if (a == 1234.5f) out[0] = a;
}

int main(int argc, char** argv) {
  const int nodes = argc > 1 ? atoi(argv[1]) : 96, reps = argc > 2 ? atoi(argv[2]) : 10;
  const int M = 100, n = 1280, L = 32;
  half_t *W, *X, *Y;
  float *part, *x, *bias, *g, *b, *out;
  const size_t wsz = (size_t)4 * n * n;
  CK(hipMalloc(&W, wsz * L * sizeof(half_t)));
  CK(hipMemset(W, 0, wsz * L * sizeof(half_t)));
  CK(hipMalloc(&X, (size_t)M * 4 * n * sizeof(half_t)));
  CK(hipMemset(X, 0, (size_t)M * 4 * n * sizeof(half_t)));
  CK(hipMalloc(&Y, (size_t)M * n * sizeof(half_t)));
  CK(hipMalloc(&part, (size_t)16 * M * n * sizeof(float)));
  CK(hipMemset(part, 0, (size_t)16 * M * n * sizeof(float)));
  CK(hipMalloc(&x, (size_t)M * n * sizeof(float)));
  CK(hipMemset(x, 0, (size_t)M * n * sizeof(float)));
  CK(hipMalloc(&bias, n * sizeof(float)));
  CK(hipMalloc(&g, n * sizeof(float)));
  CK(hipMalloc(&b, n * sizeof(float)));
  CK(hipMemset(bias, 0, n * 4));
  CK(hipMemset(g, 0, n * 4));
  CK(hipMemset(b, 0, n * 4));
  CK(hipMalloc(&out, 4096));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  auto proj_args = [&](int i, int N, int K) {
    GemmArgs a;
    a.X = X; a.ldx = K; a.W = W + wsz * (i % L); a.M = M; a.N = N; a.K = K; a.x_group_rows = M;
    a.out_f32 = part; a.ldo = N;
    return a;
  };
  auto time_chain = [&](const char* name, std::function<void(int)> body) {
    hipGraph_t gr;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < nodes; ++i) body(i);
    CK(hipStreamEndCapture(st, &gr));
    CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-44s %7.2f us per repetition\n", name, ms * 1e3 / (reps * nodes));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(gr));
  };
  auto proj = [&](int i, int N, int K) {
    int z = 0;
    if (launch_proj_partial<half_t>(proj_args(i, N, K), 16, st, &z) != 0) {
      fprintf(stderr, "no k_proj tiling\n");
      exit(1);
    }
    return z;
  };
  int z_out = 0, z_fc2 = 0;
  {
    // probe the split counts once (not captured)
    z_out = proj(0, n, n);
    z_fc2 = proj(0, n, 4 * n);
    CK(hipStreamSynchronize(st));
    printf("out z %d, fc2 z %d\n", z_out, z_fc2);
  }
  time_chain("proj (out, z=8)", [&](int i) { proj(i, n, n); });
  time_chain("rln (8 slabs)", [&](int) {
    launch_resid_ln<half_t>(x, part, z_out, (int64_t)M * n, bias, Y, g, b, M, n, 1e-5f, st);
  });
  time_chain("proj + rln (out seam)", [&](int i) {
    proj(i, n, n);
    launch_resid_ln<half_t>(x, part, z_out, (int64_t)M * n, bias, Y, g, b, M, n, 1e-5f, st);
  });
  time_chain("fc2 proj (z=16)", [&](int i) { proj(i, n, 4 * n); });
  time_chain("fc2 proj + rln (16 slabs)", [&](int i) {
    proj(i, n, 4 * n);
    launch_resid_ln<half_t>(x, part, z_fc2, (int64_t)M * n, bias, Y, g, b, M, n, 1e-5f, st);
  });
  time_chain("rln (16 slabs)", [&](int) {
    launch_resid_ln<half_t>(x, part, z_fc2, (int64_t)M * n, bias, Y, g, b, M, n, 1e-5f, st);
  });
  time_chain("rln (0 slabs: plain LayerNorm of x)", [&](int) {
    launch_resid_ln<half_t>(x, nullptr, 0, 0, nullptr, Y, g, b, M, n, 1e-5f, st);
  });
  // round 4: the seams folded into the projections (k_projx)
  float *rslab, *stats;
  int *cnt, *err;
  CK(hipMalloc(&rslab, (size_t)16 * M * 4 * n * sizeof(float)));
  CK(hipMemset(rslab, 0, (size_t)16 * M * 4 * n * sizeof(float)));
  CK(hipMalloc(&stats, (size_t)M * 64 * 8));
  CK(hipMemset(stats, 0, (size_t)M * 64 * 8));
  CK(hipMalloc(&cnt, 4 * 1024));
  CK(hipMemset(cnt, 0, 4 * 1024));
  CK(hipMalloc(&err, 256));
  CK(hipMemset(err, 0, 256));
  half_t* hm;
  CK(hipMalloc(&hm, (size_t)M * 4 * n * sizeof(half_t)));
  CK(hipMemset(hm, 0, (size_t)M * 4 * n * sizeof(half_t)));
  auto px = [&](int i, int N, int K, int pro, int red, int* c, int st_tiles, int st_tw) {
    PxArgs a;
    static_cast<GemmArgs&>(a) = proj_args(i, N, K);
    a.bias = bias; a.red_slab = rslab; a.red_cnt = c; a.red_err = err; a.st_out = stats; a.st_ld = 64;
    a.st_in = stats; a.st_tiles = st_tiles; a.st_tw = st_tw; a.xf32 = x; a.ln_g = g; a.ln_b = b;
    if (red == RX_RESID) { a.out_f32 = x; a.ldo = n; }
    if (red == RX_GELU) { a.out = hm; a.ldo = N; }
    if (red == RX_SLABS) { a.out_f32 = part; a.ldo = N; }
    if (pro == PX_PLAIN) { a.X = red == RX_RESID && K == 4 * n ? (const void*)hm : (const void*)X; a.ldx = K; }
    if (launch_projx(a, pro, red, st) != 0) {
      fprintf(stderr, "launch_projx failed N %d K %d pro %d red %d\n", N, K, pro, red);
      exit(1);
    }
  };
  time_chain("old: out proj + rln + cross-q proj", [&](int i) {
    proj(i, n, n);
    launch_resid_ln<half_t>(x, part, z_out, (int64_t)M * n, bias, Y, g, b, M, n, 1e-5f, st);
    proj(i + 1, n, n);
  });
  time_chain("new: out projx(RESID) + cross-q projx(LN)", [&](int i) {
    px(i, n, n, PX_PLAIN, RX_RESID, cnt, 0, 0);
    px(i + 1, n, n, PX_LN, RX_SLABS, nullptr, 20, 64);
  });
  time_chain("new: out projx(RESID) alone", [&](int i) { px(i, n, n, PX_PLAIN, RX_RESID, cnt, 0, 0); });
  time_chain("new: cross-q projx(LN) alone", [&](int i) { px(i, n, n, PX_LN, RX_SLABS, nullptr, 20, 64); });
  time_chain("old: fc1 proj + reduce_store + fc2 proj + rln", [&](int i) {
    int z1 = proj(i, 4 * n, n);
    launch_reduce_store<half_t>(part, z1, (int64_t)M * 4 * n, bias, hm, 4 * n, M, 4 * n, 1, st);
    proj(i + 1, n, 4 * n);
    launch_resid_ln<half_t>(x, part, z_fc2, (int64_t)M * n, bias, Y, g, b, M, n, 1e-5f, st);
  });
  time_chain("new: fc1 projx(LN, GELU) + fc2 projx(RESID)", [&](int i) {
    px(i, 4 * n, n, PX_LN, RX_GELU, cnt + 256, 20, 64);
    px(i + 1, n, 4 * n, PX_PLAIN, RX_RESID, cnt + 512, 0, 0);
  });
  time_chain("new: qkv projx(LN) alone", [&](int i) { px(i, 3 * n, n, PX_LN, RX_SLABS, nullptr, 16, 80); });
  time_chain("old: qkv proj alone", [&](int i) { proj(i, 3 * n, n); });
  {
    int h_err = 0;
    CK(hipMemcpy(&h_err, err, 4, hipMemcpyDeviceToHost));
    printf("rendezvous error word: %d\n", h_err);
  }
  // local variants of the out tiling <7, 4, 1, 5>: 160 workgroups
  using PS = ProjShape<half_t, 7, 4, 1, 5>;
  auto var = [&](const char* name, void (*f)(GemmArgs)) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(f), hipFuncAttributeMaxDynamicSharedMemorySize, PS::LDS));
    time_chain(name, [&](int i) { hipLaunchKernelGGL(f, dim3(160), dim3(256), PS::LDS, st, proj_args(i, n, n)); });
  };
  var("variant: local copy (write-through)", &k_projv<7, 4, 5, 0>);
  var("variant: no epilogue store", &k_projv<7, 4, 5, 1>);
  var("variant: plain stores", &k_projv<7, 4, 5, 2>);
  // fp16 split-K slabs (half the slab bytes) + a k_resid_ln reading them
  {
    using PF = ProjShape<half_t, 7, 5, 1, 10>;
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_projv<7, 5, 10, 0>), hipFuncAttributeMaxDynamicSharedMemorySize,
                           PF::LDS));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_projv<7, 5, 10, 4>), hipFuncAttributeMaxDynamicSharedMemorySize,
                           PF::LDS));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_projv<7, 4, 5, 4>), hipFuncAttributeMaxDynamicSharedMemorySize,
                           PS::LDS));
    half_t* part16 = reinterpret_cast<half_t*>(part);
    time_chain("fp32 slabs: out projv + rln", [&](int i) {
      hipLaunchKernelGGL((k_projv<7, 4, 5, 0>), dim3(160), dim3(256), PS::LDS, st, proj_args(i, n, n));
      launch_resid_ln<half_t>(x, part, 8, (int64_t)M * n, bias, Y, g, b, M, n, 1e-5f, st);
    });
    time_chain("fp16 slabs: out projv + rln16", [&](int i) {
      hipLaunchKernelGGL((k_projv<7, 4, 5, 4>), dim3(160), dim3(256), PS::LDS, st, proj_args(i, n, n));
      hipLaunchKernelGGL((k_rln16<8>), dim3(M), dim3(320), 0, st, x, part16, (int64_t)M * n, bias, Y, g, b, n, 1e-5f);
    });
    time_chain("fp32 slabs: fc2 projv + rln", [&](int i) {
      hipLaunchKernelGGL((k_projv<7, 5, 10, 0>), dim3(256), dim3(320), PF::LDS, st, proj_args(i, n, 4 * n));
      launch_resid_ln<half_t>(x, part, 16, (int64_t)M * n, bias, Y, g, b, M, n, 1e-5f, st);
    });
    time_chain("fp16 slabs: fc2 projv + rln16", [&](int i) {
      hipLaunchKernelGGL((k_projv<7, 5, 10, 4>), dim3(256), dim3(320), PF::LDS, st, proj_args(i, n, 4 * n));
      hipLaunchKernelGGL((k_rln16<16>), dim3(M), dim3(320), 0, st, x, part16, (int64_t)M * n, bias, Y, g, b, n, 1e-5f);
    });
  }
  // the same bytes per workgroup with nothing else: X slice 35 KB shared by 20, W 20 KB
  time_chain("ingest: 35 KB shared + 20 KB streamed", [&](int i) {
    k_ingest<<<160, 256, 0, st>>>(reinterpret_cast<const float4_t*>(W + wsz * (i % L)),
                                  reinterpret_cast<const float4_t*>(X), 20 * 1024 / 16, 35 * 1024 / 16, 20, out);
  });
  time_chain("ingest: nothing", [&](int i) {
    k_ingest<<<160, 256, 0, st>>>(reinterpret_cast<const float4_t*>(W), reinterpret_cast<const float4_t*>(X), 0, 0, 20,
                                  out);
  });
  return 0;
}
