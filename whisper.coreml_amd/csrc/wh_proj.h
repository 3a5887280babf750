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
// WH_PROJ_XSLOW=1 (A/B build): the general X-slice addressing for every launch
#ifndef WH_PROJ_XSLOW
#define WH_PROJ_XSLOW 0
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
  const int ct_slot = a.N == a.K ? CT_PROJ_NN : a.N == 3 * a.K ? CT_PROJ_QKV : a.N == 4 * a.K ? CT_PROJ_FC1 : CT_PROJ_FC2;
  CT_MARK(ct_slot, 0);

  // 1. X slice -> registers
  const char* X = reinterpret_cast<const char*>(a.X);
  float4_t xv[P::XC];
  if (!a.x_rows && !WH_PROJ_XSLOW) {
    // (the decoder step: no gather) chunk c = tid + NT i sits at row c / CPR, column c % CPR;
    // both advance by compile-time steps, so the addresses are a few adds per chunk on a
    // 32-bit buffer offset (the general form below spent ~20 instructions and a branch per
    // chunk, ~0.7 us before the first weight load left), and every load is issued
    // unconditionally: rows past M read row M - 1 (their MFMA outputs are never stored)
    constexpr int DR = NT / P::CPR, DC = NT % P::CPR;
    const int ldx2 = a.ldx * (int)sizeof(T);
    // the buffer covers this workgroup's valid rows only: chunks of rows >= M read 0 (the
    // padding rows' zeros, as the general form), with no clamp or branch per chunk
    const auto rsx = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(X) + ((int64_t)m0 * a.ldx + kb) * (int)sizeof(T),
                                                       0, (a.M - m0) * ldx2 - kb * (int)sizeof(T), 0x00020000);
    int col = tid % P::CPR, off = (tid / P::CPR) * ldx2 + col * 16;
#pragma unroll
    for (int i = 0; i < P::XC; ++i) {
      xv[i] = __builtin_bit_cast(float4_t, __builtin_amdgcn_raw_buffer_load_b128(rsx, off, 0, 0));
      col += DC;
      off += DR * ldx2 + DC * 16;
      if (col >= P::CPR) {
        col -= P::CPR;
        off += ldx2 - P::CPR * 16;
      }
    }
  } else {
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
#pragma unroll
    for (int i = 0; i < P::XC; ++i) {
      const int c = tid + NT * i, col = c % P::CPR;
      xv[i] = (float4_t){0.f, 0.f, 0.f, 0.f};
      if (xr[i] >= 0)
        xv[i] = *reinterpret_cast<const float4_t*>(X + ((int64_t)xr[i] * a.ldx + kb) * (int)sizeof(T) + col * 16);
    }
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
  CT_MARK(ct_slot, 1);

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
  CT_MARK(ct_slot, 2);

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
#if WH_WT
      // write-through (sc1): the slab leaves no dirty L2 lines for the kernel-end release;
      // fp16 contexts store fp16 slabs (8 B per lane): half the bytes written here and read
      // by every consumer (round 4: out seam 9.50 -> 8.37 us in a graph chain,
      // profiles/r04/fp16_slab_chain_bench.txt)
      const int64_t e = ((int64_t)kz * a.M + m) * a.ldo + n;
      if (sizeof(T) == 2 && a.slab_half) {
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        const half4_t hv = (half4_t){(half_t)v[0], (half_t)v[1], (half_t)v[2], (half_t)v[3]};
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, hv), wt_rsrc(a.out_f32), (int)(e * 2), 0, 16);
      } else {
        wt_store4(wt_rsrc(a.out_f32), (int)(e * 4), v);
      }
#else
      store4(a.out_f32 + ((int64_t)kz * a.M + m) * a.ldo + n, v[0], v[1], v[2], v[3]);
#endif
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
  CT_END(ct_slot);
}

// ------------------------------------------------------------ single-window step layer
// k_proj1: the decoder-step projections at <= P1_RMAX rows (one window's beams: the
// per-token latency path), with no separate reduction launch on either side:
//  * prologue (CPL > 0): X = LayerNorm(x) of the fp32 residual rows, re-derived by every
//    workgroup from the full rows (R x n x 4 B of L2 reads, one wave per row, CPL float4
//    per lane) — replaces the k_resid_ln launch before the projection;
//  * a workgroup owns NSUB x 16 output columns x a K range of KC = KW*NSTEP*32 (the
//    k_proj tilings: <= 256 workgroups of 20-51 KB of weights); its KW waves split the
//    range and are summed in LDS in fixed order;
//  * ZS = K / KC > 1: the ZS waves that hold one 16-column tile's slices meet in an
//    in-launch split-K reduction (cdna_hip_programming.md §5 "Projection GEMM at M =
//    256" item 2, write-through form): fp32 1 KB slab stored sc1 by the wave, vmcnt(0),
//    relaxed agent fetch_add on the tile's counter; the wave drawing ZS-1 re-arms the
//    counter and sums the ZS slabs (sc1 loads) in slice order (deterministic for any
//    arrival order);
//  * epilogue owns every output element: bias + in-place residual add (EPI_RESID),
//    GELU, or the decoder QKV scatter (q + self-KV rows).
// A decoder layer is 8 launches instead of 12 (wh_runtime.hip dec_layers_p1).
// Load order: LN rows / X fragments (L2) first, then the wave's weight fragments (HBM),
// all issued before the first wait, so the LN math overlaps the weight stream.
constexpr int P1_RMAX = 8;

template <typename T, int NSUB, int KW, int NSTEP, int CPL>
struct Proj1Shape {
  static constexpr int KC = KW * NSTEP * 32;             // K per workgroup
  static constexpr int XROW = KC * (int)sizeof(T) + 16;  // padded LDS row (bytes)
  static constexpr int XBYTES = CPL ? P1_RMAX * XROW : 0;
  static constexpr int RBYTES = (KW - 1) * NSUB * 64 * 16;
  static constexpr int LDS = (XBYTES > RBYTES ? XBYTES : RBYTES) > 16 ? (XBYTES > RBYTES ? XBYTES : RBYTES) : 16;
};

// MODE bit 0 (P1_PEND, LayerNorm prologues): a deferred residual is pending on the input
// rows (GemmArgs::res_slab); bit 1 (P1_DEFER, residual projections, ZS == 2): store the
// two K-half slabs and stop — the next LayerNorm prologue adds them (no in-launch
// reduction: no drain, counter or second slab read on this launch's critical path).
constexpr int P1_PEND = 1, P1_DEFER = 2;

template <typename T, int NSUB, int KW, int NSTEP, int ZS, int CPL, int EPI, int MODE>
__global__ __launch_bounds__(64 * NSUB * KW) void k_proj1(GemmArgs a) {
  using P = Proj1Shape<T, NSUB, KW, NSTEP, CPL>;
  constexpr bool LN = CPL > 0;
  constexpr bool PEND = LN && (MODE & P1_PEND), DEFER = (MODE & P1_DEFER) && ZS == 2 && EPI == EPI_RESID;
  constexpr int NWV = NSUB * KW;
  constexpr int RPW = (P1_RMAX + NWV - 1) / NWV;  // LayerNorm rows per wave
  extern __shared__ __attribute__((aligned(16))) char xs[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const int sub = wave % NSUB, kw = wave / NSUB;
  const int R = a.M, K = a.K, kz = blockIdx.y;
  const int tile = blockIdx.x * NSUB + sub;  // this wave's 16-column tile
  const int n0 = tile * 16;
  const int kb = kz * P::KC;               // this workgroup's K range [kb, kb + KC)
  const int kw0 = kb + kw * NSTEP * 32;    // this wave's
  const T* W = reinterpret_cast<const T*>(a.W);
  const int ct_slot = a.N == a.K ? CT_PROJ_NN : a.N == 3 * a.K ? CT_PROJ_QKV : a.N == 4 * a.K ? CT_PROJ_FC1 : CT_PROJ_FC2;
  CT_MARK(ct_slot, 0);

  // 1. activations (clamped addresses, no branch around a load)
  const int CH = K / 4;  // LN: float4 chunks per residual row
  float4_t xv[LN ? RPW : 1][LN ? CPL : 1], gv[LN ? CPL : 1], bv[LN ? CPL : 1];
  float4_t s0v[PEND ? RPW : 1][PEND ? CPL : 1], s1v[PEND ? RPW : 1][PEND ? CPL : 1], rbv[PEND ? CPL : 1];
  Frag<T> xf[LN ? 1 : NSTEP];
  if constexpr (LN) {
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const float* xr = a.xf32 + (int64_t)min(wave + NWV * j, R - 1) * K;
#pragma unroll
      for (int i = 0; i < CPL; ++i) xv[j][i] = load4f(xr + 4 * min(lane + 64 * i, CH - 1));
    }
    if constexpr (PEND) {
      // the pending residual's two K-half slabs, row-major [2][R][K] like the rows
#pragma unroll
      for (int j = 0; j < RPW; ++j) {
        const int row = min(wave + NWV * j, R - 1);
#pragma unroll
        for (int i = 0; i < CPL; ++i) {
          const int off = row * K + 4 * min(lane + 64 * i, CH - 1);
          s0v[j][i] = load4f(a.res_slab + off);
          s1v[j][i] = load4f(a.res_slab + R * K + off);
        }
      }
#pragma unroll
      for (int i = 0; i < CPL; ++i) rbv[i] = load4f(a.res_bias + 4 * min(lane + 64 * i, CH - 1));
    }
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = min(lane + 64 * i, CH - 1);
      gv[i] = load4f(a.ln_g + 4 * c);
      bv[i] = load4f(a.ln_b + 4 * c);
    }
  } else {
    const T* xp = reinterpret_cast<const T*>(a.X) + (int64_t)min(r, R - 1) * a.ldx + kw0 + 8 * g;
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) frag_load(xf[s], xp + s * 32);
  }
  // 2. the wave's weight fragments: 16 columns x NSTEP k-steps
  const T* wp = W + (int64_t)min(n0 + r, a.N - 1) * K + kw0 + 8 * g;
  Frag<T> wf[NSTEP];
#pragma unroll
  for (int s = 0; s < NSTEP; ++s) frag_load_stream(wf[s], wp + s * 32);
  // the epilogue's operands ride in the same round trip: bias (every k_proj1 call has
  // one) and, for the residual add, this lane's x (only this tile's reducer writes it)
  const int n = n0 + 4 * g, re = min(r, R - 1);
  float4_t pre_b = (float4_t){0.f, 0.f, 0.f, 0.f}, pre_x = (float4_t){0.f, 0.f, 0.f, 0.f};
  if constexpr (!DEFER) pre_b = load4f(a.bias + n);
  if constexpr (EPI == EPI_RESID && !DEFER) pre_x = load4f(a.out_f32 + (int64_t)re * a.ldo + n);
  // every load above is issued before any wait (else hipcc streams them through a
  // sliding window of ~9, several round trips per wave)
  __builtin_amdgcn_sched_barrier(0);

  // 3. LayerNorm of the full rows (biased variance, two passes in registers: the
  // arithmetic of k_layernorm); this workgroup's K range of it -> LDS
  if constexpr (LN) {
    if constexpr (PEND) {
      // x_new = x + ((slab0 + slab1) + bias): the order of the in-launch reduction
#pragma unroll
      for (int j = 0; j < RPW; ++j)
#pragma unroll
        for (int i = 0; i < CPL; ++i) {
          float4_t t = s0v[j][i] + s1v[j][i];
          t += rbv[i];
          xv[j][i] += t;
        }
      if (blockIdx.x == 0 && blockIdx.y == 0) {  // one workgroup publishes x_new
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
          const int row = wave + NWV * j;
          if (row < R) {
#pragma unroll
            for (int i = 0; i < CPL; ++i)
              if (lane + 64 * i < CH) {
                const float4_t v = xv[j][i];
                store4(a.x_out + (int64_t)row * K + 4 * (lane + 64 * i), v[0], v[1], v[2], v[3]);
              }
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const int row = wave + NWV * j;
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < CPL; ++i)
        if (lane + 64 * i < CH) s += xv[j][i][0] + xv[j][i][1] + xv[j][i][2] + xv[j][i][3];
      const float mean = wave_sum(s) / (float)K;
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < CPL; ++i)
        if (lane + 64 * i < CH) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float d = xv[j][i][e] - mean;
            q += d * d;
          }
        }
      const float rstd = rsqrtf(wave_sum(q) / (float)K + a.ln_eps);
      if (row < R) {
#pragma unroll
        for (int i = 0; i < CPL; ++i) {
          const int k = 4 * (lane + 64 * i) - kb;
          if (k >= 0 && k < P::KC) {
            const float4_t v = xv[j][i];
            store4(reinterpret_cast<T*>(xs + row * P::XROW) + k, (v[0] - mean) * rstd * gv[i][0] + bv[i][0],
                   (v[1] - mean) * rstd * gv[i][1] + bv[i][1], (v[2] - mean) * rstd * gv[i][2] + bv[i][2],
                   (v[3] - mean) * rstd * gv[i][3] + bv[i][3]);
          }
        }
      }
    }
    __syncthreads();
  }

  // 4. MFMAs in load order
  float4_t acc = (float4_t){0.f, 0.f, 0.f, 0.f};
  if constexpr (LN) {
    const char* xl = xs + min(r, R - 1) * P::XROW + (kw * NSTEP * 32 + 8 * g) * (int)sizeof(T);
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) {
      Frag<T> x1;
      frag_load(x1, reinterpret_cast<const T*>(xl + s * 32 * (int)sizeof(T)));
      mfma_step(acc, wf[s], x1);
    }
  } else {
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) mfma_step(acc, wf[s], xf[s]);
  }

  // 5. fixed-order sum of the KW wave tiles
  if constexpr (KW > 1) {
    if constexpr (LN) __syncthreads();  // xs is reused
    float4_t* red = reinterpret_cast<float4_t*>(xs);  // [KW-1][NSUB][64]
    if (kw > 0) red[((kw - 1) * NSUB + sub) * 64 + lane] = acc;
    __syncthreads();
    if (kw > 0) return;  // (thread 0 is kw 0)
#pragma unroll
    for (int q = 1; q < KW; ++q) acc += red[((q - 1) * NSUB + sub) * 64 + lane];
  }

  // 6. split-K: the column tile's ZS workgroups meet; the last to arrive sums the slabs
  if constexpr (ZS > 1) {
    // write-through form (cdna_hip_programming.md §6 Guideline 16 R1): the slab is stored
    // sc1 and drained by its one storing wave, the counter add is a relaxed agent atomic,
    // and the reducer reads every slab with sc1 loads, so neither side needs a fence
    // (the plain-store + release / acquire form measured 2.5 us slower per launch)
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const int ntile = gridDim.x * NSUB;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(a.p1_slab, 0, 0x7fffffff, 0x00020000);
    if constexpr (DEFER) {  // row-major [2][R][N] for the next LayerNorm prologue, which sums them
      if (r < R) store4(a.p1_slab + ((int64_t)kz * R + r) * a.N + n, acc[0], acc[1], acc[2], acc[3]);
      CT_END(ct_slot);
      return;
    }
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc), rs, ((kz * ntile + tile) * 256 + lane * 4) * 4,
                                           0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int ticket = 0;
    if (lane == 0) ticket = __hip_atomic_fetch_add(a.p1_cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ticket = __shfl(ticket, 0, 64);
    if (ticket != ZS - 1) {
      CT_END(ct_slot);
      return;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the add
    if (lane == 0) __hip_atomic_store(a.p1_cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float4_t pv[ZS];  // every slab load issued before the first add; summed in slice order
#pragma unroll
    for (int s = 0; s < ZS; ++s)
      pv[s] = __builtin_bit_cast(float4_t,
                                 __builtin_amdgcn_raw_buffer_load_b128(rs, ((s * ntile + tile) * 256 + lane * 4) * 4, 0, 16));
    acc = pv[0];
#pragma unroll
    for (int s = 1; s < ZS; ++s) acc += pv[s];
  }

  // 7. epilogue: lane holds Y[r][n0 + 4g .. +3]
  if (r >= R) {
    CT_END(ct_slot);
    return;
  }
  acc += pre_b;
  if constexpr (EPI == EPI_RESID) {
    pre_x += acc;
    store4(a.out_f32 + (int64_t)r * a.ldo + n, pre_x[0], pre_x[1], pre_x[2], pre_x[3]);
  } else {
    epilogue_store<T, EPI>(a, r, 0, r, n, acc);
  }
  CT_END(ct_slot);
}

// launch_proj1 (wh_gemm.h): a.M <= P1_RMAX rows; the configuration comes from the
// model width (wh_proj.hip p1_launch); split tiles need a.p1_slab / a.p1_cnt

}  // namespace wh
