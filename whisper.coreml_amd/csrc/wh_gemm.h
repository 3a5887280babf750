// GEMM argument block and fused epilogues (see wh_gemm.hip).
#pragma once
#include "wh_common.h"

namespace wh {

enum Epi {
  EPI_STORE = 0,       // out[T]  = acc + bias
  EPI_STORE_GELU = 1,  // out[T]  = gelu(acc + bias)
  EPI_RESID = 2,       // out_f32 += acc + bias            (residual stream, in place)
  EPI_GELU_POS = 3,    // out_f32  = gelu(acc + bias) + pos[row-in-group]   (conv2 -> x)
  EPI_HEADSPLIT = 4,   // cross-KV: K -> [l2][win][head][t][d], V -> [l2][win][head][d][t]
  EPI_QKV_DEC = 5,     // decoder q -> out[T]; k,v -> self-KV cache at (win, slot, head, pos)
  EPI_F32_COLS = 6,    // logits: out_f32[m][n] (ragged N)
  EPI_PARTIAL = 7,     // split-K partial: out_f32[z][m][n] (no bias; summed by k_resid_ln)
  EPI_QKV_ENC = 8,     // encoder qkv: q, k -> out[T] (groups); v -> vc as V^T [win][head][64][perm(t)]
};

struct GemmArgs {
  const void* X = nullptr;  // [M rows] x K, element (m,k) at X + grp*x_group_stride + rowInGrp*ldx + k
  const void* W = nullptr;  // [N][K]
  const float* bias = nullptr;
  int M = 0, N = 0, K = 0;
  int ldx = 0;
  int x_group_rows = 1 << 30;     // rows per group (windows); M for a plain matrix
  int64_t x_group_stride = 0;     // elements between groups
  // outputs
  void* out = nullptr;            // T output
  float* out_f32 = nullptr;       // f32 output / residual
  int ldo = 0;
  int64_t out_group_stride = 0;   // elements between groups (EPI_STORE / GELU)
  int out_row_off = 0;            // row offset inside a group (conv1 writes after a zero pad row)
  const float* pos = nullptr;     // EPI_GELU_POS: [rows-in-group][N]
  // head-split (cross-KV) layout: out[((l2*nslots + slot0+grp)*H + h)*T + t][64]
  int hs_state = 0, hs_heads = 0, hs_T = 0, hs_nslots = 0, hs_slot0 = 0;
  // decoder QKV: row metadata + caches [win][slot][head][ctx][64]
  const int* row_win = nullptr;
  const int* row_slot = nullptr;
  const int* row_pos = nullptr;
  void* kc = nullptr;
  void* vc = nullptr;
  int kv_beams = 0, kv_ctx = 0;
  // skinny GEMM only: row gather (X row of output row m = x_rows[m]) and split-K
  const int* x_rows = nullptr;
  int ksplit = 1;
  int mt_block = 0;  // 16-row tiles per block (0 = min(ceil(M/16), 8))
  int row_groups = 1;  // k_vocab_small: row groups (set by the launcher)
  // k_proj PRO_LN prologue: X = LayerNorm(xf32 rows; ln_g, ln_b, ln_eps)
  const float* xf32 = nullptr;
  const float* ln_g = nullptr;
  const float* ln_b = nullptr;
  float ln_eps = 1e-5f;
  // k_proj1 in-launch split-K: fp32 slabs [ZS][N/16][256] and one arrival counter per
  // 16-column tile (zero between launches: the last arriver re-arms it)
  float* p1_slab = nullptr;
  int* p1_cnt = nullptr;
  int p1_slabs = 0;  // slab capacity (1 KB slabs) of p1_slab
  // k_proj1 deferred residual (wh_proj.h): a residual projection launched with p1_defer
  // only stores its two K-half slabs; the next LayerNorm prologue (res_slab != null)
  // forms x_new = xf32 + ((slab0 + slab1) + res_bias), normalises it, and the workgroup
  // (0, 0) writes x_new to x_out (another buffer: the other workgroups still read xf32)
  int p1_defer = 0;
  const float* res_slab = nullptr;
  const float* res_bias = nullptr;
  float* x_out = nullptr;
  // k_proj EPI_PARTIAL in an fp16 context: store the split-K slabs as fp16 (out_f32 then
  // holds half_t elements; wh_kernels.h slab consumers take slab_half = 1)
  int slab_half = 0;
};

template <typename T, int EPI>
WH_DEV void epilogue_store(const GemmArgs& a, int m, int gi, int ri, int n, float4_t v) {
  if constexpr (EPI == EPI_STORE || EPI == EPI_STORE_GELU) {
    if constexpr (EPI == EPI_STORE_GELU) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = gelu_f(v[j]);
    }
    T* o = reinterpret_cast<T*>(a.out) + (int64_t)gi * a.out_group_stride + (int64_t)(ri + a.out_row_off) * a.ldo + n;
    store4(o, v[0], v[1], v[2], v[3]);
  } else if constexpr (EPI == EPI_RESID) {
    float* o = a.out_f32 + (int64_t)m * a.ldo + n;
    float4_t c = load4f(o);
    c += v;
    store4(o, c[0], c[1], c[2], c[3]);
  } else if constexpr (EPI == EPI_GELU_POS) {
    const float4_t p = load4f(a.pos + (int64_t)ri * a.N + n);
    float* o = a.out_f32 + (int64_t)m * a.ldo + n;
    store4(o, gelu_f(v[0]) + p[0], gelu_f(v[1]) + p[1], gelu_f(v[2]) + p[2], gelu_f(v[3]) + p[3]);
  } else if constexpr (EPI == EPI_HEADSPLIT) {
    // l2 even: K -> [l2][slot][h][t][64]; l2 odd: V transposed, tile-major ->
    // [l2][slot][h][t / 64][64 d][perm(t % 64)] (blocks of hs_T = TKP keys, a multiple of
    // 64); perm: within each 32-key group, key 16*hi+4*g+j moves to 8*g+4*hi+j so a lane's
    // 8 P.V keys are contiguous (k_cross_attn, k_xattn_seg)
    const int l2 = n / a.hs_state, c = n - l2 * a.hs_state, h = c >> 6, d = c & 63;
    const int64_t blk = (((int64_t)l2 * a.hs_nslots + a.hs_slot0 + gi) * a.hs_heads + h) * a.hs_T * 64;
    T* o = reinterpret_cast<T*>(a.out) + blk;
    if ((l2 & 1) == 0) {
      store4(o + (int64_t)ri * 64 + d, v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[xv_index(d + j, ri)] = from_f32<T>(v[j]);
    }
  } else if constexpr (EPI == EPI_QKV_ENC) {
    if (n < 2 * a.hs_state) {
      T* o = reinterpret_cast<T*>(a.out) + (int64_t)gi * a.out_group_stride + (int64_t)ri * a.ldo + n;
      store4(o, v[0], v[1], v[2], v[3]);
    } else {
      // V transposed per (window, head), keys permuted within 32-key groups as the
      // cross-KV V^T (EPI_HEADSPLIT): k_attn_enc stages a 64-key tile with 16 B copies
      // and reads its P.V fragments with one 16 B LDS read each
      const int c = n - 2 * a.hs_state, h = c >> 6, d = c & 63;
      const int q = ri & 31;
      const int pt = (ri & ~31) + 8 * ((q & 15) >> 2) + 4 * (q >> 4) + (q & 3);
      T* o = reinterpret_cast<T*>(a.vc) + (((int64_t)gi * a.hs_heads + h) * 64 + d) * a.hs_T + pt;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[(int64_t)j * a.hs_T] = from_f32<T>(v[j]);
    }
  } else if constexpr (EPI == EPI_QKV_DEC) {
    const int ns = a.hs_state;
    if (n < ns) {
      store4(reinterpret_cast<T*>(a.out) + (int64_t)m * a.ldo + n, v[0], v[1], v[2], v[3]);
    } else {
      const int which = n >= 2 * ns;  // 0 = k, 1 = v
      const int c = n - ns * (1 + which), h = c >> 6, d = c & 63;
      const int w = a.row_win[m], sl = a.row_slot[m], p = a.row_pos[m];
      const int64_t idx = ((((int64_t)w * a.kv_beams + sl) * a.hs_heads + h) * a.kv_ctx + p) * 64 + d;
      T* base = reinterpret_cast<T*>(which ? a.vc : a.kc);
      store4(base + idx, v[0], v[1], v[2], v[3]);
    }
  }
}

// The epilogue of a tile whose lane holds acc[mi][ni] = Y[mrow(mi)][ncol(ni) .. +3]:
// the bias of the lane's columns is loaded once (it depends on n only), and an epilogue
// that reads memory per element (EPI_RESID: the residual x; EPI_GELU_POS: pos) issues
// every such load of a group of MG row tiles before the group's first store.  Written as
// one loop of epilogue_store calls, the compiler keeps each load behind the previous
// store (they may alias) and waits on it at once: 2 x MI x NI dependent round trips per
// tile (k_gemm_256 EPI_RESID: ~57 us of a 256 x 256 tile; profiles/r03/gemm_epilogue_ab.txt).
// Same arithmetic as epilogue_store: v = acc (+ bias), then the epilogue's own op.
template <typename T, int EPI, int MI, int NI, int MG, typename RowF, typename ColF>
WH_DEV void tile_epilogue(const GemmArgs& a, const float4_t (&acc)[MI][NI], RowF mrow, ColF ncol) {
  static_assert(MI % MG == 0, "row-tile groups");
  constexpr bool LD = EPI == EPI_RESID || EPI == EPI_GELU_POS;
  float4_t bv[NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) bv[ni] = a.bias ? load4f(a.bias + ncol(ni)) : (float4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g0 = 0; g0 < MI; g0 += MG) {
    float4_t xv[LD ? MG : 1][LD ? NI : 1];
    if constexpr (LD) {
#pragma unroll
      for (int j = 0; j < MG; ++j) {
        const int m = mrow(g0 + j);
        const int gi = m / a.x_group_rows, ri = m - gi * a.x_group_rows;
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          xv[j][ni] = (float4_t){0.f, 0.f, 0.f, 0.f};
          if (m < a.M) {
            if constexpr (EPI == EPI_RESID) xv[j][ni] = load4f(a.out_f32 + (int64_t)m * a.ldo + ncol(ni));
            else xv[j][ni] = load4f(a.pos + (int64_t)ri * a.N + ncol(ni));
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < MG; ++j) {
      const int m = mrow(g0 + j);
      if (m >= a.M) continue;
      const int gi = m / a.x_group_rows, ri = m - gi * a.x_group_rows;
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const int n = ncol(ni);
        float4_t v = acc[g0 + j][ni];
        if (a.bias) v += bv[ni];
        if constexpr (EPI == EPI_RESID) {
          float4_t c = xv[j][ni];
          c += v;
          store4(a.out_f32 + (int64_t)m * a.ldo + n, c[0], c[1], c[2], c[3]);
        } else if constexpr (EPI == EPI_GELU_POS) {
          const float4_t p = xv[j][ni];
          store4(a.out_f32 + (int64_t)m * a.ldo + n, gelu_f(v[0]) + p[0], gelu_f(v[1]) + p[1], gelu_f(v[2]) + p[2],
                 gelu_f(v[3]) + p[3]);
        } else {
          epilogue_store<T, EPI>(a, m, gi, ri, n, v);
        }
      }
    }
  }
}

template <typename T>
int launch_gemm(const GemmArgs& a, int epi, hipStream_t st);
// launch_gemm with the large-M tile chosen explicitly: 256 = k_gemm_256 where the shape
// allows it, 257 = the same with v_mfma_f32_32x32x16_f16 (A/B), 128 = k_gemm_tile (128 x 64
// tiles below 256 tiles), 129 = k_gemm_tile with 128 x 128 tiles only (tools/gemm_bench
// A/B; launch_gemm uses 256 unless WHISPER_HIP_GEMM)
template <typename T>
int launch_gemm_tiles(const GemmArgs& a, int epi, int tile_sel, hipStream_t st);

// decoder-step projections (k_proj, wh_proj.hip) into split-K partial slabs
// out_f32[z][M][N]; returns 0 and the split count, or < 0 when no tile configuration
// fits the shape (callers then use launch_gemm's EPI_PARTIAL path)
template <typename T>
// ev0/ev1 (optional): timestamps of the kernel's own dispatch (hipExtLaunchKernelGGL),
// i.e. its execution time as a profiler sees it, with no marker packets around it
int launch_proj_partial(const GemmArgs& a, int max_z, hipStream_t st, int* z_out, hipEvent_t ev0 = nullptr,
                        hipEvent_t ev1 = nullptr);

// single-window decoder-step projections (k_proj1, wh_proj.h): <= 8 rows, fused
// epilogue, optional LayerNorm prologue, in-launch split-K for the n-wide outputs;
// proj1_supported(R, n): model width n has a configuration; launch returns -1 otherwise
bool proj1_supported(int R, int n);
template <typename T>
int launch_proj1(const GemmArgs& a, int epi, bool ln, hipStream_t st, hipEvent_t ev0 = nullptr,
                 hipEvent_t ev1 = nullptr);

// split-K factor the skinny paths use for EPI_PARTIAL at this shape (<= min(16, max_z))
int gemv_ksplit(int M, int N, int K, int max_z = 16, int mt_block = 0);

}  // namespace wh
