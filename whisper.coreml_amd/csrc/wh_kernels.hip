// Attention, LayerNorm, embedding and log-mel kernels for libwhisper_hip.
#include "wh_kernels.h"

#include <cstdio>
#include <type_traits>
#include <cstdlib>

namespace wh {

// ============================================================ LayerNorm
// One wave per row: x f32 [rows][n] -> y T [rows][n]; biased variance, two-pass in
// registers (nn.LayerNorm semantics).  rows_in (nullable) gathers input rows.
template <typename T>
__global__ __launch_bounds__(256) void k_layernorm(const float* __restrict__ x, T* __restrict__ y, const float* __restrict__ gamma,
                                                   const float* __restrict__ beta, int rows, int n, float eps,
                                                   const int* __restrict__ rows_in) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int src = rows_in ? rows_in[row] : row;
  const float* xr = x + (int64_t)src * n;
  constexpr int MAXV = 8;  // n <= 64*4*8 = 2048
  float4_t v[MAXV];
  const int nv = n >> 2;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < nv) v[i] = load4f(xr + 4 * c);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
    if (lane + 64 * i < nv) s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
  const float mean = wave_sum(s) / (float)n;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < nv) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = v[i][j] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)n + eps);
  T* yr = y + (int64_t)row * n;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < nv) {
      const float4_t gm = load4f(gamma + 4 * c), bt = load4f(beta + 4 * c);
      store4(yr + 4 * c, (v[i][0] - mean) * rstd * gm[0] + bt[0], (v[i][1] - mean) * rstd * gm[1] + bt[1],
             (v[i][2] - mean) * rstd * gm[2] + bt[2], (v[i][3] - mean) * rstd * gm[3] + bt[3]);
    }
  }
}

template <typename T>
void launch_layernorm(const float* x, T* y, const float* g, const float* b, int rows, int n, float eps,
                      const int* rows_in, hipStream_t st) {
  if (rows <= 0) return;
  k_layernorm<T><<<(rows + 3) / 4, 256, 0, st>>>(x, y, g, b, rows, n, eps, rows_in), wh_launched("k_layernorm");
}

// x[r] += bias + sum_s part[s][r] (fixed order: deterministic split-K reduction of the
// residual GEMVs), then y = LayerNorm(x).  One 256-thread block per row; every load
// of the row is issued before the first reduction (latency-bound at decode sizes).
// PF (round 6): the workgroup also carries its share of an L2Prefetch (wh_kernels.h) for the
// next launch, issued after its own loads (they return first) and waited for at its end.
template <typename T, int NS, int MAXV = 2, typename S = float, bool PF = false>
__global__ __launch_bounds__(512) void k_resid_ln(float* __restrict__ x, const S* __restrict__ part, int nsplit,
                                                  int64_t part_stride, const float* __restrict__ bias,
                                                  T* __restrict__ y, const float* __restrict__ gamma,
                                                  const float* __restrict__ beta, int n, float eps, L2Prefetch pf) {
  __shared__ float red[2][8];
  __shared__ __attribute__((aligned(16))) char pf_sink[PF ? 1024 : 16];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, NT = blockDim.x, nwv = NT >> 6;
  CT_MARK(CT_RESID_LN, 0);
  float* xr = x + (int64_t)row * n;
  // NT * 4 * MAXV >= n (n <= 2048): 256 threads x 2 float4, or ceil(n / 256) waves x 1
  const int nv = n >> 2;
  float4_t v[MAXV], gm[MAXV], bt[MAXV];
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = tid + NT * i;
    if (c < nv) {
      // LayerNorm's gamma / beta ride with the first round trip, not after the reductions
      gm[i] = load4f(gamma + 4 * c);
      bt[i] = load4f(beta + 4 * c);
      float4_t a = load4f(xr + 4 * c);
      // the slabs' raw elements first, converted after every load is issued (an fp16 slab
      // converted where it is loaded puts a wait behind each predicated load)
      typedef typename std::conditional<sizeof(S) == 2, half4_t, float4_t>::type R4;
      R4 pp[NS > 0 ? NS : 1];
#pragma unroll
      for (int sp = 0; sp < NS; ++sp)
        if (sp < nsplit) pp[sp] = *reinterpret_cast<const R4*>(part + sp * part_stride + (int64_t)row * n + 4 * c);
      if (bias) a += load4f(bias + 4 * c);
#pragma unroll
      for (int sp = 0; sp < NS; ++sp)
        if (sp < nsplit) a += (float4_t){(float)pp[sp][0], (float)pp[sp][1], (float)pp[sp][2], (float)pp[sp][3]};
      v[i] = a;
    }
  }
  if constexpr (PF) {
    // this workgroup's share of its XCD's byte range, in 1 KB blocks dealt to its waves
    const int xcd = blockIdx.x & 7, idx = blockIdx.x >> 3, m = ((int)gridDim.x - xcd + 7) >> 3;
    const int64_t b0 = pf.lo[xcd] * pf.unit, nb = (pf.hi[xcd] - pf.lo[xcd]) * pf.unit / 1024;
    const int64_t k0 = nb * idx / m, k1 = nb * (idx + 1) / m;
    for (int64_t k = k0 + wv; k < k1; k += nwv)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(pf.base + b0 + k * 1024 + lane * 16),
                                       (__attribute__((address_space(3))) void*)(pf_sink), 16, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
    if (tid + NT * i < nv) {
      store4(xr + 4 * (tid + NT * i), v[i][0], v[i][1], v[i][2], v[i][3]);
      s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
    }
  s = wave_sum(s);
  if (lane == 0) red[0][wv] = s;
  __syncthreads();
  CT_MARK(CT_RESID_LN, 1);
  float tot = 0.f;
  for (int k = 0; k < nwv; ++k) tot += red[0][k];
  const float mean = tot / (float)n;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
    if (tid + NT * i < nv) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = v[i][j] - mean;
        q += d * d;
      }
    }
  q = wave_sum(q);
  if (lane == 0) red[1][wv] = q;
  __syncthreads();
  float qt = 0.f;
  for (int k = 0; k < nwv; ++k) qt += red[1][k];
  const float rstd = rsqrtf(qt / (float)n + eps);
  T* yr = y + (int64_t)row * n;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = tid + NT * i;
    if (c < nv)
      store4(yr + 4 * c, (v[i][0] - mean) * rstd * gm[i][0] + bt[i][0], (v[i][1] - mean) * rstd * gm[i][1] + bt[i][1],
             (v[i][2] - mean) * rstd * gm[i][2] + bt[i][2], (v[i][3] - mean) * rstd * gm[i][3] + bt[i][3]);
  }
  if constexpr (PF) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the workgroup
  CT_END(CT_RESID_LN);
}


template <typename T>
void launch_resid_ln(float* x, const float* part, int nsplit, int64_t part_stride, const float* bias, T* y,
                     const float* g, const float* b, int rows, int n, float eps, hipStream_t st, int slab_half,
                     const L2Prefetch* pf) {
  if (rows <= 0) return;
  const L2Prefetch none;
  // one float4 per thread (n <= 2048; 1280: 5 waves); tuning builds WHISPER_HIP_RLN_256=1
  // for the round-3 form (256 threads, up to two float4 each)
  const char* e = tune_env("WHISPER_HIP_RLN_256");
  const int nt = (e && atoi(e) == 1) ? 256 : ((n >> 2) + 63) / 64 * 64;
  if (slab_half && nsplit > 0 && nt != 256) {  // fp16 slabs (fp16 contexts, k_proj)
    const half_t* ph = reinterpret_cast<const half_t*>(part);
    if (pf && pf->base) {
      if (nsplit <= 4) k_resid_ln<T, 4, 1, half_t, true><<<rows, nt, 0, st>>>(x, ph, nsplit, part_stride, bias, y, g, b, n, eps, *pf), wh_launched("k_resid_ln<pf>");
      else k_resid_ln<T, 16, 1, half_t, true><<<rows, nt, 0, st>>>(x, ph, nsplit, part_stride, bias, y, g, b, n, eps, *pf), wh_launched("k_resid_ln<pf>");
      return;
    }
    if (nsplit <= 4) k_resid_ln<T, 4, 1, half_t><<<rows, nt, 0, st>>>(x, ph, nsplit, part_stride, bias, y, g, b, n, eps, none), wh_launched("k_resid_ln");
    else k_resid_ln<T, 16, 1, half_t><<<rows, nt, 0, st>>>(x, ph, nsplit, part_stride, bias, y, g, b, n, eps, none), wh_launched("k_resid_ln");
    return;
  }
#define RLN(NS_, MV_) \
  k_resid_ln<T, NS_, MV_><<<rows, nt, 0, st>>>(x, part, NS_ ? nsplit : 0, part_stride, bias, y, g, b, n, eps, none), wh_launched("k_resid_ln")
  if (nsplit <= 0) {
    if (nt == 256) RLN(0, 2); else RLN(0, 1);
  } else if (nsplit <= 4) {
    if (nt == 256) RLN(4, 2); else RLN(4, 1);
  } else {
    if (nt == 256) RLN(16, 2); else RLN(16, 1);
  }
#undef RLN
}

// ============================================================ encoder flash attention (non-causal)
// qkv: [T rows][ld] per window (q at col h*64, k at ns + h*64); K is pre-scaled by 1/8
// (folded into Wk at load, exact).  vt: V^T per (window, head) [64][tkp] with keys
// permuted within 32-key groups (EPI_QKV_ENC), so a 64-key tile of V^T is staged with
// 16 B copies and each P.V fragment is one 16 B LDS read.  The last tile reads 32 keys
// past tkp (the next row, or 64 elements of slack): finite values under p = 0.
// out: [T][ns] per window.
// Block = ENC_NW waves x ENC_RT row tiles of 16 queries; each K / V fragment read from
// LDS feeds ENC_RT MFMAs.  S^T = K Q^T and O^T = V^T P^T so each lane owns one query row per row tile
// (see wh_common.h).
// query row tiles per wave: 2 measured 414 vs 289 us in round 2 (264 VGPRs, one block per
// CU) and, after the round-3 VALU trims (134 VGPRs), 3.60 vs 3.45 ms per encoder window
// (profiles/r03/enc_rt_ab.txt)
constexpr int ENC_RT = 1;
// ENC_NW waves per block: the K/V tile staged once for 16 * ENC_NW * ENC_RT queries; 8,
// or 4 when 8-wave blocks would give fewer than two per CU (one window: 240 -> 480 blocks)
template <typename T, int ENC_NW, int RT = ENC_RT>
__global__ __launch_bounds__(64 * ENC_NW) void k_attn_enc(const T* __restrict__ qkv, int ld, int ns, int Tlen,
                                                  int64_t win_stride_in, const T* __restrict__ vt, int tkp,
                                                  T* __restrict__ out, int64_t win_stride_out) {
  constexpr int NT = 64 * ENC_NW;
  // LDS row stride: 160 B for fp16 (40 dwords) makes the fragment reads (ds_read_b128,
  // lane (r, g) at row r, 16 B chunk 2s + g) conflict-free in every 16-lane group of the
  // instruction; the round-2 stride of 144 B gave 40 % extra LDS cycles
  // (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, profiles/r03/enc_pmc.json)
  constexpr int RS = 64 * (int)sizeof(T) + (sizeof(T) == 2 ? 32 : 16);
  __shared__ __attribute__((aligned(16))) char Ks[2][64 * RS];
  __shared__ __attribute__((aligned(16))) char Vt[2][64 * RS];
  const int h = blockIdx.y, w = blockIdx.z, H = gridDim.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const T* base = qkv + (int64_t)w * win_stride_in;
  const T* vbase = vt + ((int64_t)w * H + h) * 64 * tkp;
  const int q0 = blockIdx.x * 16 * ENC_NW * RT + wave * 16 * RT;
  Frag<T> qf[RT][2];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const int qrow = min(q0 + 16 * t + r, Tlen - 1);
    frag_load(qf[t][0], base + (int64_t)qrow * ld + h * 64 + 8 * g);
    frag_load(qf[t][1], base + (int64_t)qrow * ld + h * 64 + 32 + 8 * g);
  }

  float4_t acc_o[RT][4];
  float m_run[RT], l_run[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    m_run[t] = -INFINITY;
    l_run[t] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) acc_o[t][i] = (float4_t){0.f, 0.f, 0.f, 0.f};
  }
  constexpr float LOG2E = 1.4426950408889634f;
  constexpr int EPC = 16 / (int)sizeof(T);       // elements per 16 B chunk
  constexpr int CPR = 64 / EPC;                   // chunks per 64-element row
  constexpr int NCH = 64 * CPR / NT;              // chunks per thread per operand
  const int nkb = (Tlen + 63) / 64;
  // 64 keys x 64 d of K and 64 d x 64 (permuted) keys of V^T per tile; the next tile's
  // loads are in flight while this one is computed (double-buffered LDS, one barrier
  // per tile that waits for LDS only, so the prefetch stays in flight)
  float4_t kv[NCH], vv[NCH];
  auto load_tile = [&](int kb) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = tid + NT * i, row = c / CPR, ch = c % CPR;
      const int kr = min(kb * 64 + row, Tlen - 1);
      kv[i] = *reinterpret_cast<const float4_t*>(base + (int64_t)kr * ld + ns + h * 64 + ch * EPC);
      vv[i] = *reinterpret_cast<const float4_t*>(vbase + (int64_t)row * tkp + kb * 64 + ch * EPC);
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = tid + NT * i, row = c / CPR, ch = c % CPR;
      *reinterpret_cast<float4_t*>(Ks[buf] + row * RS + ch * 16) = kv[i];
      *reinterpret_cast<float4_t*>(Vt[buf] + row * RS + ch * 16) = vv[i];
    }
  };
  load_tile(0);
  store_tile(0);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  for (int kb = 0; kb < nkb; ++kb) {
    const int buf = kb & 1;
    load_tile(min(kb + 1, nkb - 1));
    const char* Kb = Ks[buf];
    const char* Vb = Vt[buf];
    float4_t sc[RT][4];
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) sc[t][kt] = (float4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        Frag<T> kf;
        frag_load(kf, reinterpret_cast<const T*>(Kb + (kt * 16 + r) * RS) + 32 * s + 8 * g);
#pragma unroll
        for (int t = 0; t < RT; ++t) mfma_step(sc[t][kt], kf, qf[t][s]);
      }
    Frag<T> pf[RT][2];
    float alpha[RT];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      // mask the ragged last tile (a uniform branch: every other tile is whole); row max
      // over the 64 keys
      if (kb * 64 + 64 > Tlen) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (kb * 64 + kt * 16 + 4 * g + j >= Tlen) sc[t][kt][j] = -INFINITY;
      }
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j) mx = fmaxf(mx, sc[t][kt][j]);
      mx = xor16_max(mx);
      mx = xor32_max(mx);
      const float m_new = fmaxf(m_run[t], mx);
      alpha[t] = hw_exp2((m_run[t] - m_new) * LOG2E);
      // p = 2^(s log2e - m log2e): one fma per score; the row sum in pairs (packed adds)
      const float mL = m_new * LOG2E;
      f32x2_t ps2 = {0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int j = 0; j < 4; j += 2) {
          const float p0 = hw_exp2(__builtin_fmaf(sc[t][kt][j], LOG2E, -mL));
          const float p1 = hw_exp2(__builtin_fmaf(sc[t][kt][j + 1], LOG2E, -mL));
          ps2 += (f32x2_t){p0, p1};
          pf[t][kt >> 1].v[(kt & 1) * 4 + j] = from_f32<T>(p0);
          pf[t][kt >> 1].v[(kt & 1) * 4 + j + 1] = from_f32<T>(p1);
        }
      float ps = ps2[0] + ps2[1];
      ps = xor16_sum(ps);
      ps = xor32_sum(ps);
      l_run[t] = l_run[t] * alpha[t] + ps;
      m_run[t] = m_new;
    }
    // rescale the output only when some row's running max moved (alpha == 1 otherwise:
    // after the first tiles the max mostly settles; a wave-uniform branch, exact either way)
#pragma unroll
    for (int t = 0; t < RT; ++t)
      if (__any(alpha[t] != 1.f)) {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) acc_o[t][dt] *= alpha[t];
      }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        // lane (r, g): V^T[d = dt*16 + r][keys 32s + {4g..4g+3, 16+4g..16+4g+3}], which
        // the permuted layout stores contiguously at 32s + 8g
        Frag<T> vf;
        frag_load(vf, reinterpret_cast<const T*>(Vb + (dt * 16 + r) * RS) + 32 * s + 8 * g);
#pragma unroll
        for (int t = 0; t < RT; ++t) mfma_step(acc_o[t][dt], vf, pf[t][s]);
      }
    }
    store_tile(buf ^ 1);  // buffer last read in the previous tile, before that barrier
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const int q = q0 + 16 * t + r;
    if (q < Tlen) {
      const float inv = 1.f / l_run[t];
      T* o = out + (int64_t)w * win_stride_out + (int64_t)q * ns + h * 64;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        store4(o + dt * 16 + 4 * g, acc_o[t][dt][0] * inv, acc_o[t][dt][1] * inv, acc_o[t][dt][2] * inv,
               acc_o[t][dt][3] * inv);
    }
  }
}

template <typename T>
void launch_attn_enc(const T* qkv, int ld, int ns, int H, int Tlen, int nwin, int64_t wsi, const T* vt, int tkp, T* out,
                     int64_t wso, hipStream_t st) {
  const int blocks8 = (Tlen + 127) / 128 * H * nwin;
  if (blocks8 < 512) {
    dim3 grid((Tlen + 63) / 64, H, nwin);
    k_attn_enc<T, 4><<<grid, 256, 0, st>>>(qkv, ld, ns, Tlen, wsi, vt, tkp, out, wso), wh_launched("k_attn_enc");
  } else {
    dim3 grid((Tlen + 127) / 128, H, nwin);
    k_attn_enc<T, 8><<<grid, 512, 0, st>>>(qkv, ld, ns, Tlen, wsi, vt, tkp, out, wso), wh_launched("k_attn_enc");
  }
}

// One online-softmax pass of the coalesced-K self-attention (round 6): lane (kg, dc) holds
// the 16-B chunk dc (dims dc .. dc+7) of keys key0 + 8u, u < NU, of both K and V (eight
// lanes per 128-B row, so a load instruction covers whole rows); keys >= lim are masked.  A
// key's score is its 8 chunk partials summed across the group's lanes with DPP (pairs, quads,
// then the other quad: after the quad steps a quad's lanes agree, so the half-row mirror is a
// partner; each step adds two operands equal for both lanes, so the 8 lanes hold the same
// sum) and lands in the lanes whose V chunks it weights: no LDS hand-off of the weights.
template <typename T, int NU>
WH_DEV void kco_pass(const float (&qd8)[8], const Frag<T> (&k)[NU], const Frag<T> (&v)[NU], int key0, int lim,
                     float& m, float& lsum, float (&o)[8]) {
  constexpr int XOR1 = 0xB1, XOR2 = 0x4E, HALF_MIRROR = 0x141;  // quad_perm [1,0,3,2], [2,3,0,1]
  float s[NU], mx = -INFINITY;
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    float a = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) a += qd8[e] * to_f32(k[u].v[e]);
    a += dpp_f<XOR1>(a);
    a += dpp_f<XOR2>(a);
    a += dpp_f<HALF_MIRROR>(a);
    s[u] = a;
    if (key0 + 8 * u < lim) mx = fmaxf(mx, a);
  }
  mx = fmaxf(mx, dpp_f<DPP_ROR8>(mx));
  mx = xor16_max(mx);
  mx = xor32_max(mx);
  const float mn = fmaxf(m, mx), scale = __expf(m - mn);
  m = mn;
  float es = 0.f;
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    s[u] = key0 + 8 * u < lim ? __expf(s[u] - mn) : 0.f;
    es += s[u];
  }
  lsum = lsum * scale + xor32_sum(xor16_sum(xor8_sum(es)));
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] *= scale;
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] += s[u] * to_f32(v[u].v[e]);
}

// ============================================================ decoder self-attention
// One wave per (row, head).  Keys = positions 0..pos of the row's sequence; position
// p < pos lives in beam slot anc[win][slot][p] (beam reorder by index indirection,
// no KV copies), position pos in the row's own slot.  Cache: [win][slot][head][ctx][64].
// PIPE (fp16, round 4): 64-key passes with the next pass's loads in flight, as
// k_self_attn_qkv<T, true>.  KCO (fp16, round 6): the 128-key passes with K read like V
// (kco_pass)
template <typename T, bool PIPE = false, bool KCO = false>
__global__ __launch_bounds__(64) void k_self_attn(const T* __restrict__ q, int ldq, const T* __restrict__ kc,
                                                  const T* __restrict__ vc, const int* __restrict__ row_win,
                                                  const int* __restrict__ row_slot, const int* __restrict__ row_pos,
                                                  const int* __restrict__ anc, int anc_beams, int nbeam, int H,
                                                  int ctx, T* __restrict__ out, int ldo, int kco_min = 0) {
  CT_MARK(CT_SELF_ATTN, 0);

  __shared__ float sc[512];
  __shared__ int slot_of[512];
  const int row = blockIdx.x, h = blockIdx.y, lane = threadIdx.x;
  // the query row leaves first, one element per lane (a vector load: a uniform-address
  // load compiled to scalar loads that the compiler sank behind the ancestry's round trip);
  // the fp16 path reads it from LDS (qs), the others unpack it into registers (qv)
  __shared__ float qs[64];
  const T q_lane = q[(int64_t)row * ldq + h * 64 + lane];
  const int w = row_win[row], sl = row_slot[row], pos = row_pos[row];
  const int* an = anc + ((int64_t)w * anc_beams + sl) * ctx;
  float qv[64];
  auto unpack_q = [&] {  // (after qs is written and its lgkmcnt drained)
#pragma unroll
    for (int c = 0; c < 64; ++c) qv[c] = qs[c];
  };
  const int64_t head_stride = (int64_t)ctx * 64;
  const int64_t wbase = (int64_t)w * nbeam;
  auto kv_off = [&](int slot, int p) -> int64_t { return ((wbase + slot) * H + h) * head_stride + (int64_t)p * 64; };
  // cached K / V reads: 32-bit byte offsets into buffer resources (a context caps one
  // layer's cache below 2 GiB, wh_runtime.hip); slot_of holds each position's slot already
  // multiplied by the slot stride, so an address is two adds and a shift (the int64 form
  // was a chain of 64-bit multiplies per load: ~1 us of VALU per pass at 100 rows)
  constexpr int TB = (int)sizeof(T), ROWB = 64 * TB;
  const int slotB = H * ctx * ROWB, baseB = ((int)wbase * H + h) * ctx * ROWB;
  const auto rk = wt_rsrc(kc), rv = wt_rsrc(vc);
  if constexpr (sizeof(T) == 2 && PIPE) {
    int sv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) sv[i] = an[min(lane + 64 * i, ctx - 1)];
    qs[lane] = to_f32(q_lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int pp = lane + 64 * i;
      if (pp <= pos) slot_of[pp] = (pp == pos ? sl : sv[i]) * slotB;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: its own LDS writes
    unpack_q();
    const int kg = lane >> 3, dc = (lane & 7) * 8;
    float m = -INFINITY, lsum = 0.f, o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.f;
    auto load = [&](int p0, Frag<T>(&k)[8], Frag<T>(&v)[8]) {
      const int pa = min(p0 + lane, pos);
      const int ra = baseB + slot_of[pa] + pa * ROWB;
#pragma unroll
      for (int c = 0; c < 8; ++c) frag_load_buf(k[c], rk, ra + 8 * c * TB);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int pc = min(p0 + kg + 8 * u, pos);
        frag_load_buf(v[u], rv, baseB + slot_of[pc] + pc * ROWB + dc * TB);
      }
    };
    auto pass = [&](int p0, const Frag<T>(&k)[8], const Frag<T>(&v)[8]) {
      float sa = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) sa += qv[8 * c + e] * to_f32(k[c].v[e]);
      const bool va = p0 + lane <= pos;
      const float mp = wave_max(va ? sa : -INFINITY);
      const float mn = fmaxf(m, mp), scale = __expf(m - mn);
      m = mn;
      const float ea = va ? __expf(sa - m) : 0.f;
      lsum = lsum * scale + wave_sum(ea);
      sc[lane] = ea;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] *= scale;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float pw = sc[kg + 8 * u];  // 0 past the end
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += pw * to_f32(v[u].v[e]);
      }
    };
    Frag<T> ka[8], va[8], kb[8], vb[8];
    load(0, ka, va);
    int p0 = 0;
    for (; p0 + 64 <= pos; p0 += 128) {
      load(p0 + 64, kb, vb);
      pass(p0, ka, va);
      if (p0 + 128 <= pos) load(p0 + 128, ka, va);
      pass(p0 + 64, kb, vb);
    }
    if (p0 <= pos) pass(p0, ka, va);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = xor8_sum(o[e]);
      o[e] = xor16_sum(o[e]);
      o[e] = xor32_sum(o[e]);
    }
    if (kg == 0) {
      const float inv = 1.f / lsum;
      T* op = out + (int64_t)row * ldo + h * 64 + dc;
      store4(op, o[0] * inv, o[1] * inv, o[2] * inv, o[3] * inv);
      store4(op + 4, o[4] * inv, o[5] * inv, o[6] * inv, o[7] * inv);
    }
    CT_END(CT_SELF_ATTN);
    return;
  }
  if constexpr (sizeof(T) == 2 && KCO) {
    if (pos + 1 > kco_min) {  // (one 128-key pass below: the lane-per-key form)
      int sv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) sv[i] = an[min(lane + 64 * i, ctx - 1)];
      qs[lane] = to_f32(q_lane);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int pp = lane + 64 * i;
        if (pp <= pos) slot_of[pp] = (pp == pos ? sl : sv[i]) * slotB;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: its own LDS writes
      const int kg = lane >> 3, dc = (lane & 7) * 8;
      float qd8[8], m = -INFINITY, lsum = 0.f, o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        qd8[e] = qs[dc + e];
        o[e] = 0.f;
      }
      for (int p0 = 0; p0 <= pos; p0 += 128) {
        Frag<T> k[16], v[16];
        int off[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int pc = min(p0 + kg + 8 * u, pos);
          off[u] = baseB + slot_of[pc] + pc * ROWB + dc * TB;
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) frag_load_buf(k[u], rk, off[u]);
#pragma unroll
        for (int u = 0; u < 16; ++u) frag_load_buf(v[u], rv, off[u]);
        kco_pass<T, 16>(qd8, k, v, p0 + kg, pos + 1, m, lsum, o);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        o[e] = xor8_sum(o[e]);
        o[e] = xor16_sum(o[e]);
        o[e] = xor32_sum(o[e]);
      }
      if (kg == 0) {
        const float inv = 1.f / lsum;
        T* op = out + (int64_t)row * ldo + h * 64 + dc;
        store4(op, o[0] * inv, o[1] * inv, o[2] * inv, o[3] * inv);
        store4(op + 4, o[4] * inv, o[5] * inv, o[6] * inv, o[7] * inv);
      }
      CT_END(CT_SELF_ATTN);
      return;
    }
  }
  if constexpr (sizeof(T) == 2) {
    // round 3 (fp16): the k_self_attn_qkv schedule — the ancestry of every context
    // position in the first round trip (8 per lane, with q), then per 128-key pass K
    // (lane per key) and V (8 lanes per key) in ONE round trip with an online softmax
    // across passes; the round-2 form (ancestry, then K, then V four keys per lane at a
    // time) took up to 8 dependent round trips at mid context (9.6 us average per layer
    // over a one-window decode, profiles/r03/bench_eager_rocprof_summary.txt)
    int sv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) sv[i] = an[min(lane + 64 * i, ctx - 1)];
    qs[lane] = to_f32(q_lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int pp = lane + 64 * i;
      if (pp <= pos) slot_of[pp] = (pp == pos ? sl : sv[i]) * slotB;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: its own LDS writes
    const int kg = lane >> 3, dc = (lane & 7) * 8;
    float m = -INFINITY, lsum = 0.f, o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.f;
    for (int p0 = 0; p0 <= pos; p0 += 128) {
      const int pa = min(p0 + lane, pos), pb = min(p0 + 64 + lane, pos);
      const int ra = baseB + slot_of[pa] + pa * ROWB, rb = baseB + slot_of[pb] + pb * ROWB;
      Frag<T> ka[8], kb[8], vf[16];
#pragma unroll
      for (int c = 0; c < 8; ++c) frag_load_buf(ka[c], rk, ra + 8 * c * TB);
#pragma unroll
      for (int c = 0; c < 8; ++c) frag_load_buf(kb[c], rk, rb + 8 * c * TB);
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int pc = min(p0 + kg + 8 * u, pos);
        frag_load_buf(vf[u], rv, baseB + slot_of[pc] + pc * ROWB + dc * TB);
      }
      __builtin_amdgcn_sched_barrier(0);  // every load of the pass ahead of the math
      float sa = 0.f, sb = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float4_t q0 = *reinterpret_cast<const float4_t*>(&qs[8 * c]);
        const float4_t q1 = *reinterpret_cast<const float4_t*>(&qs[8 * c + 4]);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float qe = e < 4 ? q0[e] : q1[e - 4];
          sa += qe * to_f32(ka[c].v[e]);
          sb += qe * to_f32(kb[c].v[e]);
        }
      }
      const bool va = p0 + lane <= pos, vb = p0 + 64 + lane <= pos;
      const float mp = wave_max(fmaxf(va ? sa : -INFINITY, vb ? sb : -INFINITY));
      const float mn = fmaxf(m, mp), scale = __expf(m - mn);
      m = mn;
      const float ea = va ? __expf(sa - m) : 0.f, eb = vb ? __expf(sb - m) : 0.f;
      lsum = lsum * scale + wave_sum(ea + eb);
      sc[lane] = ea;
      sc[64 + lane] = eb;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] *= scale;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const float pw = sc[kg + 8 * u];  // 0 past the end
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += pw * to_f32(vf[u].v[e]);
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = xor8_sum(o[e]);
      o[e] = xor16_sum(o[e]);
      o[e] = xor32_sum(o[e]);
    }
    if (kg == 0) {
      const float inv = 1.f / lsum;
      T* op = out + (int64_t)row * ldo + h * 64 + dc;
      store4(op, o[0] * inv, o[1] * inv, o[2] * inv, o[3] * inv);
      store4(op + 4, o[4] * inv, o[5] * inv, o[6] * inv, o[7] * inv);
    }
    CT_END(CT_SELF_ATTN);
    return;
  }
  qs[lane] = to_f32(q_lane);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: its own LDS write
  unpack_q();
  // scores: lane per key
  float mx = -INFINITY;
  for (int p = lane; p <= pos; p += 64) {
    const int slot = ((p == pos) ? sl : an[p]) * slotB;
    slot_of[p] = slot;
    const int kr = baseB + slot + p * ROWB;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 64; c += 8) {
      Frag<T> f;
      frag_load_buf(f, rk, kr + c * TB);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += qv[c + e] * to_f32(f.v[e]);
    }
    sc[p] = s;
    mx = fmaxf(mx, s);
  }
  mx = wave_max(mx);
  float sum = 0.f;
  for (int p = lane; p <= pos; p += 64) {
    const float e = __expf(sc[p] - mx);
    sc[p] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  __syncthreads();
  // P.V: lane = (key group kg = lane>>3, dim chunk dc = lane&7): 8 keys x 128 B per instruction
  const int kg = lane >> 3, dc = (lane & 7) * 8;
  float o[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = 0.f;
  int p = kg;
  for (; p + 24 <= pos; p += 32) {  // 4 keys per lane in flight
    Frag<T> f[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) frag_load_buf(f[u], rv, baseB + slot_of[p + 8 * u] + (p + 8 * u) * ROWB + dc * TB);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float pw = sc[p + 8 * u];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] += pw * to_f32(f[u].v[e]);
    }
  }
  for (; p <= pos; p += 8) {
    Frag<T> f;
    frag_load_buf(f, rv, baseB + slot_of[p] + p * ROWB + dc * TB);
    const float pw = sc[p];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] += pw * to_f32(f.v[e]);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    o[e] = xor8_sum(o[e]);
    o[e] = xor16_sum(o[e]);
    o[e] = xor32_sum(o[e]);
  }
  if (kg == 0) {
    const float inv = 1.f / sum;
    T* op = out + (int64_t)row * ldo + h * 64 + dc;
    store4(op, o[0] * inv, o[1] * inv, o[2] * inv, o[3] * inv);
    store4(op + 4, o[4] * inv, o[5] * inv, o[6] * inv, o[7] * inv);
  }
  CT_END(CT_SELF_ATTN);
}

template <typename T>
void launch_self_attn(const T* q, int ldq, const T* kc, const T* vc, const int* rw, const int* rs, const int* rp,
                      const int* anc, int anc_beams, int nbeam, int H, int ctx, T* out, int ldo, int rows,
                      hipStream_t st) {
  if (rows <= 0) return;
  // tuning build only (WHISPER_HIP_SA_PIPE1=1): the pipelined 64-key passes at one window
  // measured p50 1.670 -> 1.679 ms per token (profiles/r04/self_attn_pipe_ab.txt): not kept
  static const bool pipe = [] {
    const char* e = tune_env("WHISPER_HIP_SA_PIPE1");
    return e && e[0] == '1';
  }();
  if constexpr (sizeof(T) == 2) {
    if (self_attn_kco_on()) {
      k_self_attn<T, false, true><<<dim3(rows, H), 64, 0, st>>>(q, ldq, kc, vc, rw, rs, rp, anc, anc_beams, nbeam, H,
                                                                ctx, out, ldo, self_attn_kco_min()), wh_launched("k_self_attn");
      return;
    }
    if (pipe) {
      k_self_attn<T, true><<<dim3(rows, H), 64, 0, st>>>(q, ldq, kc, vc, rw, rs, rp, anc, anc_beams, nbeam, H, ctx, out,
                                                         ldo), wh_launched("k_self_attn");
      return;
    }
  }
  k_self_attn<T><<<dim3(rows, H), 64, 0, st>>>(q, ldq, kc, vc, rw, rs, rp, anc, anc_beams, nbeam, H, ctx, out, ldo), wh_launched("k_self_attn");
}

// Step-mode variant: the QKV projection arrives as split-K fp32 partial slabs
// part[z][row][3n] (k_gemv_*, EPI_PARTIAL).  Each (row, head) wave sums its q/k/v
// slices in fixed order, adds the bias, writes k/v (rounded to T) into its own slot
// at position pos and attends with them directly (no read-back of the fresh row).
// Only valid when no other row of the launch needs this row's K/V (one row per beam).
// Grid: one single-wave workgroup per (row, head), rows w * G + beam; the logical order
// (window, head, beam) is laid over the XCDs in contiguous runs (xcd_remap), so the G
// beams of one (window, head), whose ancestries mostly name the same cached (slot,
// position) rows, run on one XCD and share its L2 (x-fastest order put them on G
// different XCDs).
//
// PIPE (fp16, round 4): passes of 64 keys, the NEXT pass's K and V loads issued before
// the current pass is computed (two register buffers of 8 K + 8 V fragments), q read from
// LDS: at long contexts the passes' round trips overlap instead of adding up (the step's
// growth over the decode is those round trips, profiles/r04/self_attn_grp64_ab.txt).
// PIPE 3 (round 6): the PIPE 1 passes with K read like V — lane (kg, dc) holds the 16-B
// chunk dc of keys kg + 8u, eight lanes per 128-B key row — so one load instruction covers
// 8 whole rows (the lane-per-key form touched 64 rows, 16 B of each, per instruction, and
// the rows' other chunks came back by later instructions from wherever the lines still
// were).  A key's score is its 8 chunk partials summed across the group's lanes (DPP) and
// lands in the lanes whose V chunks it weights: no LDS hand-off of the probabilities.
template <typename T, int PIPE = 0, typename S = float>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_self_attn_qkv(const S* __restrict__ part, int nsplit, int64_t part_stride,
                                                      const float* __restrict__ bqkv, int ns, T* __restrict__ kc,
                                                      T* __restrict__ vc, const int* __restrict__ row_win,
                                                      const int* __restrict__ row_slot, const int* __restrict__ row_pos,
                                                      const int* __restrict__ anc, int anc_beams, int nbeam, int H,
                                                      int ctx, T* __restrict__ out, int ldo, int kco_min = 0) {
  __shared__ float sc[512];
  __shared__ int slot_of[512];
  __shared__ float qs[64], vs[64];
  const int lane = threadIdx.x, G = anc_beams;
  CT_MARK(CT_SELF_ATTN, 0);
  // step rows: window w = row / G, beam slot = row % G (row_win / row_slot hold the same)
  const int L = xcd_remap(blockIdx.x, gridDim.x), sl = L % G, wh = L / G, h = wh % H, w = wh / H, row = w * G + sl;
  const int* an = anc + ((int64_t)w * anc_beams + sl) * ctx;
  const int64_t head_stride = (int64_t)ctx * 64;
  const int64_t wbase = (int64_t)w * nbeam;
  auto kv_off = [&](int slot, int p) -> int64_t { return ((wbase + slot) * H + h) * head_stride + (int64_t)p * 64; };
  // cached K / V reads: 32-bit byte offsets into buffer resources (a context caps one
  // layer's cache below 2 GiB, wh_runtime.hip); slot_of holds each position's slot already
  // multiplied by the slot stride, so an address is two adds and a shift (the int64 form
  // was a chain of 64-bit multiplies per load: ~1 us of VALU per pass at 100 rows)
  constexpr int TB = (int)sizeof(T), ROWB = 64 * TB;
  const int slotB = H * ctx * ROWB, baseB = ((int)wbase * H + h) * ctx * ROWB;
  const auto rk = wt_rsrc(kc), rv = wt_rsrc(vc);
  // one round trip for everything that does not depend on this step's projection:
  // the position, the ancestry slot of every context position (8 per lane, clamped to
  // the context, issued together) and the q/k/v partial slabs of this row and head
  // (lane = d)
  const int pos = row_pos[row];
  int sv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) sv[i] = an[min(lane + 64 * i, ctx - 1)];
  float qd, kd, vd;
  {
    // fp16 slabs: all 16 slab indices loaded unconditionally (clamped to the last split:
    // the same addresses again), converted after every load is issued — guarded per split,
    // the compiler converted each fp16 element inside its branch and waited there
    constexpr bool H16 = sizeof(S) == 2;
    const S* pr = part + (int64_t)row * 3 * ns + h * 64 + lane;
    qd = bqkv[h * 64 + lane];
    kd = bqkv[ns + h * 64 + lane];
    vd = bqkv[2 * ns + h * 64 + lane];
    S a0[16], a1[16], a2[16];
#pragma unroll
    for (int z = 0; z < 16; ++z)
      if (H16 || z < nsplit) {
        const int64_t zo = (int64_t)(H16 ? min(z, nsplit - 1) : z) * part_stride;
        a0[z] = pr[zo];
        a1[z] = pr[zo + ns];
        a2[z] = pr[zo + 2 * ns];
      }
    if constexpr (H16) {  // keeps the loads here (the compiler sank each into its split's sum,
      // and the position's scalar load behind them all)
      asm volatile("" ::"s"(pos));
#pragma unroll
      for (int z = 0; z < 16; ++z) asm volatile("" ::"v"(a0[z]), "v"(a1[z]), "v"(a2[z]));
    }
    auto f32 = [](S r) -> float { return (float)r; };
#pragma unroll
    for (int z = 0; z < 16; ++z)
      if (z < nsplit) {
        qd += f32(a0[z]);
        kd += f32(a1[z]);
        vd += f32(a2[z]);
      }
  }
  for (int i = 0; i < 8; ++i)
    if (lane + 64 * i < pos) slot_of[lane + 64 * i] = sv[i] * slotB;
  const int plast = max(pos - 1, 0);
  const T qT = from_f32<T>(qd), kT = from_f32<T>(kd), vT = from_f32<T>(vd);
  kc[kv_off(sl, pos) + lane] = kT;
  vc[kv_off(sl, pos) + lane] = vT;
  qs[lane] = to_f32(qT);
  vs[lane] = to_f32(vT);
  const float s_cur = wave_sum(to_f32(qT) * to_f32(kT));
  // the block is one wave: its LDS writes are visible to all its lanes once they have
  // completed (no barrier, and no wait for the K/V row stores above)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if constexpr (sizeof(T) == 2 && PIPE) {
    const int kg = lane >> 3, dc = (lane & 7) * 8;
    float m = s_cur, lsum = 0.f, o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.f;
    float qd8[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) qd8[e] = qs[dc + e];
    auto load = [&](auto kc, int p0, Frag<T>(&k)[8], Frag<T>(&v)[8]) {
      if constexpr (decltype(kc)::value) {
        int off[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int pc = min(p0 + kg + 8 * u, plast);
          off[u] = baseB + slot_of[pc] + pc * ROWB + dc * TB;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) frag_load_buf(k[u], rk, off[u]);
#pragma unroll
        for (int u = 0; u < 8; ++u) frag_load_buf(v[u], rv, off[u]);
        return;
      }
      const int pa = min(p0 + lane, plast);
      const int ra = baseB + slot_of[pa] + pa * ROWB;
#pragma unroll
      for (int c = 0; c < 8; ++c) frag_load_buf(k[c], rk, ra + 8 * c * TB);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int pc = min(p0 + kg + 8 * u, plast);
        frag_load_buf(v[u], rv, baseB + slot_of[pc] + pc * ROWB + dc * TB);
      }
    };
    auto pass = [&](auto kc, int p0, const Frag<T>(&k)[8], const Frag<T>(&v)[8]) {
      if constexpr (decltype(kc)::value) {
        kco_pass<T, 8>(qd8, k, v, p0 + kg, pos, m, lsum, o);
        return;
      }
      float sa = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float4_t q0 = *reinterpret_cast<const float4_t*>(&qs[8 * c]);
        const float4_t q1 = *reinterpret_cast<const float4_t*>(&qs[8 * c + 4]);
#pragma unroll
        for (int e = 0; e < 8; ++e) sa += (e < 4 ? q0[e] : q1[e - 4]) * to_f32(k[c].v[e]);
      }
      const bool va = p0 + lane < pos;
      const float mp = wave_max(va ? sa : -INFINITY);
      const float mn = fmaxf(m, mp), scale = __expf(m - mn);
      m = mn;
      const float ea = va ? __expf(sa - m) : 0.f;
      lsum = lsum * scale + wave_sum(ea);
      sc[lane] = ea;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] *= scale;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float pw = sc[kg + 8 * u];  // 0 past the end
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += pw * to_f32(v[u].v[e]);
      }
    };
    // the coalesced-K passes (PIPE 3) from kco_min cached keys on: below that (one pass)
    // the lane-per-key form measured faster (20-window step 3.186 -> 3.198 ms at 12
    // tokens, 3.475 -> 3.448 at 162, profiles/r06/ab_self_attn_kco.txt)
    auto run = [&](auto kc) {
      Frag<T> ka[8], va[8], kb[8], vb[8];
      if (pos > 0) load(kc, 0, ka, va);
      int p0 = 0;
      if constexpr (PIPE == 2) {
        // two passes in flight ahead of the one computed (three register sets, <= 256
        // VGPRs: still two waves per SIMD, every (row, head) wave resident at once); the
        // passes are computed in the same order, so the result is bit-identical to PIPE 1
        Frag<T> kx[8], vx[8];
        if (pos > 64) load(kc, 64, kb, vb);
        for (; p0 + 128 < pos; p0 += 192) {
          load(kc, p0 + 128, kx, vx);
          pass(kc, p0, ka, va);
          if (p0 + 192 < pos) load(kc, p0 + 192, ka, va);
          pass(kc, p0 + 64, kb, vb);
          if (p0 + 256 < pos) load(kc, p0 + 256, kb, vb);
          pass(kc, p0 + 128, kx, vx);
        }
        if (p0 < pos) pass(kc, p0, ka, va);
        if (p0 + 64 < pos) pass(kc, p0 + 64, kb, vb);
      } else {
        for (; p0 + 64 < pos; p0 += 128) {
          load(kc, p0 + 64, kb, vb);
          pass(kc, p0, ka, va);
          if (p0 + 128 < pos) load(kc, p0 + 128, ka, va);
          pass(kc, p0 + 64, kb, vb);
        }
        if (p0 < pos) pass(kc, p0, ka, va);
      }
    };
    if constexpr (PIPE == 3) {
      if (pos > kco_min) run(std::true_type());
      else run(std::false_type());
    } else {
      run(std::false_type());
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = xor8_sum(o[e]);
      o[e] = xor16_sum(o[e]);
      o[e] = xor32_sum(o[e]);
    }
    if (kg == 0) {
      const float e_cur = __expf(s_cur - m), inv = 1.f / (lsum + e_cur);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (o[e] + e_cur * vs[dc + e]) * inv;
      T* op = out + (int64_t)row * ldo + h * 64 + dc;
      store4(op, o[0], o[1], o[2], o[3]);
      store4(op + 4, o[4], o[5], o[6], o[7]);
    }
    CT_END(CT_SELF_ATTN);
    return;
  }
  float qv[64];
#pragma unroll
  for (int c = 0; c < 64; ++c) qv[c] = qs[c];
  if constexpr (sizeof(T) == 2) {
    // passes of 128 cached keys, K and V of the pass in ONE round trip (V's addresses do
    // not depend on the scores), online softmax across passes: K rows lane per key (two
    // keys per lane), V lane = (key group kg, 16 B chunk dc) keys kg, kg+8, .. kg+120
    const int kg = lane >> 3, dc = (lane & 7) * 8;
    float m = s_cur, lsum = 0.f, o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.f;
    for (int p0 = 0; p0 < pos; p0 += 128) {
      const int pa = min(p0 + lane, plast), pb = min(p0 + 64 + lane, plast);
      const int ra = baseB + slot_of[pa] + pa * ROWB, rb = baseB + slot_of[pb] + pb * ROWB;
      Frag<T> ka[8], kb[8], vf[16];
#pragma unroll
      for (int c = 0; c < 8; ++c) frag_load_buf(ka[c], rk, ra + 8 * c * TB);
#pragma unroll
      for (int c = 0; c < 8; ++c) frag_load_buf(kb[c], rk, rb + 8 * c * TB);
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int pc = min(p0 + kg + 8 * u, plast);
        frag_load_buf(vf[u], rv, baseB + slot_of[pc] + pc * ROWB + dc * TB);
      }
      __builtin_amdgcn_sched_barrier(0);  // every load of the pass ahead of the math
      float sa = 0.f, sb = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          sa += qv[8 * c + e] * to_f32(ka[c].v[e]);
          sb += qv[8 * c + e] * to_f32(kb[c].v[e]);
        }
      const bool va = p0 + lane < pos, vb = p0 + 64 + lane < pos;
      const float mp = wave_max(fmaxf(va ? sa : -INFINITY, vb ? sb : -INFINITY));
      const float mn = fmaxf(m, mp), scale = __expf(m - mn);
      m = mn;
      const float ea = va ? __expf(sa - m) : 0.f, eb = vb ? __expf(sb - m) : 0.f;
      lsum = lsum * scale + wave_sum(ea + eb);
      sc[lane] = ea;
      sc[64 + lane] = eb;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] *= scale;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const float pw = sc[kg + 8 * u];  // 0 past the end
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += pw * to_f32(vf[u].v[e]);
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = xor8_sum(o[e]);
      o[e] = xor16_sum(o[e]);
      o[e] = xor32_sum(o[e]);
    }
    if (kg == 0) {
      const float e_cur = __expf(s_cur - m), inv = 1.f / (lsum + e_cur);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (o[e] + e_cur * vs[dc + e]) * inv;
      T* op = out + (int64_t)row * ldo + h * 64 + dc;
      store4(op, o[0], o[1], o[2], o[3]);
      store4(op + 4, o[4], o[5], o[6], o[7]);
    }
    CT_END(CT_SELF_ATTN);
    return;
  }
  // fp32 (parity context): scores of the cached positions p < pos: lane per key, two
  // keys per lane per pass with all 16 row loads in flight (clamped addresses, no branch
  // around a load), then P.V
  float mx = s_cur;
  for (int p0 = 0; p0 < pos; p0 += 128) {
    const int pa = min(p0 + lane, plast), pb = min(p0 + 64 + lane, plast);
    const int ra = baseB + slot_of[pa] + pa * ROWB, rb = baseB + slot_of[pb] + pb * ROWB;
    Frag<T> ka[8], kb[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) frag_load_buf(ka[c], rk, ra + 8 * c * TB);
#pragma unroll
    for (int c = 0; c < 8; ++c) frag_load_buf(kb[c], rk, rb + 8 * c * TB);
    __builtin_amdgcn_sched_barrier(0);  // keep all 16 loads ahead of the math
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sa += qv[8 * c + e] * to_f32(ka[c].v[e]);
        sb += qv[8 * c + e] * to_f32(kb[c].v[e]);
      }
    if (p0 + lane < pos) {
      sc[p0 + lane] = sa;
      mx = fmaxf(mx, sa);
    }
    if (p0 + 64 + lane < pos) {
      sc[p0 + 64 + lane] = sb;
      mx = fmaxf(mx, sb);
    }
  }
  mx = wave_max(mx);
  float sum = 0.f;
  for (int p = lane; p < pos; p += 64) {
    const float e = __expf(sc[p] - mx);
    sc[p] = e;
    sum += e;
  }
  const float e_cur = __expf(s_cur - mx);
  sum = wave_sum(sum) + e_cur;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  // P.V: lane = (key group kg, 16 B chunk dc); keys kg, kg+8, ... accumulated in order,
  // 8 per lane in flight (weight 0 past the end)
  const int kg = lane >> 3, dc = (lane & 7) * 8;
  float o[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = 0.f;
  for (int p0 = kg; p0 < pos; p0 += 64) {
    Frag<T> f[8];
    float pw[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int pc = min(p0 + 8 * u, plast);
      frag_load_buf(f[u], rv, baseB + slot_of[pc] + pc * ROWB + dc * TB);
      pw[u] = p0 + 8 * u < pos ? sc[pc] : 0.f;
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] += pw[u] * to_f32(f[u].v[e]);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    o[e] = xor8_sum(o[e]);
    o[e] = xor16_sum(o[e]);
    o[e] = xor32_sum(o[e]);
  }
  if (kg == 0) {
    const float inv = 1.f / sum;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (o[e] + e_cur * vs[dc + e]) * inv;
    T* op = out + (int64_t)row * ldo + h * 64 + dc;
    store4(op, o[0], o[1], o[2], o[3]);
    store4(op + 4, o[4], o[5], o[6], o[7]);
  }
  CT_END(CT_SELF_ATTN);
}

// Grouped form (fp16, a window's G <= 8 beams as the G waves of one workgroup per
// (window, head)).  Per wave the arithmetic is k_self_attn_qkv's fp16 path operation for
// operation (same passes of 128 keys, same lane roles and orders: bit-identical outputs);
// only where the cached K / V rows come from changes.  Beam histories form a tree: beam b
// names beam 0's (slot, position) rows exactly on [0, d_b), d_b = the first position where
// their ancestries differ, and never again after it.  So each pass stages beam 0's 128 K
// and V rows in LDS once (global_load_lds, 32 KB shared by the G waves) and a lane reads a
// key from LDS below its beam's d_b and from HBM at or above it (profiles/ancestry_probe.py:
// at 20 windows the beams share 37-97 % of their context, 1.1-2.4 distinct rows per
// position, where every wave streamed its own rows).  K rows are stored with their 16 B
// chunks XOR-swizzled by (row >> 1) & 7, so lane-per-row reads of a chunk are conflict-free.
WH_DEV void sa_glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src),
                                   (__attribute__((address_space(3))) void*)(lds), 16, 0, 0);
}

constexpr int SA_GMAX = 8;
// PK keys per pass: 128 (k_self_attn_qkv's passes, bit-identical) or 64 (half the register
// buffers: at <= 168 VGPRs two 5-wave workgroups share a CU, so the 400 (window, head)
// workgroups of 20 windows run in one round; its own passes, so its own bits)
template <typename T, int PK>
__global__ __launch_bounds__(64 * SA_GMAX) void k_self_attn_grp(const float* __restrict__ part, int nsplit,
                                                                 int64_t part_stride, const float* __restrict__ bqkv,
                                                                 int ns, T* __restrict__ kc, T* __restrict__ vc,
                                                                 const int* __restrict__ row_pos,
                                                                 const int* __restrict__ anc, int G, int nbeam, int H,
                                                                 int ctx, T* __restrict__ out, int ldo) {
  static_assert(sizeof(T) == 2, "fp16 path");
  static_assert(PK == 128 || PK == 64, "keys per pass");
  constexpr int NKI = PK / 8;  // glds instructions of 8 rows per K (and per V) stage
  constexpr int VU = PK / 8;   // V rows per lane per pass
  __shared__ __attribute__((aligned(1024))) T kref[PK * 64];
  __shared__ __attribute__((aligned(1024))) T vref[PK * 64];
  __shared__ int slot_of[SA_GMAX][512];
  __shared__ __attribute__((aligned(16))) float qs[SA_GMAX][64], vs[SA_GMAX][64], sc[SA_GMAX][PK];
  const int lane = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int h = blockIdx.x % H, w = blockIdx.x / H, row = w * G + sl;
  const int* an = anc + ((int64_t)w * G + sl) * ctx;
  const int64_t head_stride = (int64_t)ctx * 64;
  const int64_t wbase = (int64_t)w * nbeam;
  auto kv_off = [&](int slot, int p) -> int64_t { return ((wbase + slot) * H + h) * head_stride + (int64_t)p * 64; };
  // the prologue of k_self_attn_qkv (one round trip: position, ancestry, q/k/v slabs)
  const int pos = row_pos[row];
  int sv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) sv[i] = an[min(lane + 64 * i, ctx - 1)];
  float qd, kd, vd;
  {
    const float* pr = part + (int64_t)row * 3 * ns + h * 64 + lane;
    float a0[16], a1[16], a2[16];
#pragma unroll
    for (int z = 0; z < 16; ++z)
      if (z < nsplit) {
        a0[z] = pr[z * part_stride];
        a1[z] = pr[z * part_stride + ns];
        a2[z] = pr[z * part_stride + 2 * ns];
      }
    qd = bqkv[h * 64 + lane];
    kd = bqkv[ns + h * 64 + lane];
    vd = bqkv[2 * ns + h * 64 + lane];
#pragma unroll
    for (int z = 0; z < 16; ++z)
      if (z < nsplit) {
        qd += a0[z];
        kd += a1[z];
        vd += a2[z];
      }
  }
  for (int i = 0; i < 8; ++i)
    if (lane + 64 * i < pos) slot_of[sl][lane + 64 * i] = sv[i];
  const int plast = max(pos - 1, 0);
  const T qT = from_f32<T>(qd), kT = from_f32<T>(kd), vT = from_f32<T>(vd);
  kc[kv_off(sl, pos) + lane] = kT;
  vc[kv_off(sl, pos) + lane] = vT;
  qs[sl][lane] = to_f32(qT);
  vs[sl][lane] = to_f32(vT);
  const float s_cur = wave_sum(to_f32(qT) * to_f32(kT));
  __syncthreads();  // every beam's ancestry in LDS
  // d: the first position where this beam's ancestry leaves beam 0's
  int d = pos;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int p = lane + 64 * i;
    if (p < pos && slot_of[sl][p] != slot_of[0][p]) d = min(d, p);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) d = min(d, __shfl_xor(d, o, 64));
  // q stays in LDS (broadcast reads in the dot products: 64 VGPRs fewer than a register copy)
  const int kg = lane >> 3, dc = (lane & 7) * 8;
  float m = s_cur, lsum = 0.f, o[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = 0.f;
  for (int p0 = 0; p0 < pos; p0 += PK) {
    // beam 0's rows p0 .. p0 + PK - 1 (< pos) -> LDS: PK / 8 K and PK / 8 V instructions of
    // 8 rows, dealt over the G waves; lane (row r0 + lane / 8, chunk lane % 8)
    for (int i = sl; i < 2 * NKI; i += G) {
      const int r0 = (i % NKI) * 8, r = r0 + (lane >> 3), p = p0 + r;
      if (p <= plast) {
        const int pc = lane & 7;
        if (i < NKI) {  // K: physical chunk pc holds logical chunk pc ^ ((r >> 1) & 7)
          sa_glds16(kc + kv_off(slot_of[0][p], p) + 8 * (pc ^ ((r >> 1) & 7)), kref + r0 * 64);
        } else {
          sa_glds16(vc + kv_off(slot_of[0][p], p) + 8 * pc, vref + r0 * 64);
        }
      }
    }
    // this beam's own rows at or past d, straight from HBM into registers
    const int pa = min(p0 + lane, plast), pb = min(p0 + 64 + lane, plast);
    const bool la = pa < d, lb = pb < d;
    Frag<T> ka[8], kb[PK == 128 ? 8 : 1], vf[VU];
    if (!la) {
      const T* ra = kc + kv_off(slot_of[sl][pa], pa);
#pragma unroll
      for (int c = 0; c < 8; ++c) frag_load(ka[c], ra + 8 * c);
    }
    if constexpr (PK == 128) {
      if (!lb) {
        const T* rb = kc + kv_off(slot_of[sl][pb], pb);
#pragma unroll
        for (int c = 0; c < 8; ++c) frag_load(kb[c], rb + 8 * c);
      }
    }
#pragma unroll
    for (int u = 0; u < VU; ++u) {
      const int pc = min(p0 + kg + 8 * u, plast);
      if (pc >= d) frag_load(vf[u], vc + kv_off(slot_of[sl][pc], pc) + dc);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // the staged rows of every wave
    if (la) {
      const int r = pa - p0, sw = (r >> 1) & 7;
#pragma unroll
      for (int c = 0; c < 8; ++c) ka[c].v = *reinterpret_cast<const half8_t*>(kref + r * 64 + 8 * (c ^ sw));
    }
    if constexpr (PK == 128) {
      if (lb) {
        const int r = pb - p0, sw = (r >> 1) & 7;
#pragma unroll
        for (int c = 0; c < 8; ++c) kb[c].v = *reinterpret_cast<const half8_t*>(kref + r * 64 + 8 * (c ^ sw));
      }
    }
#pragma unroll
    for (int u = 0; u < VU; ++u) {
      const int pc = min(p0 + kg + 8 * u, plast);
      if (pc < d) vf[u].v = *reinterpret_cast<const half8_t*>(vref + (pc - p0) * 64 + dc);
    }
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const float4_t q0 = *reinterpret_cast<const float4_t*>(&qs[sl][8 * c]);
      const float4_t q1 = *reinterpret_cast<const float4_t*>(&qs[sl][8 * c + 4]);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float qe = e < 4 ? q0[e] : q1[e - 4];
        sa += qe * to_f32(ka[c].v[e]);
        if constexpr (PK == 128) sb += qe * to_f32(kb[c].v[e]);
      }
    }
    const bool va = p0 + lane < pos, vb = PK == 128 && p0 + 64 + lane < pos;
    const float mp = wave_max(fmaxf(va ? sa : -INFINITY, vb ? sb : -INFINITY));
    const float mn = fmaxf(m, mp), scale = __expf(m - mn);
    m = mn;
    const float ea = va ? __expf(sa - m) : 0.f, eb = vb ? __expf(sb - m) : 0.f;
    lsum = lsum * scale + wave_sum(ea + eb);
    sc[sl][lane] = ea;
    if constexpr (PK == 128) sc[sl][64 + lane] = eb;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] *= scale;
#pragma unroll
    for (int u = 0; u < VU; ++u) {
      const float pw = sc[sl][kg + 8 * u];  // 0 past the end
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] += pw * to_f32(vf[u].v[e]);
    }
    __syncthreads();  // the staged rows are read: the next pass may overwrite them
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    o[e] = xor8_sum(o[e]);
    o[e] = xor16_sum(o[e]);
    o[e] = xor32_sum(o[e]);
  }
  if (kg == 0) {
    const float e_cur = __expf(s_cur - m), inv = 1.f / (lsum + e_cur);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (o[e] + e_cur * vs[sl][dc + e]) * inv;
    T* op = out + (int64_t)row * ldo + h * 64 + dc;
    store4(op, o[0], o[1], o[2], o[3]);
    store4(op + 4, o[4], o[5], o[6], o[7]);
  }
}

// the self-attention form launch_self_attn_qkv picks (also what wh_step_kernels reports):
// the grouped form only in the tuning build with WHISPER_HIP_SA_GRP set; the pipelined
// 64-key passes unless WHISPER_HIP_SA_PIPE=0 (tuning build)
int self_attn_grp_mode() {
  static const int grp = [] {
    const char* e = tune_env("WHISPER_HIP_SA_GRP");
    return e ? atoi(e) : 0;
  }();
  return grp;
}
// the coalesced-K passes (PIPE 3) of the fp16-slab step form; WHISPER_HIP_SA_KCO=0 in the
// tuning build: the lane-per-key K loads (PIPE 1)
bool self_attn_kco_on() {
  static const bool on = [] {
    const char* e = tune_env("WHISPER_HIP_SA_KCO");
    return !(e && e[0] == '0');
  }();
  return on;
}
// the cached-key count from which the coalesced-K passes run (tuning WHISPER_HIP_SA_KCO_MIN)
int self_attn_kco_min() {
  static const int v = [] {
    const char* e = tune_env("WHISPER_HIP_SA_KCO_MIN");
    return e ? atoi(e) : 64;
  }();
  return v;
}
bool self_attn_pipe_on() {
  static const bool pipe = [] {
    const char* e = tune_env("WHISPER_HIP_SA_PIPE");
    return !(e && e[0] == '0');
  }();
  return pipe;
}


template <typename T>
int launch_self_attn_qkv(const float* part, int nsplit, int64_t part_stride, const float* bqkv, int ns, T* kc, T* vc,
                          const int* rw, const int* rs, const int* rp, const int* anc, int anc_beams, int nbeam, int H,
                          int ctx, T* out, int ldo, int rows, hipStream_t st, int slab_half) {
  if (rows <= 0) return 0;
  // the kernel takes window and beam from the row index: step rows are w * G + beam
  // fp16 slabs: the pipelined fp16 form only (round 4 measured an fp16-slab form of the
  // 128-key kernel 8.7 -> 13.9 us per launch)
  if (anc_beams < 1 || rows % anc_beams || nsplit > 16) return -1;
  if (slab_half) {
    if constexpr (sizeof(T) == 2) {
      if (self_attn_pipe_on() && !self_attn_grp_mode()) {
        if (self_attn_kco_on()) {
          k_self_attn_qkv<T, 3, half_t><<<rows * H, 64, 0, st>>>(reinterpret_cast<const half_t*>(part), nsplit,
                                                                part_stride, bqkv, ns, kc, vc, rw, rs, rp, anc,
                                                                anc_beams, nbeam, H, ctx, out, ldo,
                                                                self_attn_kco_min()), wh_launched("k_self_attn_qkv");
          return 0;
        }
        k_self_attn_qkv<T, 1, half_t><<<rows * H, 64, 0, st>>>(reinterpret_cast<const half_t*>(part), nsplit,
                                                              part_stride, bqkv, ns, kc, vc, rw, rs, rp, anc,
                                                              anc_beams, nbeam, H, ctx, out, ldo), wh_launched("k_self_attn_qkv");
        return 0;
      }
    }
    return -1;
  }
  // fp16 beams, tuning build only (WHISPER_HIP_SA_GRP=1): the grouped form, same arithmetic
  // per row.  Measured slower at every context length (20 windows: step 3.456 -> 3.655 ms
  // at 12 tokens, 3.834 -> 4.114 at 220, profiles/r04/self_attn_grp_ab.txt): at 238 VGPRs a
  // CU holds one 5-wave workgroup, so the 400 (window, head) workgroups run in two rounds.
  // WHISPER_HIP_SA_GRP=2: 64-key passes, 132 VGPRs, one round — slower still (3.423 -> 3.523
  // ms at 12 tokens, 3.819 -> 4.145 at 220, profiles/r04/self_attn_grp64_ab.txt): the
  // growth with the context is the passes' round trips, not the bytes the beams share
  const int grp = self_attn_grp_mode();
  if constexpr (sizeof(T) == 2) {
    if (grp && anc_beams >= 2 && anc_beams <= SA_GMAX && ctx <= 512) {
      if (grp == 2)
        k_self_attn_grp<T, 64><<<(rows / anc_beams) * H, 64 * anc_beams, 0, st>>>(
            part, nsplit, part_stride, bqkv, ns, kc, vc, rp, anc, anc_beams, nbeam, H, ctx, out, ldo), wh_launched("k_self_attn_grp");
      else
        k_self_attn_grp<T, 128><<<(rows / anc_beams) * H, 64 * anc_beams, 0, st>>>(
            part, nsplit, part_stride, bqkv, ns, kc, vc, rp, anc, anc_beams, nbeam, H, ctx, out, ldo), wh_launched("k_self_attn_grp");
      return 0;
    }
  }
  // fp16: the pipelined 64-key passes (WHISPER_HIP_SA_PIPE=0 in the tuning build: the
  // 128-key passes): 20-window step 3.419 -> 3.363 ms at 12 tokens, 3.810 -> 3.756 at 220,
  // config 3 675.6 -> 684.6 xRT (profiles/r04/self_attn_pipe_ab.txt)
  const bool pipe = self_attn_pipe_on();
  if constexpr (sizeof(T) == 2) {
    if (pipe) {
      // WHISPER_HIP_SA_DEPTH=2 (tuning): two passes in flight ahead (A/B)
      static const int depth = [] {
        const char* e = tune_env("WHISPER_HIP_SA_DEPTH");
        return e && e[0] == '2' ? 2 : 1;
      }();
      if (self_attn_kco_on())
        k_self_attn_qkv<T, 3><<<rows * H, 64, 0, st>>>(part, nsplit, part_stride, bqkv, ns, kc, vc, rw, rs, rp, anc,
                                                      anc_beams, nbeam, H, ctx, out, ldo, self_attn_kco_min()),
            wh_launched("k_self_attn_qkv");
      else if (depth == 2)
        k_self_attn_qkv<T, 2><<<rows * H, 64, 0, st>>>(part, nsplit, part_stride, bqkv, ns, kc, vc, rw, rs, rp, anc,
                                                      anc_beams, nbeam, H, ctx, out, ldo), wh_launched("k_self_attn_qkv");
      else
        k_self_attn_qkv<T, 1><<<rows * H, 64, 0, st>>>(part, nsplit, part_stride, bqkv, ns, kc, vc, rw, rs, rp, anc,
                                                      anc_beams, nbeam, H, ctx, out, ldo), wh_launched("k_self_attn_qkv");
      return 0;
    }
  }
  k_self_attn_qkv<T><<<rows * H, 64, 0, st>>>(part, nsplit, part_stride, bqkv, ns, kc, vc, rw, rs, rp, anc, anc_beams,
                                             nbeam, H, ctx, out, ldo), wh_launched("k_self_attn_qkv");
  return 0;
}

// out[m][n] = act(bias[n] + sum_z part[z][m][n]) as T (split-K epilogue of the
// non-residual decoder GEMVs: cross-attention query, MLP fc1 + GELU)
template <typename T, int ACT, typename S = float>
__global__ __launch_bounds__(256) void k_reduce_store(const S* __restrict__ part, int nsplit, int64_t part_stride,
                                                      const float* __restrict__ bias, T* __restrict__ out, int ldo, int M,
                                                      int N) {
  // 32-bit index arithmetic (M x N < 2^31, launch_reduce_store): the int64 divide was
  // ~150 vector instructions ahead of the first slab load
  const int i = (int)(blockIdx.x * 256 + threadIdx.x) * 4;
  CT_MARK(CT_REDUCE, 0);
  if (i >= M * N) return;
  const int m = (int)((unsigned)i / (unsigned)N), n = i - m * N;
  typedef typename std::conditional<sizeof(S) == 2, half4_t, float4_t>::type R4;  // raw slab elements
  R4 pp[16];
#pragma unroll
  for (int z = 0; z < 16; ++z)
    if (z < nsplit) pp[z] = *reinterpret_cast<const R4*>(part + z * part_stride + i);
  float4_t v = bias ? load4f(bias + n) : (float4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int z = 0; z < 16; ++z)
    if (z < nsplit) v += (float4_t){(float)pp[z][0], (float)pp[z][1], (float)pp[z][2], (float)pp[z][3]};
  if (ACT) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = gelu_f(v[j]);
  }
  store4(out + (int64_t)m * ldo + n, v[0], v[1], v[2], v[3]);
  CT_END(CT_REDUCE);
}

template <typename T>
void launch_reduce_store(const float* part, int nsplit, int64_t part_stride, const float* bias, T* out, int ldo, int M,
                         int N, int gelu, hipStream_t st, int slab_half) {
  if (M <= 0) return;
  if ((int64_t)M * N >= (int64_t)1 << 31) {
    wh_set_launch_error("launch_reduce_store: M x N >= 2^31");
    return;
  }
  const int64_t tot = (int64_t)M * N / 4;
  const unsigned nb = (unsigned)((tot + 255) / 256);
  if (slab_half) {
    const half_t* ph = reinterpret_cast<const half_t*>(part);
    if (gelu) k_reduce_store<T, 1, half_t><<<nb, 256, 0, st>>>(ph, nsplit, part_stride, bias, out, ldo, M, N), wh_launched("k_reduce_store");
    else k_reduce_store<T, 0, half_t><<<nb, 256, 0, st>>>(ph, nsplit, part_stride, bias, out, ldo, M, N), wh_launched("k_reduce_store");
    return;
  }
  if (gelu) k_reduce_store<T, 1><<<nb, 256, 0, st>>>(part, nsplit, part_stride, bias, out, ldo, M, N), wh_launched("k_reduce_store");
  else k_reduce_store<T, 0><<<nb, 256, 0, st>>>(part, nsplit, part_stride, bias, out, ldo, M, N), wh_launched("k_reduce_store");
}

// ============================================================ decoder cross-attention (split-K flash decoding)
// grid (windows, H, nsplit), block 64*NW = NW waves; wave w of split sp owns the 64-key
// tile sp*NW + w.  All rows of a window (its beams, or the prefill tokens) share the
// pass, in row tiles of 16: K and V of a window are streamed from HBM once per step.
// Both MFMA operands load straight from HBM into fragments: K in its natural
// [key][64] layout (A of S^T = K Q^T), V stored transposed [64][Tk] at encode time
// (A of O^T = V^T P^T), so no LDS staging is needed; LDS only combines the NW waves.
// ck: [win][head][TKP][64], cvt: [win][head] tile-major V^T (xv_index, wh_kernels.h) for this layer.
// Partials per split: po[row][h][split][64], pm/pl[row][h][split] (k_cross_combine).
// If qk_map != null the raw scores q.k of alignment heads are also written
// (word timestamps, decoder.py:306-308): qk_out[(qk_map[h] * qk_rows + row) * Tk + key].
template <typename T, int NW, int QZ>
__global__ __launch_bounds__(64 * NW) void k_cross_attn(const T* __restrict__ q, int ldq, const T* ck,
                                                    const T* cvt, int Tk, int H, int nsplit,
                                                    const int* __restrict__ win_row0, const int* __restrict__ win_nrows,
                                                    const int* __restrict__ win_slot, int64_t win_stride,
                                                    float* __restrict__ po, float* __restrict__ pm, float* __restrict__ pl,
                                                    float* qk_out, const int* qk_map, int qk_rows, XQPart xq) {
  __shared__ float red_m[NW][16], red_l[NW][16];
  __shared__ float red_o[NW][64][17];
  constexpr bool QP = QZ > 0;
  __shared__ __attribute__((aligned(16))) T qs[QP ? 32 : 1][72];  // rows 16..31: waves 4..7's dummy copies
  const int wi = blockIdx.x, h = blockIdx.y, sp = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int row0 = win_row0[wi], nrows = win_nrows[wi];
  const int kt0 = (sp * NW + wave) * 64;
  const bool active = kt0 < Tk;
  const int qslot = qk_map ? qk_map[h] : -1;
  const T* kbase = ck + (int64_t)win_slot[wi] * win_stride + (int64_t)h * TKP * 64;
  const T* vbase = cvt + (int64_t)win_slot[wi] * win_stride + (int64_t)h * 64 * TKP;
  constexpr float LOG2E = 1.4426950408889634f;
  // K and V fragments of this wave's tile do not depend on the rows: load them once,
  // all in flight together (V^T is key-permuted so each lane's 8 keys are contiguous).
  // QP (decoder step, <= 16 rows per window): q = bias + sum of the projection's
  // split-K slabs (k_reduce_store's order), reduced here into LDS instead of by a
  // separate launch; its loads go between K's and V's, so the wait for them leaves
  // V in flight (the first MFMAs need K and q, not V)
  // (no branch around any of these loads: a branch makes the compiler's wait for q
  // a full drain; an inactive wave loads tile 0 and skips its MFMAs)
  const int ktl = active ? kt0 : 0;
  Frag<T> kf[4][2], vf[4][2];
#pragma unroll
  for (int kt = 0; kt < 4; ++kt) {
    const T* kp = kbase + (int64_t)(ktl + kt * 16 + r) * 64 + 8 * g;
    frag_load(kf[kt][0], kp);
    frag_load(kf[kt][1], kp + 32);
  }
  float4_t qv = (float4_t){0.f, 0.f, 0.f, 0.f}, pp[QP ? QZ : 1];
  __builtin_amdgcn_sched_barrier(0);  // keep the load groups in K, q, V order
  if constexpr (QP) {
    // waves 4..7 repeat waves 0..3's loads (L1 hits) to stay branch-free; the slab
    // count is a template constant so no load is sunk into a conditional
    const int t = tid & 255, qq = min(t >> 4, nrows - 1), c = h * 64 + (t & 15) * 4;
    const float* src = xq.part + (int64_t)(row0 + qq) * ldq + c;
#pragma unroll
    for (int z = 0; z < QZ; ++z) pp[z] = load4f(src + z * xq.stride);
    qv = load4f(xq.bias + c);
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int s = 0; s < 2; ++s) frag_load(vf[dt][s], vbase + ((int64_t)(ktl >> 6) * 64 + dt * 16 + r) * 64 + 32 * s + 8 * g);
  if constexpr (QP) {
#pragma unroll
    for (int z = 0; z < QZ; ++z) qv += pp[z];
    store4(&qs[tid >> 4][(tid & 15) * 4], qv[0], qv[1], qv[2], qv[3]);  // unconditional: no load is sunk
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // LDS only: V stays in flight
  }
  for (int rt = 0; rt < nrows; rt += 16) {
    int qr = rt + r;
    const bool qvalid = qr < nrows;
    if (!qvalid) qr = nrows - 1;
    float m = -INFINITY, l = 0.f;
    float4_t acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = (float4_t){0.f, 0.f, 0.f, 0.f};
    if (active) {
      Frag<T> qf[2];
      if constexpr (QP) {
        frag_load(qf[0], &qs[qr][8 * g]);
        frag_load(qf[1], &qs[qr][32 + 8 * g]);
      } else {
        const T* qp = q + (int64_t)(row0 + qr) * ldq + h * 64 + 8 * g;
        frag_load(qf[0], qp);
        frag_load(qf[1], qp + 32);
      }
      float4_t sc[4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        sc[kt] = (float4_t){0.f, 0.f, 0.f, 0.f};
        mfma_step(sc[kt], kf[kt][0], qf[0]);
        mfma_step(sc[kt], kf[kt][1], qf[1]);
      }
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int key = kt0 + kt * 16 + 4 * g + j;
          if (key >= Tk) sc[kt][j] = -INFINITY;
          else if (qslot >= 0 && qvalid) qk_out[((int64_t)qslot * qk_rows + row0 + qr) * Tk + key] = sc[kt][j];
          mx = fmaxf(mx, sc[kt][j]);
        }
      mx = xor16_max(mx);
      mx = xor32_max(mx);
      m = mx;
      Frag<T> pf[2];
      float ps = 0.f;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float p = hw_exp2((sc[kt][j] - m) * LOG2E);
          ps += p;
          pf[kt >> 1].v[(kt & 1) * 4 + j] = from_f32<T>(p);
        }
      ps = xor16_sum(ps);
      ps = xor32_sum(ps);
      l = ps;
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) mfma_step(acc[dt], vf[dt][s], pf[s]);
    }
    // combine the NW waves of this split (lanes of every g hold the row stats of q = r)
    if (g == 0) {
      red_m[wave][r] = m;
      red_l[wave][r] = l;
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int j = 0; j < 4; ++j) red_o[wave][dt * 16 + 4 * g + j][r] = acc[dt][j];
    __syncthreads();
    if (tid < 256) {
      const int qq = tid >> 4, dc = (tid & 15) * 4;  // 16 rows x 16 chunks of 4 dims
      float M = -INFINITY;
#pragma unroll
      for (int w = 0; w < NW; ++w) M = fmaxf(M, red_m[w][qq]);
      float f[NW], L = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        f[w] = red_m[w][qq] == -INFINITY ? 0.f : hw_exp2((red_m[w][qq] - M) * LOG2E);
        L += f[w] * red_l[w][qq];
      }
      const int row = rt + qq;
      if (row < nrows) {
        const int64_t pi = ((int64_t)(row0 + row) * H + h) * nsplit + sp;
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o[e] = 0.f;
#pragma unroll
          for (int w = 0; w < NW; ++w) o[e] += f[w] * red_o[w][dc + e][qq];
        }
        store4(po + pi * 64 + dc, o[0], o[1], o[2], o[3]);
        if (dc == 0) {
          pm[pi] = M;
          pl[pi] = L;
        }
      }
    }
    __syncthreads();
  }
}

template <typename T>
__global__ __launch_bounds__(64) void k_cross_combine(const float* __restrict__ po, const float* __restrict__ pm,
                                                      const float* __restrict__ pl, int H, int nsplit,
                                                      T* __restrict__ out, int ldo) {
  const int row = blockIdx.x, h = blockIdx.y, lane = threadIdx.x;
  const int64_t b = ((int64_t)row * H + h) * nsplit;
  float M = -INFINITY;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, pm[b + s]);
  float num = 0.f, den = 0.f;
  for (int s = 0; s < nsplit; ++s) {
    const float f = __expf(pm[b + s] - M);
    num += f * po[(b + s) * 64 + lane];
    den += f * pl[b + s];
  }
  out[(int64_t)row * ldo + h * 64 + lane] = from_f32<T>(num / den);
}

// ------------------------------------------------------------ step cross-attention
// Decoder-step cross-attention (decoder.py:74-91 for the step's query rows: <= 16 rows
// per window, the beams), batch-invariant and balanced over the chip.
//
// Numerics are fixed per (window, head) pair, whatever the batch: every 64-key tile of
// the pair gives one softmax partial (m = the tile's max score, l = sum exp(s - m),
// O = sum exp(s - m) v), and the pair's nsp = ceil(Tk / 64) partials are merged in tile
// order by the flat merge of xs_merge (M = max m, then L and O accumulated over the
// tiles in order).  How many windows share the launch changes only which workgroup
// computes a tile and where the pair is merged, never an arithmetic operation, so a
// window's output is bit-identical in any batch.
//
// Work distribution (speed only): the tiles of all pairs, in (pair, tile) order, are
// dealt in contiguous ranges to nwg <= 256 workgroups; the workgroup's 8 waves take its
// tiles round-robin, the next tile's K and V in flight while one is computed (no tile
// depends on another, the last one is peeled: no load is clamped or wasted).  A pair
// whose tiles are all in the workgroup merges from LDS.  A pair cut between workgroups
// has this workgroup's partials stored write-through (sc1) at [pair][tile] (the window's
// rows only), drained by every storing wave, and counted on the pair's arrival counter
// (relaxed agent atomic, + the tiles contributed); the workgroup that completes the
// count re-arms it and merges every partial with sc1 loads (cdna_hip_programming.md §6
// Guideline 16 R1, MI355X_MICROARCH.md "Valid forms").  RR: rows kept per partial in LDS
// (8 when the beams are <= 8, else 16).
// K: [slot][head][TKP][64]; V transposed, tile-major (xv_index: a 64-key tile's 64 x 64
// V^T is 8 KB contiguous, keys permuted within 32-key groups), so both MFMA operands load
// straight from HBM into fragments and each tile is two contiguous 8 KB streams.
constexpr float XS_LOG2E = 1.4426950408889634f;

template <int RR>
struct XsShape {
  static constexpr int SMAX = RR == 8 ? 48 : 32;  // tiles per workgroup (LDS partials)
};

// the pair merge shared by the LDS and the record path: `get(k, m, l, o)` fetches tile
// k's partial; every fetch is issued before the first use (one round trip on the record
// path), then M = max m, and L, O accumulate over the tiles in order
template <typename Get>
WH_DEV float4_t xs_merge(int n, Get get) {
  float mv[XS_NSP], lv[XS_NSP];
  float4_t ov[XS_NSP];
#pragma unroll
  for (int k = 0; k < XS_NSP; ++k) get(k < n ? k : n - 1, mv[k], lv[k], ov[k]);
  float M = -INFINITY;
#pragma unroll
  for (int k = 0; k < XS_NSP; ++k)
    if (k < n) M = fmaxf(M, mv[k]);
  float L = 0.f;
  float4_t acc = (float4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < XS_NSP; ++k)
    if (k < n) {
      const float f = mv[k] == -INFINITY ? 0.f : hw_exp2((mv[k] - M) * XS_LOG2E);
      L = __builtin_fmaf(f, lv[k], L);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] = __builtin_fmaf(f, ov[k][e], acc[e]);
    }
  const float inv = 1.f / L;
  return acc * inv;
}

#if WH_TUNING
// tuning build: per-workgroup wall-clock marks (s_memrealtime, 100 MHz) of the last
// k_xattn_seg launch, read by wh_tune_xs_trace (profiles/xattn_trace.py)
constexpr int XS_MARKS = 10;
__device__ unsigned long long g_xs_trace[256][XS_MARKS];
#define XS_MARK(k)                                                                         \
  do {                                                                                     \
    if (threadIdx.x == 0) g_xs_trace[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();   \
  } while (0)
#else
#define XS_MARK(k) \
  do {             \
  } while (0)
#endif

// Round 6: the decoder step's cross-attention query projected inside k_xattn_seg (QK > 0)
// instead of by a split-K k_proj launch whose fp16 slabs the kernel summed: the range's
// pairs (at most XS_QF: a range holds <= 2 x nsp tiles with nsp = 24) each need
//   q[row][c] = (S0 + S1) + bias[c],  S_kh = sum over the K half kh of X[row][k] W_q[c][k]
// (MFMA accumulation in k-step order; the two halves meet in LDS in that order), the
// same arithmetic whichever workgroup, grid form or batch computes it (batch invariance).
// The 8 waves are (16-column tile c of the head's 64, K half kh); a pair's window rows
// (<= RR) are staged in LDS (rows past the window are never emitted), the wave's
// 16 x n / 2 slice of W_q (QK fragments) is loaded once per head.  X, the K-half sums and
// the biases live in the tile partials' LDS (dead until the first tile).  Reference:
// decoder.py:73-91 (cross-attention query), :42 (the 0.125 query scale, folded in W_q).
//
// Load order variants (QV; the arithmetic is the same in all three):
//  0: X (registers), bias, W_q, then the first tile's K / V; the second tile is loaded by the
//     tile loop.  Traced at 20 windows (profiles/r06/xattn_trace_qv.txt): X staged at 8.8 us
//     — the X and bias requests queue behind every CU's W_q and first-tile K / V (63 MB asked
//     for at once), so the query was staged at 10.5 us against 4.4 with the slabs.
//  1: X and biases by LDS-DMA (no VGPRs), the first two tiles' K / V with W_q.  hipcc puts a
//     vmcnt(0) ahead of the first LDS read after an LDS-DMA (it cannot tell the DMA's slot
//     in the count), so the projection waits for both tiles as well.
//  2: X and bias (registers) and W_q first; the two tiles' K / V are issued only once X is
//     staged, so the few KB the projection waits on are not queued behind 25 MB of K / V;
//     the tiles then stream while W_q lands and the projection runs.
//  4: variant 2 with the W_q fragments issued first, ahead of the window-row metadata round
//     trip (their addresses need only the pair's head); 5: variant 4 with the two tiles'
//     K / V issued only after the projection's MFMAs (nothing competes with W_q and X).
//  3: variant 2 for the single-window step (k_proj1 layers, no k_resid_ln): X is the fp32
//     residual rows and each workgroup computes their LayerNorm (k_proj1's arithmetic: one
//     wave per row, two register passes) into the staged fp16 rows; the grid gives every
//     workgroup tiles of ONE pair (launch_cross_attn).
constexpr int XS_QF = 3;
template <typename T, int QK, int RR, int QV, typename PairWH, typename LoadKV>
WH_DEV void xq_project(const XQPart& xq, int pa, int plast, int cnt, const int* __restrict__ win_row0,
                       const int* __restrict__ win_nrows, PairWH pair_wh, LoadKV load_kv, Frag<T> (&kA)[4][2],
                       Frag<T> (&vA)[4][2], Frag<T> (&kB)[4][2], Frag<T> (&vB)[4][2], char* xst, T (*qs)[16][72],
                       int* s_wnr, int* s_wr0) {
  static_assert(sizeof(T) == 2, "fused query projection: fp16 contexts");
  constexpr int N = QK * 64;                           // model width = K
  constexpr int CPR = N * (int)sizeof(T) / 16;         // 16-B chunks per row
  constexpr bool DMA = QV == 1;                        // X / bias by LDS-DMA
  constexpr int XROWB = DMA ? N * (int)sizeof(T) : N * (int)sizeof(T) + 16;  // LDS row (bytes)
  constexpr int XPT = (RR * CPR + 511) / 512;          // chunks per thread per pair
  static_assert(!DMA || (RR * CPR) % 64 == 0, "whole 1 KB LDS-DMA blocks per pair");
  static_assert(!DMA || CPR % 8 == 0, "the row swizzle stays inside the row");
  // LDS (byte offsets in xst): X rows, the K-half sums [2][XS_QF][4][64] float4, the biases
  constexpr int RED_OFF = XS_QF * RR * XROWB, BIAS_OFF = RED_OFF + 2 * XS_QF * 4 * 64 * 16;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const int c = wave & 3, kh = wave >> 2;
  const int np = plast - pa + 1;
  // the pairs' heads (arithmetic only) and window rows (scalar loads, one round trip)
  int q_h[XS_QF], q_w[XS_QF], q_nr[XS_QF], q_r0[XS_QF];
#pragma unroll
  for (int j = 0; j < XS_QF; ++j) {
    const int pj = __builtin_amdgcn_readfirstlane(min(pa + j, plast));
    pair_wh(pj, q_w[j], q_h[j]);
  }
  // QV 4 / 5: the wave's W_q fragments leave first, ahead of the metadata round trip
  constexpr bool W_FIRST = QV >= 4;
  Frag<T> wf[QK];
  auto load_w = [&](int h) {
    if (xq.qwf) {  // fragment order (launch_wq_frag): each k-step one 1 KB contiguous wave load
      const T* wp = reinterpret_cast<const T*>(xq.qwf) + ((int64_t)((h * 4 + c) * 2 + kh) * QK * 64 + lane) * 8;
#pragma unroll
      for (int s = 0; s < QK; ++s) frag_load_stream(wf[s], wp + s * 512);
    } else {
      const T* wp = reinterpret_cast<const T*>(xq.qw) + (int64_t)(h * 64 + c * 16 + r) * N + kh * QK * 32 + 8 * g;
#pragma unroll
      for (int s = 0; s < QK; ++s) frag_load_stream(wf[s], wp + s * 32);
    }
  };
  if constexpr (W_FIRST) {
    load_w(q_h[0]);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int j = 0; j < XS_QF; ++j) {
    q_nr[j] = win_nrows[q_w[j]];
    q_r0[j] = win_row0[q_w[j]];
  }
  // 1. each pair's window rows and head biases
  constexpr bool LN = QV == 3;
  constexpr int CPL = N / 256;  // (LN) float4 chunks of a fp32 row per lane
  float4_t xv[DMA ? 1 : XS_QF][DMA ? 1 : XPT];
  float bv[DMA ? 1 : XS_QF];
  float4_t lx[LN ? CPL : 1], lg[LN ? CPL : 1], lb[LN ? CPL : 1];
  if constexpr (LN) {
    // wave w: row min(w, nr - 1) of the range's one pair (every LDS row a real row)
    const float* xr = reinterpret_cast<const float*>(xq.qx) + (int64_t)(q_r0[0] + min(wave, q_nr[0] - 1)) * N;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      lx[i] = load4f(xr + 4 * (lane + 64 * i));
      lg[i] = load4f(xq.ln_g + 4 * (lane + 64 * i));
      lb[i] = load4f(xq.ln_b + 4 * (lane + 64 * i));
    }
    bv[0] = xq.bias[q_h[0] * 64 + lane];
  } else if constexpr (DMA) {
    // LDS chunk q of pair j's block holds row q / CPR, chunk (q % CPR) ^ (row & 7) (rows past
    // the window repeat its last row, pairs past the range the last pair: never read)
    constexpr int NBLK = RR * CPR / 64, BPW = (NBLK + 7) / 8;  // 1 KB blocks per pair, per wave
#pragma unroll
    for (int j = 0; j < XS_QF; ++j) {
      const int jj = min(j, np - 1);
      const char* src = reinterpret_cast<const char*>(xq.qx) + (int64_t)q_r0[jj] * (N * (int)sizeof(T));
#pragma unroll
      for (int t = 0; t < BPW; ++t) {
        const int blk = min(wave + 8 * t, NBLK - 1), q = blk * 64 + lane, row = q / CPR, cs = q - row * CPR;
        const char* sp = src + min(row, q_nr[jj] - 1) * (N * (int)sizeof(T)) + ((cs ^ (row & 7)) * 16);
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(sp),
                                         (__attribute__((address_space(3))) void*)(xst + (j * RR * CPR + blk * 64) * 16),
                                         16, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < XS_QF; ++j)
      if (lane < 16)  // 16 lanes x 16 B: the head's 64 fp32 biases
        __builtin_amdgcn_global_load_lds(
            (__attribute__((address_space(1))) void*)(xq.bias + q_h[min(j, np - 1)] * 64 + 4 * lane),
            (__attribute__((address_space(3))) void*)(xst + BIAS_OFF + j * 256), 16, 0, 0);
  } else {
    // unconditional buffer loads: the buffer limit is the window's rows (0 past it and for
    // pairs past the range); the biases by wave 0, one float per lane and pair
    static_assert(N % 256 == 0 || !LN, "LN rows: whole float4 chunks per lane");
#pragma unroll
    for (int j = 0; j < XS_QF; ++j) {
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<T*>(reinterpret_cast<const T*>(xq.qx)) + (int64_t)q_r0[j] * N, 0, j < np ? q_nr[j] * N * (int)sizeof(T) : 0,
          0x00020000);
#pragma unroll
      for (int i = 0; i < XPT; ++i) {
        const int ch = tid + 512 * i, off = (ch / CPR) * (N * (int)sizeof(T)) + (ch % CPR) * 16;
        xv[j][i] = __builtin_bit_cast(float4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      }
    }
#pragma unroll
    for (int j = 0; j < XS_QF; ++j) bv[j] = xq.bias[q_h[min(j, np - 1)] * 64 + lane];
  }
  __builtin_amdgcn_sched_barrier(0);
  // 2. the wave's W_q fragments for the first pair's head: rows h*64 + 16c + r, K half kh
  if constexpr (!W_FIRST) {
    load_w(q_h[0]);
    __builtin_amdgcn_sched_barrier(0);
  }
  // 3. (QV 0 / 1) the first tile's K / V, (1) the second's too
  if constexpr (QV <= 1) {
    load_kv(min(wave, cnt - 1), kA, vA);
    if constexpr (QV == 1) load_kv(min(wave + 8, cnt - 1), kB, vB);
    __builtin_amdgcn_sched_barrier(0);
  }
  // 4. X (and the biases) -> LDS: waits for them alone (issued first; vmcnt retires in order)
  if constexpr (LN) {
    // LayerNorm of the wave's row (biased variance, two passes in registers: k_proj1's
    // prologue arithmetic), stored as the fp16 row
    float sm = 0.f;
#pragma unroll
    for (int i = 0; i < CPL; ++i) sm += lx[i][0] + lx[i][1] + lx[i][2] + lx[i][3];
    const float mean = wave_sum(sm) / (float)N;
    float qv2 = 0.f;
#pragma unroll
    for (int i = 0; i < CPL; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = lx[i][e] - mean;
        qv2 += d * d;
      }
    const float rstd = rsqrtf(wave_sum(qv2) / (float)N + xq.ln_eps);
    if (wave < RR) {
#pragma unroll
      for (int i = 0; i < CPL; ++i) {
        const float4_t v = lx[i];
        store4(reinterpret_cast<T*>(xst + wave * XROWB) + 4 * (lane + 64 * i), (v[0] - mean) * rstd * lg[i][0] + lb[i][0],
               (v[1] - mean) * rstd * lg[i][1] + lb[i][1], (v[2] - mean) * rstd * lg[i][2] + lb[i][2],
               (v[3] - mean) * rstd * lg[i][3] + lb[i][3]);
      }
    }
    if (wave == 0) reinterpret_cast<float*>(xst + BIAS_OFF)[lane] = bv[0];
  } else if constexpr (DMA) {
    static_assert(QK + 32 <= 63, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(QK + 32) : "memory");
  } else {
#pragma unroll
    for (int j = 0; j < XS_QF; ++j)
#pragma unroll
      for (int i = 0; i < XPT; ++i) {
        const int ch = tid + 512 * i;
        if (ch < RR * CPR)
          *reinterpret_cast<float4_t*>(xst + (j * RR + ch / CPR) * XROWB + (ch % CPR) * 16) = xv[j][i];
      }
    if (wave == 0) {
#pragma unroll
      for (int j = 0; j < XS_QF; ++j) reinterpret_cast<float*>(xst + BIAS_OFF)[j * 64 + lane] = bv[j];
    }
  }
  if (tid == 0) {  // the merge's window rows (LDS, behind the barriers below)
#pragma unroll
    for (int j = 0; j < XS_QF; ++j) {
      s_wnr[j] = q_nr[j];
      s_wr0[j] = q_r0[j];
    }
  }
  wh_lds_barrier();
  XS_MARK(7);  // X staged
  // 3'. (QV 2 - 4) the first two tiles' K / V leave now, behind the few KB the projection waited on
  if constexpr (QV >= 2 && QV <= 4) {
    load_kv(min(wave, cnt - 1), kA, vA);
    load_kv(min(wave + 8, cnt - 1), kB, vB);
  }
  // 5. pair by pair: MFMAs in k-step order (W reloaded only where the head changes); each
  // pair's K-half sum goes to LDS at once (no register per pair)
  float4_t* red2 = reinterpret_cast<float4_t*>(xst + RED_OFF);  // [kh][pair][c][lane]
#pragma unroll
  for (int j = 0; j < XS_QF; ++j) {
    if (j < np) {
      if (j > 0 && q_h[j] != q_h[j - 1]) load_w(q_h[j]);
      float4_t acc = (float4_t){0.f, 0.f, 0.f, 0.f};
      const int rr = min(r, RR - 1);
      const char* xl = xst + (j * RR + rr) * XROWB;
#pragma unroll
      for (int s = 0; s < QK; ++s) {
        Frag<T> xf;
        const int ch = kh * QK * 4 + 4 * s + g;  // 16-B chunk of k = kh * N / 2 + 32 s + 8 g
        frag_load(xf, reinterpret_cast<const T*>(xl + (DMA ? (ch ^ (rr & 7)) : ch) * 16));
        mfma_step(acc, wf[s], xf);
      }
      red2[((kh * XS_QF + j) * 4 + c) * 64 + lane] = acc;
    }
  }
  // 3''. (QV 5) the first two tiles' K / V only once the projection has its operands
  if constexpr (QV == 5) {
    load_kv(min(wave, cnt - 1), kA, vA);
    load_kv(min(wave + 8, cnt - 1), kB, vB);
  }
  XS_MARK(8);  // this wave's (thread 0's) MFMAs done: its W_q fragments landed
  // 6. the K halves meet (half 0 + half 1, then the bias) -> qs[pair][row][64] (fp16)
  wh_lds_barrier();
  if (kh == 0) {
    const float* bl = reinterpret_cast<const float*>(xst + BIAS_OFF);
#pragma unroll
    for (int j = 0; j < XS_QF; ++j)
      if (j < np) {
        float4_t v = red2[(j * 4 + c) * 64 + lane] + red2[((XS_QF + j) * 4 + c) * 64 + lane];
        v += *reinterpret_cast<const float4_t*>(bl + j * 64 + c * 16 + 4 * g);
        store4(&qs[j][r][c * 16 + 4 * g], v[0], v[1], v[2], v[3]);
      }
  }
}

// QV 6 (round 6, the single-window step): the query projection split over the XQ1_P workgroups
// of each (window, head) pair instead of computed whole by each of them (QV 3: every one of
// the 240 workgroups ingested its head's 164 KB W_q slice before any tile, 6.1 -> 15.3 us).
// The grid gives every workgroup nsp / XQ1_P tiles of ONE pair; workgroup kpart of the pair
// computes the partial query over k-steps [kpart KS, kpart KS + KS) (KS = 2 QK / XQ1_P), stores
// it write-through into xq.q_part, drains and counts it on the pair's arrival counter; the
// query is the XQ1_P partials summed in kpart order + the bias (the same arithmetic in every
// workgroup of the pair).  Roles: waves < cnt (the tile waves) issue their tile's K / V first
// and wait at the barriers; waves 3-7 compute the LayerNorm of the window's rows (k_proj1's
// arithmetic) into LDS; waves 4-7 (column tile c = wave - 4) run the partial projection; wave
// 3 polls the counter (sc1 loads, bounded: a lost arrival ends the wait with a wrong query,
// never a hang).  Every workgroup of the pair is resident at once (XQ1_P x npair <= 256
// one-workgroup-per-CU launches: the launcher checks).  The last of the pair's workgroups to
// read the partials re-arms both counters (departure count).
template <typename T, int QK, int RR, typename PairWH, typename LoadKV>
WH_DEV void xq_project_split(const XQPart& xq, int pa, int kpart, int cnt, const int* __restrict__ win_row0,
                             const int* __restrict__ win_nrows, PairWH pair_wh, LoadKV load_kv, Frag<T> (&kA)[4][2],
                             Frag<T> (&vA)[4][2], char* xst, T (*qs)[16][72], int* s_wnr, int* s_wr0) {
  static_assert(sizeof(T) == 2, "fused query projection: fp16 contexts");
  constexpr int N = QK * 64, KS = 2 * QK / XQ1_P, CPL = N / 256, XROWB = N * (int)sizeof(T) + 16;
  static_assert((2 * QK) % XQ1_P == 0 && N % 256 == 0 && RR <= 10, "split geometry");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  int wi, h;
  pair_wh(pa, wi, h);
  // the tile waves' K / V leave first (nothing of theirs waits on the query until the tiles)
  if (wave < cnt) load_kv(wave, kA, vA);
  const int nr = win_nrows[wi], r0 = win_row0[wi];
  if (tid == 0) {
    s_wnr[0] = nr;
    s_wr0[0] = r0;
  }
  const bool pw = wave >= 4;  // projection waves: column tile c = wave - 4
  const int c = wave - 4;
  Frag<T> wf[KS];
  if (pw) {  // W_q rows h*64 + 16c + r, k-steps kpart*KS .. + KS - 1
    const T* wp = reinterpret_cast<const T*>(xq.qw) + (int64_t)(h * 64 + c * 16 + r) * N + kpart * KS * 32 + 8 * g;
#pragma unroll
    for (int s = 0; s < KS; ++s) frag_load_stream(wf[s], wp + s * 32);
  }
  // LayerNorm: waves 3..7 take rows wave - 3 and wave + 2 (rows past the window repeat its last)
  if (wave >= 3) {
    float4_t lg[CPL], lb[CPL];
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      lg[i] = load4f(xq.ln_g + 4 * (lane + 64 * i));
      lb[i] = load4f(xq.ln_b + 4 * (lane + 64 * i));
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int row = wave - 3 + 5 * t;
      if (row < RR) {
        const float* xr = reinterpret_cast<const float*>(xq.qx) + (int64_t)(r0 + min(row, nr - 1)) * N;
        float4_t lx[CPL];
#pragma unroll
        for (int i = 0; i < CPL; ++i) lx[i] = load4f(xr + 4 * (lane + 64 * i));
        float sm = 0.f;
#pragma unroll
        for (int i = 0; i < CPL; ++i) sm += lx[i][0] + lx[i][1] + lx[i][2] + lx[i][3];
        const float mean = wave_sum(sm) / (float)N;
        float qv2 = 0.f;
#pragma unroll
        for (int i = 0; i < CPL; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float d = lx[i][e] - mean;
            qv2 += d * d;
          }
        const float rstd = rsqrtf(wave_sum(qv2) / (float)N + xq.ln_eps);
#pragma unroll
        for (int i = 0; i < CPL; ++i) {
          const float4_t v = lx[i];
          store4(reinterpret_cast<T*>(xst + row * XROWB) + 4 * (lane + 64 * i), (v[0] - mean) * rstd * lg[i][0] + lb[i][0],
                 (v[1] - mean) * rstd * lg[i][1] + lb[i][1], (v[2] - mean) * rstd * lg[i][2] + lb[i][2],
                 (v[3] - mean) * rstd * lg[i][3] + lb[i][3]);
        }
      }
    }
  }
  wh_lds_barrier();
  XS_MARK(7);  // rows staged
  const auto rq = wt_rsrc(xq.q_part);
  const int pbase = pa * XQ1_P * 4 * 64 * 16;  // bytes: [pair][kpart][c][lane] float4
  int* const arr = xq.q_cnt + 2 * pa;          // [pair]{arrivals, departures}
  if (pw) {
    float4_t acc = (float4_t){0.f, 0.f, 0.f, 0.f};
    const char* xl = xst + min(r, RR - 1) * XROWB;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      Frag<T> xf;
      frag_load(xf, reinterpret_cast<const T*>(xl + ((kpart * KS + s) * 4 + g) * 16));
      mfma_step(acc, wf[s], xf);
    }
    wt_store4(rq, pbase + ((kpart * 4 + c) * 64 + lane) * 16, acc);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's partial is written through
    if (lane == 0) __hip_atomic_fetch_add(arr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if (wave == 3) {
    const auto ra = wt_rsrc(arr);
    int v = 0;
    for (int it = 0; it < (1 << 16); ++it) {  // (~65 ms: a normal wait is a few us)
      v = (int)__builtin_amdgcn_raw_buffer_load_b32(ra, 0, 0, 16);
      if (v >= 4 * XQ1_P) break;
      __builtin_amdgcn_s_sleep(1);
    }
    (void)v;
  }
  wh_lds_barrier();  // wave 3 has seen every partial of the pair arrive
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below
  if (pw) {
    float4_t pv[XQ1_P];
#pragma unroll
    for (int j = 0; j < XQ1_P; ++j)
      pv[j] = __builtin_bit_cast(float4_t, __builtin_amdgcn_raw_buffer_load_b128(rq, pbase + ((j * 4 + c) * 64 + lane) * 16, 0, 16));
    float4_t q = pv[0];
#pragma unroll
    for (int j = 1; j < XQ1_P; ++j) q += pv[j];
    q += load4f(xq.bias + h * 64 + c * 16 + 4 * g);
    store4(&qs[0][r][c * 16 + 4 * g], q[0], q[1], q[2], q[3]);
    if (wave == 4 && lane == 0) {
      // every workgroup of the pair departs once it has read the partials; the last re-arms
      if (__hip_atomic_fetch_add(arr + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == XQ1_P - 1) {
        __hip_atomic_store(arr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(arr + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  XS_MARK(8);  // query summed
}

template <typename T, int QZ, int RR, typename S = float, bool FULL = false, int QK = 0, int QV = 0>
__global__ __launch_bounds__(512, 1) void k_xattn_seg(const T* __restrict__ q, int ldq, const T* ck, const T* cvt, int Tk,
                                                     int H, int npair, int nsp, const int* __restrict__ win_row0,
                                                     const int* __restrict__ win_nrows,
                                                     const int* __restrict__ win_slot, int64_t win_stride, XQPart xq,
                                                     T* __restrict__ out, int ldo) {
  constexpr int NW = 8, SMAX = XsShape<RR>::SMAX, PPASS = 512 / (RR * 16);  // pairs merged per pass
  constexpr bool QP = QZ > 0;
  // QK > 0 (round 6): the query projection itself runs here (xq.qx rows x xq.qw^T + bias,
  // QK k-steps per K half), pairs are numbered head-major (p = head * nwin + window: a
  // workgroup's pairs share one head's 64 x n slice of W_q) and workgroups are laid over
  // the XCDs in contiguous logical runs, so a head's slice crosses HBM about once per XCD
  constexpr bool QF = QK > 0;
  __shared__ float seg_m[SMAX][RR], seg_l[SMAX][RR];
  // partial outputs row-major, 68-float rows: a lane's 4 columns are one 16-B store / load
  // (tile(): lanes r = 0..7 of a store group hit banks 4r.. +3, conflict-free; round 4 kept
  // [tile][64][RR + 1] and moved them as 16 + 4 single floats)
  __shared__ __attribute__((aligned(16))) float seg_o[SMAX][RR][68];
  __shared__ __attribute__((aligned(16))) T qs[XS_QP][16][72];
  __shared__ int s_ticket[2];
  __shared__ int s_wnr[XS_QP], s_wr0[XS_QP];  // the range's pairs' window rows / first row, for the merge
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int nseg = npair * nsp, nwg = gridDim.x, b = QF ? xcd_remap(blockIdx.x, nwg) : (int)blockIdx.x;
  const int s0 = range_split(b, nseg, nwg), s1 = range_split(b + 1, nseg, nwg), cnt = s1 - s0;
  const int pa = s0 / nsp, plast = (s1 - 1) / nsp;
  const int nwin = QF ? npair / H : 0;
  // pair p -> (window, head)
  auto pair_wh = [&](int p, int& wi, int& h) {
    if constexpr (QF) {
      h = p / nwin;
      wi = p - h * nwin;
    } else {
      wi = p / H;
      h = p - wi * H;
    }
  };
  XS_MARK(0);
  CT_MARK(CT_XATTN, 0);

  // local tile i: K and V fragments
  // (wsl >= 0: the tile's window slot, already loaded)
  auto load_kv = [&](int i, Frag<T>(&kf)[4][2], Frag<T>(&vf)[4][2], int wsl = -1) {
    // i is wave-uniform: the tile's window slot comes by a scalar load (lgkmcnt).  Round 4:
    // as a vector load it sat in vmcnt order, and the s_waitcnt vmcnt(0) before the K / V
    // addresses drained the tile in flight: one tile per wave in flight, not two
    const int gs = __builtin_amdgcn_readfirstlane(s0 + i), p = gs / nsp, k = gs - p * nsp;
    int wi, h;
    pair_wh(p, wi, h);
    const int64_t off = (int64_t)(wsl >= 0 ? wsl : win_slot[wi]) * win_stride;
    const T* kbase = ck + off + (int64_t)h * TKP * 64;
    const T* vbase = cvt + off + (int64_t)h * 64 * TKP;
    const int kt0 = k * 64;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const T* kp = kbase + (int64_t)(kt0 + kt * 16 + r) * 64 + 8 * g;
      frag_load_stream(kf[kt][0], kp);
      frag_load_stream(kf[kt][1], kp + 32);
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int s = 0; s < 2; ++s) frag_load_stream(vf[dt][s], vbase + ((int64_t)k * 64 + dt * 16 + r) * 64 + 32 * s + 8 * g);
  };
  // local tile i's softmax partial -> LDS slot i
  auto tile = [&](const Frag<T>(&kf)[4][2], const Frag<T>(&vf)[4][2], int i) {
    const int gs = s0 + i, p = gs / nsp, kt0 = (gs - p * nsp) * 64;
    Frag<T> qf[2];
    frag_load(qf[0], &qs[p - pa][r][8 * g]);
    frag_load(qf[1], &qs[p - pa][r][32 + 8 * g]);
    float4_t sc[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      sc[kt] = (float4_t){0.f, 0.f, 0.f, 0.f};
      mfma_step(sc[kt], kf[kt][0], qf[0]);
      mfma_step(sc[kt], kf[kt][1], qf[1]);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (kt0 + kt * 16 + 4 * g + j >= Tk) sc[kt][j] = -INFINITY;
        mx = fmaxf(mx, sc[kt][j]);
      }
    mx = xor16_max(mx);
    mx = xor32_max(mx);
    Frag<T> pf[2];
    float ps = 0.f;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float pv = hw_exp2((sc[kt][j] - mx) * XS_LOG2E);
        ps += pv;
        pf[kt >> 1].v[(kt & 1) * 4 + j] = from_f32<T>(pv);
      }
    ps = xor16_sum(ps);
    ps = xor32_sum(ps);
    float4_t acc[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) acc[dt] = (float4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) mfma_step(acc[dt], vf[dt][s], pf[s]);
    if (r < RR) {
      if (g == 0) {
        seg_m[i][r] = mx;
        seg_l[i][r] = ps;
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        *reinterpret_cast<float4_t*>(&seg_o[i][r][dt * 16 + 4 * g]) = acc[dt];
    }
  };

  Frag<T> kA[4][2], vA[4][2], kB[4][2], vB[4][2];
  // the query rows of the pairs this range touches -> LDS (rows past a window's beams
  // repeat its last row).  Round 4: their loads are issued BEFORE the first tile's K / V:
  // vmcnt retires loads in issue order, so the staging below waits for the query alone,
  // the barrier passes ~a round trip in, and the second tile's K / V leave while the first
  // burst is still landing (the query used to wait behind the whole first tile,
  // profiles/xattn_trace.py: query staged at 5.3 us of a 34 us launch at 20 windows)
  constexpr int NQP = XS_QP / 2;
  if constexpr (QF) {
    static_assert(XS_QF * RR * (QK * 64 * sizeof(T) + 16) + 2 * XS_QF * 4 * 64 * 16 + XS_QF * 256 <= sizeof(seg_o),
                  "X rows, K-half sums and biases in the partials' LDS");
    static_assert(XS_QF * 4 * 64 * 16 <= sizeof(seg_o), "K-half sums in the partials' LDS");
    if constexpr (QV == 6)
      xq_project_split<T, QK, RR>(xq, pa, (s0 - pa * nsp) / max(cnt, 1), cnt, win_row0, win_nrows, pair_wh, load_kv, kA,
                                  vA, reinterpret_cast<char*>(&seg_o[0][0][0]), qs, s_wnr, s_wr0);
    else
      xq_project<T, QK, RR, QV>(xq, pa, plast, cnt, win_row0, win_nrows, pair_wh, load_kv, kA, vA, kB, vB,
                                reinterpret_cast<char*>(&seg_o[0][0][0]), qs, s_wnr, s_wr0);
  } else {
  // FULL (the launcher: every workgroup holds >= 8 tiles, one per wave at least): the order
  // above; otherwise (few windows, <= 1 tile per wave) the first tile leaves first, as the
  // query then has no second tile to overlap
  if constexpr (!FULL) {
    if (wave < cnt) load_kv(wave, kA, vA);
  }
  float4_t qld[NQP][QP ? QZ + 1 : 1];  // QP: the QZ slabs, then the bias
  // wave-uniform pairs: their windows' metadata by scalar loads (lgkmcnt, not behind
  // vmcnt), all issued before the first use: one round trip, not one per load and pass
  int q_hj[NQP], q_nr[NQP], q_r0[NQP];
#pragma unroll
  for (int pass = 0; pass < NQP; ++pass) {
    const int pj = __builtin_amdgcn_readfirstlane(min(pa + 2 * pass + (tid >> 8), plast)), wj = pj / H;
    q_hj[pass] = pj - wj * H;
    q_nr[pass] = win_nrows[wj];
    q_r0[pass] = win_row0[wj];
  }
  // FULL: the first tile's window slot rides in the same round trip
  const int slot0 = FULL ? win_slot[__builtin_amdgcn_readfirstlane(s0 + wave) / nsp / H] : -1;
  __builtin_amdgcn_sched_barrier(0);  // (else the second pass's loads sink below the first's wait)
#pragma unroll
  for (int pass = 0; pass < NQP; ++pass) {
    const int t = tid & 255;
    if (t == 0) {  // kept for the merge (LDS, behind the staging barrier): no global round trip there
      s_wnr[2 * pass + (tid >> 8)] = q_nr[pass];
      s_wr0[2 * pass + (tid >> 8)] = q_r0[pass];
    }
    const int qq = min(t >> 4, q_nr[pass] - 1), c = q_hj[pass] * 64 + (t & 15) * 4, row = q_r0[pass] + qq;
    if constexpr (QP) {
      const S* src = reinterpret_cast<const S*>(xq.part) + (int64_t)row * ldq + c;
#pragma unroll
      for (int z = 0; z < QZ; ++z) qld[pass][z] = load4f(src + z * xq.stride);
      qld[pass][QZ] = load4f(xq.bias + c);
    } else {
      qld[pass][0] = load4f(q + (int64_t)row * ldq + c);
    }
  }
  if constexpr (FULL) {
    __builtin_amdgcn_sched_barrier(0);  // keep the K / V loads behind the query's
    // every wave's query loads enter the CU's memory pipeline before any wave's K / V
    // (a barrier that waits for nothing: no s_waitcnt before it)
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  auto stage_q = [&] {
#pragma unroll
    for (int pass = 0; pass < NQP; ++pass) {
      const int j = 2 * pass + (tid >> 8), t = tid & 255;
      float4_t qv = qld[pass][0];
      if constexpr (QP) {
        qv = qld[pass][QZ];
#pragma unroll
        for (int z = 0; z < QZ; ++z) qv += qld[pass][z];
      }
      store4(&qs[j][t >> 4][(t & 15) * 4], qv[0], qv[1], qv[2], qv[3]);
    }
  };
  // FULL: unconditional (every wave has a tile), so no branch join: behind one the
  // compiler's vmcnt bookkeeping made the query staging wait for the K / V loads as well
  if constexpr (FULL) {
    load_kv(wave, kA, vA, slot0);
    __builtin_amdgcn_sched_barrier(0);
  }
  stage_q();
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // LDS only
  XS_MARK(1);

  if (QF && QV == 6) {
    if (wave < cnt) tile(kA, vA, wave);  // (the launcher: <= NW tiles per workgroup)
  } else if (QF && QV >= 1 && wave < cnt) {
    // (QV 1 / 2) kB / vB already hold tile wave + NW (clamped): the next tile is in flight on
    // entry, so each iteration refills the buffer it has just computed
    int i = wave;
    for (; i + 2 * NW < cnt; i += 2 * NW) {
      tile(kA, vA, i);
      load_kv(i + 2 * NW, kA, vA);
      tile(kB, vB, i + NW);
      load_kv(min(i + 3 * NW, cnt - 1), kB, vB);
    }
    if (i + NW < cnt) {
      tile(kA, vA, i);
      tile(kB, vB, i + NW);
    } else {
      tile(kA, vA, i);
    }
  } else if (wave < cnt) {
    int i = wave;
    // two tiles per iteration, the next one always in flight (unconditional loads)
    for (; i + 2 * NW < cnt; i += 2 * NW) {
      load_kv(i + NW, kB, vB);
      tile(kA, vA, i);
      load_kv(i + 2 * NW, kA, vA);
      tile(kB, vB, i + NW);
    }
    if (i + NW < cnt) {
      load_kv(i + NW, kB, vB);
      tile(kA, vA, i);
      tile(kB, vB, i + NW);
    } else {
      tile(kA, vA, i);
    }
  }
  XS_MARK(2);
  __syncthreads();
  XS_MARK(3);

  // merge: RR * 16 threads per pair, (row qq, 4 columns dc)
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(xq.split_rec, 0, 0x7fffffff, 0x00020000);
  const int part = tid / (RR * 16), t = tid - part * (RR * 16), qq = t >> 4, dc = (t & 15) * 4;
  auto emit = [&](int pj, const float4_t& o) {
    int wj, hj;
    pair_wh(pj, wj, hj);
    store4(out + (int64_t)(s_wr0[pj - pa] + qq) * ldo + hj * 64 + dc, o[0], o[1], o[2], o[3]);
  };
#pragma unroll
  for (int pass = 0; pass < (XS_QP + PPASS - 1) / PPASS; ++pass) {
    const int pj = pa + pass * PPASS + part;
    if (pj <= plast && qq < s_wnr[pj - pa]) {
      const int l0 = pj * nsp - s0, l1 = l0 + nsp;  // the pair's tiles as local slots
      if (l0 >= 0 && l1 <= cnt) {                   // whole here: merge from LDS
        emit(pj, xs_merge(nsp, [&](int k, float& m, float& l, float4_t& o) {
               m = seg_m[l0 + k][qq];
               l = seg_l[l0 + k][qq];
               o = *reinterpret_cast<const float4_t*>(&seg_o[l0 + k][qq][dc]);
             }));
      } else {  // cut: this workgroup's partials of the pair -> records [pair][tile]
        for (int s = max(l0, 0); s < min(l1, cnt); ++s) {
          const int rb = (pj * nsp + (s - l0)) * XREC * 4;
          const float4_t o = *reinterpret_cast<const float4_t*>(&seg_o[s][qq][dc]);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rs, rb + (qq * 64 + dc) * 4, 0, 16);
          if (dc == 0) {
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, seg_m[s][qq]), rs, rb + (1024 + qq) * 4, 0, 16);
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, seg_l[s][qq]), rs, rb + (1040 + qq) * 4, 0, 16);
          }
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its records
  __syncthreads();
  XS_MARK(4);
  // the cut pairs: the first if it began before this range, the last if it continues
  // after it (the same pair when the range lies inside one pair)
  const bool cut_a = pa * nsp < s0 || pa * nsp + nsp > s1;
  const bool cut_b = plast != pa && plast * nsp + nsp > s1;
  if (tid == 0) {
    const int ca = min(s1, pa * nsp + nsp) - s0, cb = s1 - plast * nsp;
    s_ticket[0] = cut_a && __hip_atomic_fetch_add(xq.split_cnt + pa, ca, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + ca == nsp;
    s_ticket[1] = cut_b && __hip_atomic_fetch_add(xq.split_cnt + plast, cb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + cb == nsp;
  }
  __syncthreads();
  XS_MARK(5);
  CT_MARK(CT_XATTN, 3);
  if (part > 1 || !s_ticket[part]) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the add
  const int pj = part ? plast : pa;
  if (t == 0) __hip_atomic_store(xq.split_cnt + pj, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (qq >= s_wnr[pj - pa]) return;  // only the window's rows were recorded
  emit(pj, xs_merge(nsp, [&](int k, float& m, float& l, float4_t& o) {
         const int rb = (pj * nsp + k) * XREC * 4;
         m = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, rb + (1024 + qq) * 4, 0, 16));
         l = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, rb + (1040 + qq) * 4, 0, 16));
         o = __builtin_bit_cast(float4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, rb + (qq * 64 + dc) * 4, 0, 16));
       }));
  XS_MARK(6);
}

#if WH_TUNING
}  // namespace wh
WH_CT_READER(kernels)
extern "C" int wh_tune_xs_trace(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(wh::g_xs_trace), sizeof(wh::g_xs_trace)) == hipSuccess ? 0 : -1;
}
namespace wh {
#endif

// Workgroups for nseg = npair x nsp tiles (speed only; the numerics do not depend on it).
//  * whole pairs per workgroup when that still fills >= 3/4 of the 256 CUs (20 windows:
//    200 workgroups of 2 pairs): no pair is cut, so no records, counters or second merge;
//  * else every wave gets the same number of tiles k = ceil(nseg / (256 x 8)) (the last
//    workgroup excepted), cut pairs merged by the last arriver (15 windows: 225
//    workgroups of 32 tiles rather than 150 of 2 pairs);
//  * k = 1 spreads the tiles over up to 256 workgroups (few windows: latency).
// Tuning builds: WHISPER_HIP_XS_K forces k (read per launch; disables the whole-pair rule).
int xattn_seg_grid(int npair, int nsp, int smax) {
  const int nseg = npair * nsp;
  int k = (nseg + 256 * 8 - 1) / (256 * 8), forced = 0;
  if (const char* e = tune_env("WHISPER_HIP_XS_K")) {
    const int v = atoi(e);
    if (v >= 1) k = v, forced = 1;
    if (v < 0) {  // tuning: spread over min(-v, nseg) workgroups, uneven waves
      const int nwg = std::min(-v, nseg);
      return (nseg + nwg - 1) / nwg > smax ? (nseg + smax - 1) / smax : nwg;
    }
  }
  if (!forced && npair >= 192) {
    const int ppw = (npair + 255) / 256, nwg = (npair + ppw - 1) / ppw;
    if (nwg >= 192 && ppw * nsp <= smax) return nwg;
  }
  if (k > smax / 8) k = smax / 8;
  // k = 1: spread over 200 workgroups, not 256 (1 / 2 / 4 windows 10.2 -> 9.6, 11.2 -> 11.1,
  // 14.1 -> 13.9 us, profiles/r03/xattn_grid_few_windows.txt)
  int nwg = k == 1 ? (nseg < 200 ? nseg : 200) : (nseg + 8 * k - 1) / (8 * k);
  if ((nseg + nwg - 1) / nwg > smax) nwg = (nseg + smax - 1) / smax;
  return nwg;
}

bool xattn_l2_ranges(int nwin, int H, int max_rows, L2Prefetch* pf) {
  const int npair = nwin * H, nsp = XS_NSP, nseg = npair * nsp;
  const int nwg = xattn_seg_grid(npair, nsp, max_rows <= 8 ? XsShape<8>::SMAX : XsShape<16>::SMAX);
  if (nwg < 16) return false;
  const int q = nwg / 8, r = nwg % 8;
  for (int x = 0; x < 8; ++x) {
    const int L0 = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q, cnt = q + (x < r ? 1 : 0);
    const unsigned s0 = (unsigned)L0 * (unsigned)nseg / (unsigned)nwg,
                   s1 = (unsigned)(L0 + cnt) * (unsigned)nseg / (unsigned)nwg;  // range_split
    if (cnt == 0 || s1 <= s0) {
      pf->lo[x] = pf->hi[x] = 0;
      continue;
    }
    pf->lo[x] = (int)(s0 / nsp) / nwin;             // head-major pairs: p = head * nwin + window
    pf->hi[x] = (int)((s1 - 1) / nsp) / nwin + 1;
  }
  return true;
}

__global__ __launch_bounds__(256) void k_wq_frag(const half_t* __restrict__ w, half_t* __restrict__ f, int n) {
  const int QK = n / 64, total = n * n / 8;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int l = i % 64, t0 = i / 64, s = t0 % QK, t1 = t0 / QK, kh = t1 % 2, t2 = t1 / 2, c = t2 % 4, h = t2 / 4;
    const int row = h * 64 + c * 16 + (l & 15), col = kh * (n / 2) + 32 * s + 8 * (l >> 4);
    *reinterpret_cast<float4_t*>(f + (int64_t)i * 8) = *reinterpret_cast<const float4_t*>(w + (int64_t)row * n + col);
  }
}
void launch_wq_frag(const void* w, void* f, int n, hipStream_t st) {
  k_wq_frag<<<256, 256, 0, st>>>(reinterpret_cast<const half_t*>(w), reinterpret_cast<half_t*>(f), n), wh_launched("k_wq_frag");
}

// Round 6 probe (tuning build, WHISPER_HIP_XKV_PF=<workgroups>): pull one layer's cross-
// attention K and V blocks of the batch's windows through the memory side on a second
// stream beside the layer's launch chain, so that k_xattn_seg reads them from the Infinity
// Cache (256 MiB; 157 MB at 20 windows) instead of HBM.  (Register loads folded into a
// dummy word: hipcc copied the loop-carried registers and waited on every load.)
__global__ __launch_bounds__(256) void k_kv_pull(const char* __restrict__ ck, const char* __restrict__ cv,
                                                 const int* __restrict__ win_slot, int nwin, int64_t slot_bytes) {
  // workgroup b: 32-KB pieces b, b + grid, ... of the windows' K then V blocks; each wave
  // moves 8 KB of a piece by LDS-DMA into a 1-KB sink (no registers, nothing read back) and
  // keeps at most 24 KB in flight (explicit vmcnt: the DMA's only consumer is the exit)
  constexpr int64_t CH = 32768;
  __shared__ __attribute__((aligned(16))) char sink[1024];
  const int tid = threadIdx.x, lane = tid & 63;
  const int cpb = (int)(slot_bytes / CH), total = 2 * nwin * cpb;
  for (int c = blockIdx.x; c < total; c += gridDim.x) {
    const int blk = c / cpb, w = blk >> 1;
    int slot;  // a scalar load: a vector one would retire behind the DMA loads (vmcnt in order)
    asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(slot) : "s"(win_slot + w) : "memory");
    const char* p = ((blk & 1) ? cv : ck) + (int64_t)slot * slot_bytes + (int64_t)(c - blk * cpb) * CH + tid * 16;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(p + u * 4096),
                                       (__attribute__((address_space(3))) void*)(sink), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA into the sink after the workgroup ends
  (void)lane;
}
void launch_kv_pull(const void* ck, const void* cv, const int* win_slot, int nwin, int64_t slot_bytes, int nwg,
                    unsigned* sink, hipStream_t st) {
  (void)sink;
  if (nwin <= 0 || nwg <= 0 || slot_bytes % 32768) return;
  k_kv_pull<<<nwg, 256, 0, st>>>(reinterpret_cast<const char*>(ck), reinterpret_cast<const char*>(cv), win_slot, nwin,
                                 slot_bytes), wh_launched("k_kv_pull");
}

template <typename T>
void launch_cross_attn(const T* q, int ldq, const T* ck, const T* cv, int Tk, int H, int nsplit, int nwin,
                       const int* win_row0, const int* win_nrows, const int* win_slot, int64_t win_stride, float* po,
                       float* pm, float* pl, T* out, int ldo, int rows, float* qk_out, const int* qk_map, int qk_rows,
                       hipStream_t st, XQPart xq) {
  if (rows <= 0) return;
  const int nsp = (Tk + 63) / 64;
  // the decoder step (<= 16 query rows per window, no alignment capture): tile partials
  if (xq.max_rows >= 1 && xq.max_rows <= 16 && !qk_map && xq.split_rec && xq.split_cnt && nsp <= XS_NSP &&
      nwin * H <= xq.max_pairs) {
    const int npair = nwin * H;
    // FULL: every workgroup's range holds >= 8 tiles (one per wave), e.g. 20 windows
    const int nwg_xs = xattn_seg_grid(npair, nsp, xq.max_rows <= 8 ? XsShape<8>::SMAX : XsShape<16>::SMAX);
    const bool full = (npair * nsp) / nwg_xs >= 8;
    if (xq.qx) {  // the query projected in the kernel (round 6)
      if constexpr (sizeof(T) == 2) {
        if (!xq.qw || !xq.bias || !xattn_fused_q(H * 64, xq.max_rows, (int)sizeof(T)) || nsp != XS_NSP) {
          wh_set_launch_error("launch_cross_attn: fused query projection outside its shapes");
          return;
        }
        if (xq.ln_g) {
          // the single-window step: fp32 rows + LayerNorm in the kernel; every workgroup holds
          // 2 tiles of ONE pair (nsp even): 12 workgroups per pair, merged through records
          if (nwin != 1 || !xq.ln_b || nsp % 2) {
            wh_set_launch_error("launch_cross_attn: in-kernel LayerNorm query is the single-window form");
            return;
          }
          if (xq.q_part && xq.q_cnt) {
            // QV 6: the projection split over the XQ1_P workgroups of each pair (all resident:
            // one 512-thread workgroup per CU, npair x XQ1_P <= 256)
            if (nsp % XQ1_P || nsp / XQ1_P > 8 || npair * XQ1_P > 256 || xq.max_rows > 10) {
              wh_set_launch_error("launch_cross_attn: split query projection outside its shapes");
              return;
            }
            k_xattn_seg<T, 0, 8, float, false, 20, 6><<<npair * XQ1_P, 512, 0, st>>>(
                q, ldq, ck, cv, Tk, H, npair, nsp, win_row0, win_nrows, win_slot, win_stride, xq, out, ldo),
                wh_launched("k_xattn_seg<qproj-split+ln>");
            return;
          }
          k_xattn_seg<T, 0, 8, float, false, 20, 3><<<npair * nsp / 2, 512, 0, st>>>(
              q, ldq, ck, cv, Tk, H, npair, nsp, win_row0, win_nrows, win_slot, win_stride, xq, out, ldo),
              wh_launched("k_xattn_seg<qproj,ln>");
          return;
        }
        // load-order variant (xq_project): 2 unless the tuning build's WHISPER_HIP_XQV says 0 / 1
        static const int qv = [] {
          const char* e = tune_env("WHISPER_HIP_XQV");
          return e ? atoi(e) : 2;
        }();
#define XQF(FULL_, QV_)                                                                                            \
  k_xattn_seg<T, 0, 8, float, FULL_, 20, QV_><<<nwg_xs, 512, 0, st>>>(q, ldq, ck, cv, Tk, H, npair, nsp, win_row0, \
                                                                      win_nrows, win_slot, win_stride, xq, out, ldo), \
      wh_launched("k_xattn_seg<qproj>")
        if (full) {
          if (qv == 2) XQF(true, 2);
          else if (qv == 4) XQF(true, 4);
          else if (qv == 5) XQF(true, 5);
          else if (qv == 1) XQF(true, 1);
          else XQF(true, 0);
        } else {
          if (qv == 2) XQF(false, 2);
          else if (qv == 4) XQF(false, 4);
          else if (qv == 5) XQF(false, 5);
          else if (qv == 1) XQF(false, 1);
          else XQF(false, 0);
        }
#undef XQF
      } else {
        wh_set_launch_error("launch_cross_attn: fused query projection in an fp32 context");
      }
      return;
    }
#define XSF(QZ_, RR_, S_)                                                                                         \
  if (full)                                                                                                     \
    k_xattn_seg<T, QZ_, RR_, S_, true><<<nwg_xs, 512, 0, st>>>(q, ldq, ck, cv, Tk, H, npair, nsp, win_row0,       \
                                                               win_nrows, win_slot, win_stride, xq, out, ldo), wh_launched("k_xattn_seg");   \
  else                                                                                                          \
    k_xattn_seg<T, QZ_, RR_, S_, false><<<nwg_xs, 512, 0, st>>>(q, ldq, ck, cv, Tk, H, npair, nsp, win_row0,      \
                                                                win_nrows, win_slot, win_stride, xq, out, ldo), wh_launched("k_xattn_seg")
#define XS(QZ_, RR_)          \
  if (xq.part_half) {         \
    XSF(QZ_, RR_, half_t);    \
  } else {                    \
    XSF(QZ_, RR_, float);     \
  }
#define XSR(QZ_)                        \
  if (xq.max_rows <= 8) {               \
    XS(QZ_, 8);                         \
  } else {                              \
    XS(QZ_, 16);                        \
  }
    switch (xq.part ? xq.z : 0) {
      case 4: XSR(4) break;
      case 8: XSR(8) break;
      case 10: XSR(10) break;
      default: XSR(0) break;
    }
#undef XSR
#undef XS
#undef XSF
    return;
  }
  // first passes (prefill, alignment capture): one 64-key tile per wave, 8 waves per
  // split, partials combined by k_cross_combine (fp32 query slabs only: the runtime hands
  // fp16 slabs to the step kernel above alone)
  if (xq.part_half) {
    fprintf(stderr, "launch_cross_attn: fp16 query slabs outside the step kernel\n");
    abort();
  }
  constexpr int NW = 8;
  nsplit = (nsp + NW - 1) / NW;
  const dim3 grid(nwin, H, nsplit);
#define XA(QZ_)                                                                                          \
  k_cross_attn<T, NW, QZ_><<<grid, 64 * NW, 0, st>>>(q, ldq, ck, cv, Tk, H, nsplit, win_row0, win_nrows, win_slot, \
                                                     win_stride, po, pm, pl, qk_out, qk_map, qk_rows, xq), wh_launched("k_cross_attn")
  switch (xq.part ? xq.z : 0) {
    case 4: XA(4); break;
    case 8: XA(8); break;
    case 10: XA(10); break;
    default: XA(0); break;
  }
#undef XA
  k_cross_combine<T><<<dim3(rows, H), 64, 0, st>>>(po, pm, pl, H, nsplit, out, ldo), wh_launched("k_cross_combine");
}

// ============================================================ embedding
// x[r] = E[tok] + P[pos] (fp32 residual).  State mode (hist != null): row r = w*G + b,
// tok = hist[(w*G+b)*hctx + len[w]-1], pos = len[w]-1, and row_pos[r] is written.
template <typename T>
__global__ __launch_bounds__(256) void k_embed(const T* __restrict__ E, const T* __restrict__ P, int n,
                                               const int* __restrict__ row_tok, int* __restrict__ row_pos,
                                               const int* __restrict__ hist, const int* __restrict__ cur_len, int G,
                                               int hctx, int pmax, float* __restrict__ x) {
  const int r = blockIdx.x;
  int tok, pos;
  if (hist) {
    const int w = r / G;
    pos = min(cur_len[w] - 1, pmax);  // finished windows past n_ctx keep recomputing a valid row
    tok = hist[(int64_t)r * hctx + pos];
    if (threadIdx.x == 0) row_pos[r] = pos;
  } else {
    tok = row_tok[r];
    pos = row_pos[r];
  }
  for (int c = threadIdx.x; c < n; c += 256)
    x[(int64_t)r * n + c] = to_f32(E[(int64_t)tok * n + c]) + to_f32(P[(int64_t)pos * n + c]);
}

template <typename T>
void launch_embed(const T* E, const T* P, int n, const int* row_tok, int* row_pos, const int* hist,
                  const int* cur_len, int G, int hctx, int pmax, float* x, int rows, hipStream_t st) {
  if (rows <= 0) return;
  k_embed<T><<<rows, 256, 0, st>>>(E, P, n, row_tok, row_pos, hist, cur_len, G, hctx, pmax, x), wh_launched("k_embed");
}

// ============================================================ encoder input prep
// mel [n_mels][ld_mel] (normalized, f32) -> melT[w][1 + t][n_mels] (T), zero rows at
// t = -1 and t >= seg (pad_or_trim), slice [seek, seek+seg) of the full mel.
template <typename T>
__global__ void k_mel_windows(const float* __restrict__ mel, int64_t ld_mel, int n_mels, const int64_t* __restrict__ seeks,
                              const int* __restrict__ segs, T* __restrict__ melT, int64_t win_stride, int rows_alloc) {
  const int w = blockIdx.y;
  const int64_t seek = seeks[w];
  const int seg = segs[w];
  const int total = rows_alloc * n_mels;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int rr = i / n_mels, c = i - rr * n_mels;
    const int t = rr - 1;
    float v = 0.f;
    if (t >= 0 && t < 3000 && t < seg) v = mel[(int64_t)c * ld_mel + seek + t];
    melT[(int64_t)w * win_stride + i] = from_f32<T>(v);
  }
}

template <typename T>
void launch_mel_windows(const float* mel, int64_t ld_mel, int n_mels, const int64_t* seeks, const int* segs, T* melT,
                        int64_t win_stride, int rows_alloc, int nwin, hipStream_t st) {
  k_mel_windows<T><<<dim3(64, nwin), 256, 0, st>>>(mel, ld_mel, n_mels, seeks, segs, melT, win_stride, rows_alloc), wh_launched("k_mel_windows");
}

// zero pad rows around the conv1 output (rows 0 and 3001 of each window)
template <typename T>
__global__ void k_zero_rows(T* buf, int64_t win_stride, int n, int row_a, int row_b) {
  const int w = blockIdx.x;
  for (int c = threadIdx.x; c < n; c += blockDim.x) {
    buf[(int64_t)w * win_stride + (int64_t)row_a * n + c] = from_f32<T>(0.f);
    buf[(int64_t)w * win_stride + (int64_t)row_b * n + c] = from_f32<T>(0.f);
  }
}
template <typename T>
void launch_zero_rows(T* buf, int64_t ws, int n, int ra, int rb, int nwin, hipStream_t st) {
  k_zero_rows<T><<<nwin, 256, 0, st>>>(buf, ws, n, ra, rb), wh_launched("k_zero_rows");
}

// ============================================================ log-mel spectrogram
// audio.py:110-157.  Frame f is centred at f*160 with reflect padding; 400-point
// periodic Hann; |DFT|^2 for bins 0..200 (direct DFT, fp32, twiddles from a
// 400-entry table); mel = filters @ power; log10(max(mel, 1e-10)).  The global max
// is accumulated with an ordered-uint atomicMax; k_mel_norm applies max(x, gmax-8)
// and (x+4)/4.  16 frames per block.
constexpr int MEL_FB = 16;
__global__ __launch_bounds__(256) void k_mel_frames(const float* __restrict__ audio, int64_t n_real, int64_t n_audio, int64_t nframes,
                                                    int64_t frame0, const float* __restrict__ filters, int n_mels,
                                                    float* __restrict__ mel, int64_t ld_mel, unsigned* gmax) {
  __shared__ float xs[MEL_FB][400];
  __shared__ float cs[400], sn[400];
  __shared__ float pw[MEL_FB][201];
  const int tid = threadIdx.x;
  const int64_t f0 = frame0 + (int64_t)blockIdx.x * MEL_FB;
  for (int i = tid; i < 400; i += 256) {
    float s, c;
    sincospif((float)i / 200.0f, &s, &c);  // angle 2*pi*i/400
    cs[i] = c;
    sn[i] = s;
  }
  for (int i = tid; i < MEL_FB * 400; i += 256) {
    const int fi = i / 400, j = i - fi * 400;
    const int64_t f = f0 + fi;
    float v = 0.f;
    if (f < nframes) {
      int64_t idx = f * 160 + j - 200;
      if (idx < 0) idx = -idx;
      if (idx >= n_audio) idx = 2 * (n_audio - 1) - idx;
      v = idx < n_real ? audio[idx] : 0.f;  // right zero-padding is virtual
    }
    xs[fi][j] = v;
  }
  __syncthreads();
  for (int i = tid; i < MEL_FB * 400; i += 256) {
    const int fi = i / 400, j = i - fi * 400;
    // periodic hann: 0.5 - 0.5 cos(2 pi j / 400)
    xs[fi][j] *= 0.5f - 0.5f * cs[j];
  }
  __syncthreads();
  for (int i = tid; i < MEL_FB * 201; i += 256) {
    const int fi = i / 201, k = i - fi * 201;
    float re = 0.f, im = 0.f;
    int ph = 0;
    for (int j = 0; j < 400; ++j) {
      const float x = xs[fi][j];
      re += x * cs[ph];
      im -= x * sn[ph];
      ph += k;
      if (ph >= 400) ph -= 400;
    }
    pw[fi][k] = re * re + im * im;
  }
  __syncthreads();
  float lmax = -INFINITY;
  for (int i = tid; i < MEL_FB * n_mels; i += 256) {
    const int fi = i / n_mels, m = i - fi * n_mels;
    const int64_t f = f0 + fi;
    if (f >= nframes) continue;
    const float* fr = filters + m * 201;
    float s = 0.f;
    for (int k = 0; k < 201; ++k) s += fr[k] * pw[fi][k];
    const float lv = log10f(fmaxf(s, 1e-10f));
    mel[(int64_t)m * ld_mel + (f - frame0)] = lv;
    lmax = fmaxf(lmax, lv);
  }
  lmax = wave_max(lmax);
  if ((tid & 63) == 0) atomicMax(gmax, f2ord(lmax));
}

__global__ void k_mel_norm(float* mel, int64_t count_per_row, int64_t ld, int n_mels, const unsigned* gmax,
                           const float* gmax_override) {
  const float mx = gmax_override ? *gmax_override : ord2f(*gmax);
  const float floor_v = mx - 8.0f;
  const int64_t total = (int64_t)n_mels * count_per_row;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int m = (int)(i / count_per_row);
    const int64_t f = i - (int64_t)m * count_per_row;
    float* p = mel + (int64_t)m * ld + f;
    *p = (fmaxf(*p, floor_v) + 4.0f) * 0.25f;
  }
}

void launch_mel(const float* audio, int64_t n_real, int64_t n_padded, int64_t frame0, int64_t count,
                const float* filters, int n_mels, float* mel, int64_t ld, unsigned* gmax, hipStream_t st) {
  const int64_t nb = (count + MEL_FB - 1) / MEL_FB;
  if (nb > 0)
    k_mel_frames<<<(unsigned)nb, 256, 0, st>>>(audio, n_real, n_padded, frame0 + count, frame0, filters, n_mels, mel, ld, gmax), wh_launched("k_mel_frames");
}
void launch_mel_norm(float* mel, int64_t count, int64_t ld, int n_mels, const unsigned* gmax, const float* ovr,
                     hipStream_t st) {
  k_mel_norm<<<1024, 256, 0, st>>>(mel, count, ld, n_mels, gmax, ovr), wh_launched("k_mel_norm");
}

// explicit instantiations
#define INST(T)                                                                                                     \
  template void launch_layernorm<T>(const float*, T*, const float*, const float*, int, int, float, const int*,     \
                                    hipStream_t);                                                                   \
  template void launch_resid_ln<T>(float*, const float*, int, int64_t, const float*, T*, const float*, const float*, \
                                   int, int, float, hipStream_t, int, const L2Prefetch*);                           \
  template int launch_self_attn_qkv<T>(const float*, int, int64_t, const float*, int, T*, T*, const int*, const int*, \
                                        const int*, const int*, int, int, int, int, T*, int, int, hipStream_t, int); \
  template void launch_reduce_store<T>(const float*, int, int64_t, const float*, T*, int, int, int, int, hipStream_t, \
                                       int);                                                                        \
  template void launch_attn_enc<T>(const T*, int, int, int, int, int, int64_t, const T*, int, T*, int64_t,         \
                                   hipStream_t);                                                                    \
  template void launch_self_attn<T>(const T*, int, const T*, const T*, const int*, const int*, const int*,         \
                                    const int*, int, int, int, int, T*, int, int, hipStream_t);                          \
  template void launch_cross_attn<T>(const T*, int, const T*, const T*, int, int, int, int, const int*, const int*, \
                                     const int*, int64_t, float*, float*, float*, T*, int, int, float*,             \
                                     const int*, int, hipStream_t, XQPart);                                                 \
  template void launch_embed<T>(const T*, const T*, int, const int*, int*, const int*, const int*, int, int, int,  \
                                float*, int, hipStream_t);                                                          \
  template void launch_mel_windows<T>(const float*, int64_t, int, const int64_t*, const int*, T*, int64_t, int, int, \
                                      hipStream_t);                                                                 \
  template void launch_zero_rows<T>(T*, int64_t, int, int, int, int, hipStream_t);
INST(float)
INST(half_t)
#undef INST

}  // namespace wh
