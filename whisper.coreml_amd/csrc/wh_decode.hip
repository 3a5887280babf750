// Device-side token selection: logit filters, log-softmax, greedy/beam update.
//
// Restates, as fixed-shape kernels that can live inside the per-token hipGraph,
// the host-side Python of the reference's decode loop:
//   SuppressBlank / SuppressTokens / ApplyTimestampRules  (whisper/decoding.py:450-532)
//   GreedyDecoder.update                                  (decoding.py:304-320)
//   BeamSearchDecoder.update incl. finished bookkeeping   (decoding.py:350-409)
//   PyTorchInference.rearrange_kv_cache                   (decoding.py:189-204) -> index indirection
// k_logit_part + k_logit_combine (default): 8 or 32 vocabulary slices per row, one workgroup
//               each, then one wave per row merging the kept slices.
// k_logit_rows: the single-workgroup form (one 1024-thread workgroup per decoder row;
//               WHISPER_HIP_LOGIT_SPLIT=0).
// k_merge     : one workgroup per window (candidate merge, history/ancestry update).
#include <cstdlib>

#include "wh_gemm.h"
#include "wh_kernels.h"

namespace wh {

constexpr int LR_THREADS = 1024;
constexpr int KC = 9;       // candidates kept per row (beam + 1 <= 9)
constexpr int LU = 13;      // row loads in flight per thread per batch (13 x 1024 >= V / 4)

struct BlockRed {
  float v[16];
  int i[16];
};

__device__ __forceinline__ bool better(float a, int ia, float b, int ib) { return a > b || (a == b && ia < ib); }

__device__ float block_max(float x, BlockRed& sm) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  x = wave_max(x);
  __syncthreads();
  if (lane == 0) sm.v[wv] = x;
  __syncthreads();
  float r = sm.v[0];
  for (int k = 1; k < (int)(blockDim.x >> 6); ++k) r = fmaxf(r, sm.v[k]);
  return r;
}
__device__ float block_sum(float x, BlockRed& sm) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  x = wave_sum(x);
  __syncthreads();
  if (lane == 0) sm.v[wv] = x;
  __syncthreads();
  float r = 0.f;
  for (int k = 0; k < (int)(blockDim.x >> 6); ++k) r += sm.v[k];
  return r;
}
// (value desc, index asc) argbest across the block
__device__ void block_argbest(float& v, int& idx, BlockRed& sm) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(idx, o, 64);
    if (better(ov, oi, v, idx)) { v = ov; idx = oi; }
  }
  __syncthreads();
  if (lane == 0) { sm.v[wv] = v; sm.i[wv] = idx; }
  __syncthreads();
  v = sm.v[0];
  idx = sm.i[0];
  for (int k = 1; k < (int)(blockDim.x >> 6); ++k)
    if (better(sm.v[k], sm.i[k], v, idx)) { v = sm.v[k]; idx = sm.i[k]; }
}

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(LR_THREADS) void k_logit_rows(float* __restrict__ logits, int ldl, DecState s,
                                                           DecOpts o) {
  __shared__ BlockRed sm;
  __shared__ int info[8];
  const int r = blockIdx.x, w = r / s.G;
  const int tid = threadIdx.x;
  if (s.done[w]) return;
  const int len = s.len[w], sb = s.sample_begin[w];
  const int* hist = s.hist + (int64_t)r * s.hctx;
  const int V = o.V, tb = o.ts_begin;
  // last timestamp token of the sampled part (decoding.py:503-508): every lane checks
  // its positions, the block takes the largest (a backward scan by one lane would put
  // one memory latency per sampled token on every step)
  __shared__ int pmax_w[LR_THREADS / 64];
  {
    int pm = -1;
    for (int p = sb + tid; p < len; p += LR_THREADS)
      if (hist[p] >= tb) pm = p;
#pragma unroll
    for (int o2 = 32; o2 > 0; o2 >>= 1) pm = max(pm, __shfl_xor(pm, o2, 64));
    if ((tid & 63) == 0) pmax_w[tid >> 6] = pm;
  }
  __syncthreads();
  if (tid == 0) {
    const int nseq = len - sb;
    const int last_ts = nseq >= 1 && hist[len - 1] >= tb;
    const int penult_ts = nseq < 2 || hist[len - 2] >= tb;
    int pm = -1;
    for (int k = 0; k < LR_THREADS / 64; ++k) pm = max(pm, pmax_w[k]);
    info[0] = last_ts;
    info[1] = penult_ts;
    info[2] = pm >= 0 ? hist[pm] : -1;
    info[3] = (len == sb);
  }
  __syncthreads();
  const int last_ts = info[0], penult_ts = info[1], ts_last = info[2], first = info[3];
  // mask intervals [lo, hi)
  int mlo[4], mhi[4];
  int nm = 0;
  if (o.timestamps) {
    if (last_ts) {
      if (penult_ts) { mlo[nm] = tb; mhi[nm++] = V; }
      else { mlo[nm] = 0; mhi[nm++] = o.eot; }
    }
    if (ts_last >= 0) {
      mlo[nm] = tb;
      mhi[nm++] = (last_ts && !penult_ts) ? ts_last : ts_last + 1;
    }
    if (first) {
      mlo[nm] = 0; mhi[nm++] = tb;
      if (o.max_initial >= 0) { mlo[nm] = tb + o.max_initial + 1; mhi[nm++] = V; }
    }
  }
  float* row = logits + (int64_t)r * ldl;
  const bool sb_first = first && o.suppress_blank;
  // every pass reads the row in batches of LU loads per thread, all in flight before
  // the first use (a load-use chain per element would put one memory latency on each
  // of a thread's ~51 elements)
#define ROW_PASS(KILLTEXT, BODY)                                                  \
  for (int i0 = tid; i0 < V; i0 += LR_THREADS * LU) {                            \
    float vv[LU];                                                                \
    _Pragma("unroll") for (int u = 0; u < LU; ++u) {                             \
      const int i_ = i0 + LR_THREADS * u;                                        \
      vv[u] = i_ < V ? row[i_] : -INFINITY;                                      \
    }                                                                            \
    _Pragma("unroll") for (int u = 0; u < LU; ++u) {                             \
      const int i = i0 + LR_THREADS * u;                                         \
      if (i < V) {                                                               \
        const float x = ((KILLTEXT) && i < tb) ? -INFINITY : vv[u];              \
        BODY                                                                     \
      }                                                                          \
    }                                                                            \
  }
  // pass A: the filters, applied once in place (the logits are this step's scratch),
  // and the maxima the later passes need: m over all, and over text / timestamp ids
  // (log-probabilities are monotone in the logit, so their maxima follow exactly)
  float m = -INFINITY, mx_ts = -INFINITY, mx_tx = -INFINITY;
  for (int i0 = tid; i0 < V; i0 += LR_THREADS * LU) {
    float vv[LU];
    unsigned sw[LU];
#pragma unroll
    for (int u = 0; u < LU; ++u) {
      const int i = i0 + LR_THREADS * u;
      vv[u] = i < V ? row[i] : -INFINITY;
      sw[u] = (o.suppress && i < V) ? o.suppress[i >> 5] : 0u;
    }
#pragma unroll
    for (int u = 0; u < LU; ++u) {
      const int i = i0 + LR_THREADS * u;
      if (i >= V) continue;
      bool kill = (sw[u] >> (i & 31)) & 1u;
      if (sb_first)
        for (int b = 0; b < o.n_blank; ++b) kill |= (i == o.blank[b]);
      if (o.timestamps) {
        kill |= (i == o.no_ts);
        for (int q = 0; q < nm; ++q) kill |= (i >= mlo[q] && i < mhi[q]);
      }
      float x = vv[u];
      if (kill) {
        x = -INFINITY;
        row[i] = -INFINITY;
      }
      m = fmaxf(m, x);
      if (i >= tb) mx_ts = fmaxf(mx_ts, x);
      else mx_tx = fmaxf(mx_tx, x);
    }
  }
  m = block_max(m, sm);
  bool text_killed = false;
  if (o.timestamps) {
    // ApplyTimestampRules tail (decoding.py:522-531): if logsumexp(logprobs[tb:]) >
    // max(logprobs[:tb]) mask the text tokens
    mx_ts = block_max(mx_ts, sm);
    mx_tx = block_max(mx_tx, sm);
    float se = 0.f;
    ROW_PASS(false, se += __expf(x - m);)
    const float lS0 = logf(block_sum(se, sm));
    const float mts = mx_ts > -INFINITY ? (mx_ts - m) - lS0 : -INFINITY;
    const float mtx = mx_tx > -INFINITY ? (mx_tx - m) - lS0 : -INFINITY;
    float st = 0.f;
    if (mts > -INFINITY) {
      ROW_PASS(false, if (i >= tb) st += __expf(((x - m) - lS0) - mts);)
    }
    st = block_sum(st, sm);
    const float ts_lp = mts > -INFINITY ? mts + logf(st) : -INFINITY;
    text_killed = ts_lp > mtx;
    if (text_killed) m = mx_ts;  // the max of what is left
  }
  // final log_softmax normaliser, fused with the token choice (which does not need it)
  float se = 0.f;
  float* cv = s.cand_val + (int64_t)r * KC;
  int* ci = s.cand_idx + (int64_t)r * KC;
  if (!o.beam) {
    float bv = -INFINITY, bx = -INFINITY;
    int bi = 0x7fffffff;
    if (o.temperature > 0.f) {
      const unsigned long long key = splitmix64(s.seed[0] ^ ((unsigned long long)r << 40) ^ ((unsigned long long)len << 20));
      ROW_PASS(text_killed, {
        se += __expf(x - m);
        if (x != -INFINITY) {
          const unsigned long long z = splitmix64(key + (unsigned long long)i);
          const float u = ((float)(z >> 40) + 0.5f) * (1.0f / 16777216.0f);
          const float gsc = x / o.temperature - logf(-logf(u));
          if (better(gsc, i, bv, bi)) { bv = gsc; bi = i; bx = x; }
        }
      })
    } else {
      ROW_PASS(text_killed, {
        se += __expf(x - m);
        if (better(x, i, bv, bi)) { bv = x; bi = i; bx = x; }
      })
    }
    const float logS = logf(block_sum(se, sm));
    const int mine = bi;
    block_argbest(bv, bi, sm);
    // logprob of the chosen token: log_softmax(logits)[tok] (decoding.py:312-313)
    if (mine == bi && bi != 0x7fffffff) {
      ci[0] = bi;
      cv[0] = (bx - m) - logS;
    }
    return;
  }
  // beam: top-(G+1) of the log-probabilities (value desc, index asc).  The normaliser
  // pass also takes each lane's maximum; the need-th largest of those maxima is a
  // lower bound of the row's need-th largest value (need lanes hold an element at
  // least that large), so the insertion pass only touches elements >= it — without
  // the bound every wave would run the insertion chain on almost every element.
  const int need = s.G + 1;
  float tmax = -INFINITY;
  ROW_PASS(text_killed, {
    se += __expf(x - m);
    tmax = fmaxf(tmax, x);
  })
  float thr = -INFINITY;
  {
    float v = tmax;
    for (int q = 0; q < need; ++q) {
      float bv = v;
      int bi = tid;
      block_argbest(bv, bi, sm);
      thr = bv;
      if (bi == tid) v = -INFINITY;
    }
  }
  float lv[KC];
  int li[KC];
#pragma unroll
  for (int q = 0; q < KC; ++q) { lv[q] = -INFINITY; li[q] = 0x7fffffff; }
  float thr_v = -INFINITY;  // the thread's current need-th best (entry to beat)
  int thr_i = 0x7fffffff;
  ROW_PASS(text_killed, {
    float v = x;
    int vi = i;
    if (x >= thr && better(v, vi, thr_v, thr_i)) {
      _Pragma("unroll") for (int q = 0; q < KC; ++q) {
        if (q < need && better(v, vi, lv[q], li[q])) {
          const float tv = lv[q]; const int ti = li[q];
          lv[q] = v; li[q] = vi; v = tv; vi = ti;
        }
      }
      _Pragma("unroll") for (int q = 0; q < KC; ++q)
        if (q == need - 1) { thr_v = lv[q]; thr_i = li[q]; }
    }
  })
#undef ROW_PASS
  const float logS = logf(block_sum(se, sm));
  int head = 0;
  for (int q = 0; q < need; ++q) {
    float hv = -INFINITY;
    int hi = 0x7fffffff;
#pragma unroll
    for (int z = 0; z < KC; ++z)
      if (z == head) { hv = lv[z]; hi = li[z]; }
    float bv = hv;
    int bi = hi;
    block_argbest(bv, bi, sm);
    if (bi == hi && bi != 0x7fffffff) ++head;
    if (tid == 0) {
      cv[q] = (bv - m) - logS;
      ci[q] = bi;
    }
  }
}

// ------------------------------------------------------------ candidate merge of a window
// BeamSearchDecoder.update's bookkeeping (decoding.py:350-409) / GreedyDecoder.update
// (:304-320) for window w, by NT threads: a 256-thread k_merge workgroup, or the 512
// threads of the k_logit_part workgroup whose row combine completed the window (the merge
// folded into the selection launch, round 4).  SC1: the candidates were written in the
// same launch by other CUs (write-through stores, counted on s.lpw_cnt): read them with sc1
// loads (cdna_hip_programming.md §6 Guideline 16 R1).
constexpr int MG_MAXG = 8;
constexpr int MG_MAXCTX = 449;
struct MergeLds {
  int oh[MG_MAXG][MG_MAXCTX];
  int oa[MG_MAXG][MG_MAXCTX];
  int src[MG_MAXG], tok[MG_MAXG], fsrc[MG_MAXG * KC];
  float fsc[MG_MAXG * KC];
  int nfin_new;
  int etok[MG_MAXG];  // each row's input token for the next step
  float csc[MG_MAXG * KC];
  int csrc[MG_MAXG * KC], ctok[MG_MAXG * KC], rk[MG_MAXG * KC];
  // k_logit_part<..., WIN>: the window's row combines leave their candidates here ([G][KC])
  float wcv[MG_MAXG * KC];
  int wci[MG_MAXG * KC];
};
// the next step's input rows of window w (k_embed's arithmetic: x = E[tok] + P[pos] in
// fp32, pos = min(length - 1, pmax)); newtok[b]: row b's token at pos (passed from
// registers / LDS: that history word may have been written by another lane of this
// workgroup, and a plain reload could hit a stale L1 copy of its line)
template <typename T, int NT>
__device__ void merge_embed_rows(const MergeEmbed& em, int w, int G, int pos, const int* newtok, int tid) {
  const T* E = reinterpret_cast<const T*>(em.E);
  const T* P = reinterpret_cast<const T*>(em.P);
  const int n4 = em.n / 4, total = G * n4;
  constexpr int EB = 4;  // loads of EB items issued before their stores (one round trip per batch)
  for (int i0 = 0; i0 < total; i0 += NT * EB) {
    float4_t e[EB], p[EB];
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const int i = min(i0 + tid + NT * u, total - 1), b = i / n4, c = 4 * (i - b * n4);
      e[u] = load4f(E + (int64_t)newtok[b] * em.n + c);
      p[u] = load4f(P + (int64_t)pos * em.n + c);
    }
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const int i = i0 + tid + NT * u;
      if (i < total) {
        const int b = i / n4, c = 4 * (i - b * n4), r = w * G + b;
        const float4_t v = e[u] + p[u];
        store4(em.x + (int64_t)r * em.n + c, v[0], v[1], v[2], v[3]);
      }
    }
  }
  if (tid < G) em.row_pos[w * G + tid] = pos;
}
template <int NT>
__device__ void merge_embed(const MergeEmbed& em, int w, int G, int pos, const int* newtok, int tid) {
  if (em.half) merge_embed_rows<half_t, NT>(em, w, G, pos, newtok, tid);
  else merge_embed_rows<float, NT>(em, w, G, pos, newtok, tid);
}

// LDSC: the candidates are in L.wcv / L.wci (the window's row combines ran in this
// workgroup, k_logit_part<..., WIN>): no global round trip for them
template <int NT, bool SC1, bool LDSC = false>
__device__ __forceinline__ void merge_window(const DecState& s, const DecOpts& o, const MergeEmbed& em, int w, int tid, MergeLds& L) {
  static_assert(NT >= MG_MAXG * KC, "one lane per candidate");
  CT_MARK(CT_MERGE, 0);
  const int G = s.G, len = s.len[w], sb = s.sample_begin[w];
  int* hist = s.hist + (int64_t)w * G * s.hctx;
  int* anc = s.anc + (int64_t)w * G * s.ctx;
  if (s.done[w]) {
    // finished windows keep recomputing a valid row (as k_embed did): nothing of theirs
    // is written in this kernel, so the history words are read as they stand
    if (em.x) {
      const int pos = min(len - 1, em.pmax);
      if (tid < G) L.etok[tid] = hist[tid * s.hctx + pos];
      wh_lds_barrier();
      merge_embed<NT>(em, w, G, pos, L.etok, tid);
    }
    CT_END(CT_MERGE);
    return;
  }
  const auto rsv = wt_rsrc(s.cand_val), rsi = wt_rsrc(s.cand_idx);
  // candidate k of row b of the window
  auto cval = [&](int b, int k) -> float {
    if constexpr (LDSC) return L.wcv[b * KC + k];
    const int i = (w * G + b) * KC + k;
    if constexpr (SC1) return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsv, i * 4, 0, 16));
    else return s.cand_val[i];
  };
  auto cidx = [&](int b, int k) -> int {
    if constexpr (LDSC) return L.wci[b * KC + k];
    const int i = (w * G + b) * KC + k;
    if constexpr (SC1) return (int)__builtin_amdgcn_raw_buffer_load_b32(rsi, i * 4, 0, 16);
    else return s.cand_idx[i];
  };
  if (!o.beam) {
    if (tid < G) {
      const int r = w * G + tid;
      const int last = hist[tid * s.hctx + len - 1];
      int t = cidx(tid, 0);
      if (last == o.eot) t = o.eot;
      else s.sum_lp[r] += cval(tid, 0);
      hist[tid * s.hctx + len] = t;
      L.tok[tid] = t;
    }
    wh_lds_barrier();
    if (tid == 0) {
      int all_eot = 1;
      for (int b = 0; b < G; ++b) all_eot &= (L.tok[b] == o.eot);
      s.len[w] = len + 1;
      const int st = s.step[w] + 1;
      s.step[w] = st;
      if (all_eot || len + 1 > o.n_ctx || st >= o.sample_len) s.done[w] = 1;
    }
    if (em.x) {
      const int pos = min(len, em.pmax);  // the new length is len + 1
      if (tid < G) L.etok[tid] = pos == len ? L.tok[tid] : hist[tid * s.hctx + pos];  // pos < len: not written here
      wh_lds_barrier();
      merge_embed<NT>(em, w, G, pos, L.etok, tid);
    }
    CT_END(CT_MERGE);
    return;
  }
  // stage old histories / ancestry and gather the candidates in ONE round trip: every
  // load of the staging (unrolled, clamped addresses) and of the candidates is issued
  // before the first LDS write.  Candidates in insertion order: beam-major, top-k order
  // (decoding.py:366-373); at the first update all beams are identical: dict keys
  // collapse onto beam 0's candidates with the source of the last duplicate (G-1).
  const bool first = (len == sb);
  const int nbeams = first ? 1 : G;
  const int nc = nbeams * (G + 1);
  constexpr int MU = (MG_MAXG * MG_MAXCTX + NT - 1) / NT;
  const int nst = G * len;
  int hv[MU], av[MU];
#pragma unroll
  for (int u = 0; u < MU; ++u) {
    const int i = min(tid + NT * u, max(nst - 1, 0)), b = i / len, p = i - b * len;
    hv[u] = hist[b * s.hctx + p];
    av[u] = anc[b * s.ctx + min(p, s.ctx - 1)];
  }
  float cs = 0.f;
  int ct = 0;
  const bool cl = tid < nc;  // nc <= MG_MAXG * KC = 72 <= NT
  if (cl) {
    const int b = tid / (G + 1), k = tid - b * (G + 1), r = w * G + b;
    cs = s.sum_lp[r] + cval(b, k);
    ct = cidx(b, k);
  }
#pragma unroll
  for (int u = 0; u < MU; ++u) {
    const int i = tid + NT * u;
    if (i < nst) {
      const int b = i / len, p = i - b * len;
      L.oh[b][p] = hv[u];
      int a = (p < s.ctx) ? av[u] : 0;
      if (p == len - 1 && p >= sb) a = b;  // this step's KV of beam b was written in slot b
      L.oa[b][p] = a;
    }
  }
  if (cl) {
    L.csc[tid] = cs;
    L.ctok[tid] = ct;
    L.csrc[tid] = first ? (G - 1) : tid / (G + 1);
  }
  wh_lds_barrier();
  CT_MARK(CT_MERGE, 1);  // histories, ancestry and candidates staged
  // stable descending sort by rank (ties keep insertion order), then the walk of
  // decoding.py:375-386 in closed form: the candidate at rank q is taken iff fewer
  // than G non-EOT candidates rank above it; a non-EOT one becomes beam
  // #(non-EOT above), an EOT one finished sequence #(EOT above).  One lane per
  // candidate, no serial loop.
  auto take = [&](int c0, int ne, int ee, float sc, int tk, int sr) {
    if (ne < G) {
      if (tk == o.eot) {
        L.fsc[ee] = sc;
        L.fsrc[ee] = sr;
        atomicAdd(&L.nfin_new, 1);
      } else {
        L.src[ne] = sr;
        L.tok[ne] = tk;
        s.sum_lp[w * G + ne] = sc;
      }
    }
  };
  if (tid == 0) L.nfin_new = 0;
  if (nc <= 64) {
    // one wave, one candidate per lane: the other lanes' scores / ranks / tokens come from
    // registers (v_readlane with a uniform lane index), not from ~2 x nc dependent LDS
    // broadcast reads and a barrier between the two passes (merge 4.7 -> ~1 us of the
    // single-window tail, profiles/r05/chain_trace_w1.txt).  Same ranks, same walk.
    if (tid < 64) {
      const bool live = tid < nc;
      const float sc = live ? L.csc[tid] : 0.f;
      const int tk = live ? L.ctok[tid] : 0, sr = live ? L.csrc[tid] : 0;
      int q = 0;
      for (int c = 0; c < nc; ++c) {
        const float scc = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, sc), c));
        q += (scc > sc) || (scc == sc && c < tid);
      }
      int ne = 0, ee = 0;  // non-EOT / EOT candidates ranked above
      for (int c = 0; c < nc; ++c) {
        const int qc = __builtin_amdgcn_readlane(q, c), tc = __builtin_amdgcn_readlane(tk, c);
        if (qc < q) {
          if (tc == o.eot) ++ee;
          else ++ne;
        }
      }
      if (live) take(tid, ne, ee, sc, tk, sr);
    }
  } else {
    for (int c0 = tid; c0 < nc; c0 += NT) {
      const float sc = L.csc[c0];
      int q = 0;
      for (int c = 0; c < nc; ++c) q += (L.csc[c] > sc) || (L.csc[c] == sc && c < c0);
      L.rk[c0] = q;
    }
    wh_lds_barrier();
    for (int c0 = tid; c0 < nc; c0 += NT) {
      const int q = L.rk[c0];
      int ne = 0, ee = 0;  // non-EOT / EOT candidates ranked above
      for (int c = 0; c < nc; ++c)
        if (L.rk[c] < q) {
          if (L.ctok[c] == o.eot) ++ee;
          else ++ne;
        }
      take(c0, ne, ee, L.csc[c0], L.ctok[c0], L.csrc[c0]);
    }
  }
  wh_lds_barrier();
  CT_MARK(CT_MERGE, 2);  // ranked and walked
  // new histories / ancestry
  for (int i = tid; i < G * (len + 1); i += NT) {
    const int j = i / (len + 1), p = i - j * (len + 1);
    hist[j * s.hctx + p] = (p < len) ? L.oh[L.src[j]][p] : L.tok[j];
    if (p < len && p < s.ctx) anc[j * s.ctx + p] = L.oa[L.src[j]][p];
  }
  // finished sequences (already in descending order)
  int fin0 = s.fin_n[w];
  const int nadd = min(L.nfin_new, max(0, s.maxc - fin0));
  for (int i = tid; i < nadd * (len + 1); i += NT) {
    const int f = i / (len + 1), p = i - f * (len + 1);
    s.fin_tok[((int64_t)w * s.maxc + fin0 + f) * s.hctx + p] = (p < len) ? L.oh[L.fsrc[f]][p] : o.eot;
  }
  if (tid < nadd) {
    s.fin_score[w * s.maxc + fin0 + tid] = L.fsc[tid];
    s.fin_len[w * s.maxc + fin0 + tid] = len + 1;
  }
  wh_lds_barrier();
  if (tid == 0) {
    const int fn = fin0 + nadd;
    s.fin_n[w] = fn;
    s.len[w] = len + 1;
    const int st = s.step[w] + 1;
    s.step[w] = st;
    if (fn >= s.maxc || len + 1 > o.n_ctx || st >= o.sample_len) s.done[w] = 1;
  }
  if (em.x) {
    // row j's new history is oh[src[j]][0, len) + tok[j]: its input token from LDS
    const int pos = min(len, em.pmax);
    if (tid < G) L.etok[tid] = pos == len ? L.tok[tid] : L.oh[L.src[tid]][pos];
    wh_lds_barrier();
    merge_embed<NT>(em, w, G, pos, L.etok, tid);
  }
  CT_END(CT_MERGE);
}

// ---------------------------------------------------------------- split selection
// The same selection with each row's vocabulary in NS slices, one 512-thread
// workgroup per (row, slice): slices 0..NS-2 split the text ids [0, ts_begin),
// the last one is the timestamp range [ts_begin, V) on its own, so the
// ApplyTimestampRules tail (decoding.py:522-531: logsumexp over timestamps vs the text
// maximum) and the masking of text it may decide are both per-slice facts the combine
// selects between.  k_logit_part applies the filters in place and writes, per slice:
// max, sum of exp(x - max), argbest, Gumbel best, top-(G+1); k_logit_combine (one wave
// per row) merges the kept slices.  Same choices as k_logit_rows; the normaliser is
// summed per slice (float rounding of the log-probabilities differs in the last bits).
constexpr int LP_THREADS = 512;
// WH_LP_OCC=1: cap k_logit_part at 80 VGPRs (6 waves per SIMD: 3 workgroups per CU);
// WH_LP_OCC=2 (probe build): at 64 (8 waves per SIMD: 4 workgroups per CU)
#if defined(WH_LP_OCC) && WH_LP_OCC == 2
#define WH_LP_ATTR __attribute__((amdgpu_waves_per_eu(8)))
#elif defined(WH_LP_OCC) && WH_LP_OCC
#define WH_LP_ATTR __attribute__((amdgpu_waves_per_eu(6, 8)))
#else
#define WH_LP_ATTR
#endif
// NS slices per row (NS - 1 text slices + the timestamp range) with EPT elements per lane:
// 32 slices (EPT 4: ceil(50365 / 31) = 1625 and 1501 <= 512 x 4) for few rows, where the
// per-workgroup latency is the cost (1 window: 29.9 -> 14.4 us); 8 slices (EPT 16) for
// many rows, where 32 x rows workgroups cost more than they hide (100 rows: 54 vs 62 us)

struct LPRec {
  float mx, se, bv, gv, gx;
  int bi, gi, pad;
  float tv[KC];
  int ti[KC];
  float tail[LP_REC - 8 - 2 * KC];  // records are LP_REC words apart in s.lpart
};
static_assert(sizeof(LPRec) == LP_REC * 4, "slice record stride");

__device__ __forceinline__ void lp_slice(int j, int ns, int tb, int V, int& lo, int& hi) {
  if (j == ns - 1) { lo = tb; hi = V; return; }
  lo = (int)((int64_t)tb * j / (ns - 1));
  hi = (int)((int64_t)tb * (j + 1) / (ns - 1));
}

// wave-level (value desc, index asc) argbest; every lane ends with the winner (a total
// order: the same winner for any pairing; permlane / DPP exchanges as wave_max, wh_common.h)
__device__ __forceinline__ void wave_argbest(float& v, int& idx) {
  {
    float a = v, b = v;
    int ia = idx, ib = idx;
    perm32_pair(a, b);
    perm32_pair(ia, ib);
    const bool t = (b > a) | ((b == a) & (ib < ia));  // better(b, a) without a branch: full EXEC below
    v = t ? b : a;
    idx = t ? ib : ia;
  }
  {
    float a = v, b = v;
    int ia = idx, ib = idx;
    perm16_pair(a, b);
    perm16_pair(ia, ib);
    const bool t = (b > a) | ((b == a) & (ib < ia));  // better(b, a) without a branch: full EXEC below
    v = t ? b : a;
    idx = t ? ib : ia;
  }
  auto step = [&](float ov, int oi) {
    const bool t = (ov > v) | ((ov == v) & (oi < idx));
    v = t ? ov : v;
    idx = t ? oi : idx;
  };
  step(dpp_f<DPP_ROR8>(v), dpp_i<DPP_ROR8>(idx));
  step(dpp_f<DPP_ROR4>(v), dpp_i<DPP_ROR4>(idx));
  step(dpp_f<DPP_ROR2>(v), dpp_i<DPP_ROR2>(idx));
  step(dpp_f<DPP_ROR1>(v), dpp_i<DPP_ROR1>(idx));
}

template <int NS, bool WT>
__device__ __forceinline__ void lp_combine(const LPRec* rec, int r, const DecState& s, const DecOpts& o, int lane,
                                           float* cv_out = nullptr, int* ci_out = nullptr);

// Two barriers per workgroup: (1) after the history scan (last sampled timestamp), (2)
// after every wave has reduced its own max, rescaled sum of exp and top-(G+1) list (or
// argbest / Gumbel best); wave 0 then merges the 8 wave results and writes the record.
// The slice's logits and suppress words are loaded first, before the history, so their
// round trip overlaps it.
//
// MERGE (with FUSED): the candidates of the row combine are stored write-through and counted
// on the window's counter (s.lpw_cnt); the combine completing the window tells its
// workgroup, whose 8 waves then run the window's candidate merge (k_merge folded in:
// merge_window<512, sc1 candidate loads>).  A finished window's rows are re-embedded by
// its first row's first slice.
//
// WIN (with MERGE, round 6): the slices count on their WINDOW's counter (G x NS arrivals)
// instead of their row's; the slice completing the window runs every row's combine in its
// workgroup (wave b: row b's NS records, sc1 loads, then lp_combine into LDS) and the merge
// reads those candidates from LDS — the row-level arrival, the candidates' write-through
// stores, their drain and their sc1 reload leave the chain.  Same records, same combine
// arithmetic, same merge: bit-identical selections.
template <int NS, int LP_EPT, bool FUSED, bool MERGE = false, bool WIN = false>
__global__ __launch_bounds__(LP_THREADS) WH_LP_ATTR void k_logit_part(float* __restrict__ logits, int ldl, DecState s,
                                                           DecOpts o, MergeEmbed em) {
  CT_MARK(CT_LOGIT, 0);
  static_assert(FUSED || !MERGE, "the merge rides on the fused combine");
  static_assert(!WIN || MERGE, "window arrival: the merge runs in this launch");
  // (WIN: the launcher checks that G x NS records fit the merge's history / ancestry
  // staging, which they alias: lp_win_fits)
  constexpr int NWV = LP_THREADS / 64;
  __shared__ __attribute__((aligned(16))) char mlds_raw[MERGE ? sizeof(MergeLds) : 4];
  MergeLds& mlds = *reinterpret_cast<MergeLds*>(mlds_raw);
  __shared__ int s_go;
  __shared__ int pm_w[NWV], pt_w[NWV];
  __shared__ float wmx[NWV], wse[NWV], wv_v[NWV][KC], wg_v[NWV], wg_x[NWV];
  __shared__ int wv_i[NWV][KC], wg_i[NWV];
  const int r = blockIdx.x, j = blockIdx.y, w = r / s.G;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int V = o.V, tb = o.ts_begin;
  int lo, hi;
  lp_slice(j, NS, tb, V, lo, hi);
  float* row = logits + (int64_t)r * ldl;
  // 1. this slice's logits and suppress words (clamped addresses, masked below)
  float xv[LP_EPT];
  unsigned sw[LP_EPT];
#pragma unroll
  for (int u = 0; u < LP_EPT; ++u) {
    const int ic = min(lo + tid + LP_THREADS * u, hi - 1);
    xv[u] = row[ic];
    sw[u] = o.suppress ? o.suppress[ic >> 5] : 0u;
  }
  // the whole history row, one position per thread (hctx <= LP_THREADS, the launcher), in
  // the same round trip: its addresses do not wait for the window's len / sample_begin
  const int* hist = s.hist + (int64_t)r * s.hctx;
  const int hp = hist[min(tid, s.hctx - 1)];
  const int done = s.done[w], len = s.len[w], sb = s.sample_begin[w];
  if (done) {
    if constexpr (MERGE)
      if (j == 0 && r == w * s.G) merge_window<LP_THREADS, false>(s, o, em, w, tid, mlds);
    return;
  }
  // 2. history facts (decoding.py:503-508): the last timestamp token of the sampled
  // part [sb, len) and the last two tokens (through LDS, across the barrier)
  __shared__ int s_h12[2];
  if (tid == max(len - 1, 0)) s_h12[0] = hp;
  if (tid == max(len - 2, 0)) s_h12[1] = hp;
  int pm = (tid >= sb && tid < len && hp >= tb) ? tid : -1, pt = hp;
#pragma unroll
  for (int o2 = 32; o2 > 0; o2 >>= 1) {
    const int op = __shfl_xor(pm, o2, 64), ot = __shfl_xor(pt, o2, 64);
    if (op > pm) { pm = op; pt = ot; }
  }
  if (lane == 0) { pm_w[wv] = pm; pt_w[wv] = pt; }
  wh_lds_barrier();
  CT_MARK(CT_LOGIT_SLICE, 0);
  const int h1 = s_h12[0], h2 = s_h12[1];
  int PM = -1, PT = -1;
#pragma unroll
  for (int k = 0; k < NWV; ++k)
    if (pm_w[k] > PM) { PM = pm_w[k]; PT = pt_w[k]; }
  const int nseq = len - sb;
  const bool last_ts = nseq >= 1 && h1 >= tb, penult_ts = nseq < 2 || h2 >= tb, first = len == sb;
  const int ts_last = PM >= 0 ? PT : -1;
  // the timestamp rules as four fixed [lo, hi) masks (unused: empty), no_ts and the blank
  // tokens as four fixed ids (unused: -1): straight-line filter code per element
  int mlo[4] = {0, 0, 0, 0}, mhi[4] = {0, 0, 0, 0};
  int kid[5] = {-1, -1, -1, -1, -1};
  if (o.timestamps) {
    if (last_ts) {
      if (penult_ts) { mlo[0] = tb; mhi[0] = V; }
      else { mlo[0] = 0; mhi[0] = o.eot; }
    }
    if (ts_last >= 0) {
      mlo[1] = tb;
      mhi[1] = (last_ts && !penult_ts) ? ts_last : ts_last + 1;
    }
    if (first) {
      mlo[2] = 0; mhi[2] = tb;
      if (o.max_initial >= 0) { mlo[3] = tb + o.max_initial + 1; mhi[3] = V; }
    }
    kid[4] = o.no_ts;
  }
  if (first && o.suppress_blank)
#pragma unroll
    for (int b = 0; b < 4; ++b)
      if (b < o.n_blank) kid[b] = o.blank[b];
  // 3. filters in place, then this wave's max and sum of exp (online rescale across waves)
  float mx = -INFINITY;
#pragma unroll
  for (int u = 0; u < LP_EPT; ++u) {
    const int i = lo + tid + LP_THREADS * u;
    if (i >= hi) { xv[u] = -INFINITY; continue; }
    bool kill = (sw[u] >> (i & 31)) & 1u;
#pragma unroll
    for (int b = 0; b < 5; ++b) kill |= i == kid[b];
#pragma unroll
    for (int q = 0; q < 4; ++q) kill |= (i >= mlo[q] && i < mhi[q]);
    if (kill) {
      xv[u] = -INFINITY;
      row[i] = -INFINITY;
    }
    mx = fmaxf(mx, xv[u]);
  }
  mx = wave_max(mx);
  float se = 0.f;
  if (mx > -INFINITY) {
#pragma unroll
    for (int u = 0; u < LP_EPT; ++u) se += __expf(xv[u] - mx);  // masked entries: exp(-inf) = 0
  }
  se = wave_sum(se);
  if (lane == 0) { wmx[wv] = mx; wse[wv] = se; }
  // this slice's record, stored write-through (sc1) by lane 0 of wave 0 (NS <= LP_SLICES)
  const auto rrs = wt_rsrc(s.lpart + (int64_t)r * LP_SLICES * LP_REC);
  const int rec_off = j * LP_REC * 4;
  auto wt_rec = [&](int off, float v) { wt_store1(rrs, off, v); };
  // FUSED: the row's last slice to finish merges all NS records (the k_logit_combine
  // launch folded in; cdna_hip_programming.md §6 Guideline 16 R1, as k_xattn_seg): the
  // record's sc1 stores drained (vmcnt(0)), a relaxed agent add on the row's counter; the
  // wave drawing NS - 1 re-arms it and reads the NS records with sc1 loads into LDS
  __shared__ __attribute__((aligned(16))) float recs[FUSED ? NS * LP_REC : 4];
  // (wave 0) returns true when this combine completed the window (MERGE)
  auto arrive_and_combine = [&]() -> bool {
    CT_MARK(CT_LOGIT_SLICE, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int ticket = 0;
    if (lane == 0) ticket = __hip_atomic_fetch_add(s.lp_cnt + r, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ticket = __shfl(ticket, 0, 64);
    CT_MARK(CT_LOGIT_SLICE, 3);
    if (ticket != NS - 1) return false;
    CT_MARK(CT_LOGIT, 1);  // this workgroup combines its row
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the add
    if (lane == 0) __hip_atomic_store(s.lp_cnt + r, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    constexpr int N4 = NS * LP_REC / 4, PER = (N4 + 63) / 64;
    float4_t v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k)
      v[k] = __builtin_bit_cast(float4_t, __builtin_amdgcn_raw_buffer_load_b128(rrs, min(lane + 64 * k, N4 - 1) * 16, 0, 16));
#pragma unroll
    for (int k = 0; k < PER; ++k)
      if (lane + 64 * k < N4) reinterpret_cast<float4_t*>(recs)[lane + 64 * k] = v[k];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: its own LDS writes, no barrier
    lp_combine<NS, MERGE>(reinterpret_cast<const LPRec*>(recs), r, s, o, lane);
    if constexpr (!MERGE) return false;
    // the row's candidates (sc1 stores) drained, then the window's arrival
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int wt = 0;
    if (lane == 0) wt = __hip_atomic_fetch_add(s.lpw_cnt + w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    wt = __shfl(wt, 0, 64);
    if (wt != s.G - 1) return false;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the add
    if (lane == 0) __hip_atomic_store(s.lpw_cnt + w, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  };
  // WIN: the window's arrival (every slice of every row of window w); true for the last
  auto arrive_window = [&]() -> bool {
    CT_MARK(CT_LOGIT_SLICE, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int ticket = 0;
    if (lane == 0) ticket = __hip_atomic_fetch_add(s.lpw_cnt + w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ticket = __shfl(ticket, 0, 64);
    CT_MARK(CT_LOGIT_SLICE, 3);
    if (ticket != s.G * NS - 1) return false;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the add
    if (lane == 0) __hip_atomic_store(s.lpw_cnt + w, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  };
  // MERGE: wave 0 tells the workgroup whether it merges the window
  auto finish = [&](bool go) {
    if constexpr (MERGE) {
      if (wv == 0 && lane == 0) s_go = go;
      wh_lds_barrier();
      if (s_go) {
        if constexpr (WIN) {
          CT_MARK(CT_LOGIT, 1);  // this workgroup combines the window's rows
          // the rows' records alias the merge's history / ancestry staging (written after
          // the barrier below); wave b combines row b (G <= MG_MAXG <= 8 waves)
          float* wrec = reinterpret_cast<float*>(&mlds.oh[0][0]);
          if (wv < s.G) {
            const int rr = w * s.G + wv;
            const auto rs = wt_rsrc(s.lpart + (int64_t)rr * LP_SLICES * LP_REC);
            constexpr int N4 = NS * LP_REC / 4, PER = (N4 + 63) / 64;
            float4_t v[PER];
#pragma unroll
            for (int k = 0; k < PER; ++k)
              v[k] = __builtin_bit_cast(float4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, min(lane + 64 * k, N4 - 1) * 16, 0, 16));
            float* mine = wrec + wv * NS * LP_REC;
#pragma unroll
            for (int k = 0; k < PER; ++k)
              if (lane + 64 * k < N4) reinterpret_cast<float4_t*>(mine)[lane + 64 * k] = v[k];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: its own LDS writes
            lp_combine<NS, false>(reinterpret_cast<const LPRec*>(mine), rr, s, o, lane, mlds.wcv + wv * KC,
                                  mlds.wci + wv * KC);
          }
          wh_lds_barrier();
          CT_MARK(CT_LOGIT, 2);  // this workgroup merges its window
          merge_window<LP_THREADS, false, true>(s, o, em, w, tid, mlds);
        } else {
          CT_MARK(CT_LOGIT, 2);  // this workgroup merges its window
          merge_window<LP_THREADS, true>(s, o, em, w, tid, mlds);
        }
      }
    }
  };
  const int need = s.G + 1;
  if (!o.beam) {
    float bv = -INFINITY, gv = -INFINITY, gx = -INFINITY;
    int bi = 0x7fffffff, gi = 0x7fffffff;
    const unsigned long long key = splitmix64(s.seed[0] ^ ((unsigned long long)r << 40) ^ ((unsigned long long)len << 20));
#pragma unroll
    for (int u = 0; u < LP_EPT; ++u) {
      const int i = lo + tid + LP_THREADS * u;
      if (i >= hi) continue;
      const float x = xv[u];
      if (better(x, i, bv, bi)) { bv = x; bi = i; }
      if (o.temperature > 0.f && x != -INFINITY) {
        const unsigned long long z = splitmix64(key + (unsigned long long)i);
        const float uu = ((float)(z >> 40) + 0.5f) * (1.0f / 16777216.0f);
        const float gsc = x / o.temperature - logf(-logf(uu));
        if (better(gsc, i, gv, gi)) { gv = gsc; gi = i; gx = x; }
      }
    }
    wave_argbest(bv, bi);
    const int mine = gi;
    const float myx = gx;
    wave_argbest(gv, gi);
    const unsigned long long own = __ballot(mine == gi && gi != 0x7fffffff);
    const float gxw = own ? __shfl(myx, __ffsll((long long)own) - 1, 64) : -INFINITY;
    if (lane == 0) { wv_v[wv][0] = bv; wv_i[wv][0] = bi; wg_v[wv] = gv; wg_i[wv] = gi; wg_x[wv] = gxw; }
  } else {
    // this wave's top-(G+1) by (value desc, index asc): `need` rounds of a wave-level
    // argbest over every lane's best element not yet taken (bit u of `taken`: element u
    // left the lane's candidates).  Same list as per-lane insertion lists merged head by
    // head (the round-2 form, whose swap chains compiled to ~5k register moves per wave).
    unsigned taken = 0u;
    for (int q = 0; q < need; ++q) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int u = 0; u < LP_EPT; ++u) {
        const int i = lo + tid + LP_THREADS * u;
        if (i < hi && !((taken >> u) & 1u) && better(xv[u], i, bv, bi)) { bv = xv[u]; bi = i; }
      }
      const int mine = bi;
      wave_argbest(bv, bi);
      if (mine == bi && bi != 0x7fffffff) taken |= 1u << ((bi - lo - tid) / LP_THREADS);
      if (lane == 0) { wv_v[wv][q] = bv; wv_i[wv][q] = bi; }
    }
  }
  wh_lds_barrier();
  CT_MARK(CT_LOGIT_SLICE, 1);
  if (!MERGE && wv != 0) return;
  bool go = false;
  if (wv == 0) {
    // 4. wave 0 merges the NWV wave results
    float MX = -INFINITY;
#pragma unroll
    for (int k = 0; k < NWV; ++k) MX = fmaxf(MX, wmx[k]);
    float SE = 0.f;
    if (MX > -INFINITY) {
#pragma unroll
      for (int k = 0; k < NWV; ++k)
        if (wmx[k] > -INFINITY) SE += wse[k] * __expf(wmx[k] - MX);
    }
    if (!o.beam) {
      float bv = lane < NWV ? wv_v[lane][0] : -INFINITY, gv = lane < NWV ? wg_v[lane] : -INFINITY;
      int bi = lane < NWV ? wv_i[lane][0] : 0x7fffffff, gi = lane < NWV ? wg_i[lane] : 0x7fffffff;
      const float myx = lane < NWV ? wg_x[lane] : -INFINITY;
      const int mine = gi;
      wave_argbest(bv, bi);
      wave_argbest(gv, gi);
      const unsigned long long own = __ballot(mine == gi && gi != 0x7fffffff);
      const float gx = own ? __shfl(myx, __ffsll((long long)own) - 1, 64) : -INFINITY;
      if (lane == 0) {
        wt_rec(rec_off + offsetof(LPRec, mx), MX); wt_rec(rec_off + offsetof(LPRec, se), SE);
        wt_rec(rec_off + offsetof(LPRec, bv), bv); wt_rec(rec_off + offsetof(LPRec, bi), __builtin_bit_cast(float, bi));
        wt_rec(rec_off + offsetof(LPRec, gv), gv); wt_rec(rec_off + offsetof(LPRec, gi), __builtin_bit_cast(float, gi));
        wt_rec(rec_off + offsetof(LPRec, gx), gi != 0x7fffffff ? gx : -INFINITY);
      }
      if constexpr (WIN) go = arrive_window();
      else if constexpr (FUSED) go = arrive_and_combine();
    } else {
      // beam: each lane holds up to two wave candidates (NWV * need <= 72), sorted within
      // the lane; `need` wave-level rounds take the best remaining head
      const int c0 = lane, c1 = lane + 64, nc = NWV * need;
      float a0 = -INFINITY, a1 = -INFINITY;
      int i0 = 0x7fffffff, i1 = 0x7fffffff;
      if (c0 < nc) { a0 = wv_v[c0 / need][c0 % need]; i0 = wv_i[c0 / need][c0 % need]; }
      if (c1 < nc) { a1 = wv_v[c1 / need][c1 % need]; i1 = wv_i[c1 / need][c1 % need]; }
      if (better(a1, i1, a0, i0)) {
        const float tv = a0; const int ti = i0;
        a0 = a1; i0 = i1; a1 = tv; i1 = ti;
      }
      for (int q = 0; q < need; ++q) {
        float bv = a0;
        int bi = i0;
        wave_argbest(bv, bi);
        if (bi == i0 && bi != 0x7fffffff) { a0 = a1; i0 = i1; a1 = -INFINITY; i1 = 0x7fffffff; }
        if (lane == 0) {
          wt_rec(rec_off + offsetof(LPRec, tv) + 4 * q, bv);
          wt_rec(rec_off + offsetof(LPRec, ti) + 4 * q, __builtin_bit_cast(float, bi));
        }
      }
      if (lane == 0) { wt_rec(rec_off + offsetof(LPRec, mx), MX); wt_rec(rec_off + offsetof(LPRec, se), SE); }
      if constexpr (WIN) go = arrive_window();
      else if constexpr (FUSED) go = arrive_and_combine();
    }
  }  // wave 0
  finish(go);
  CT_END(CT_LOGIT);
}

// the merge of a row's NS slice records (in LDS, `rec`) by one wave: the timestamp-rule
// selection between text and timestamps, the normaliser, then argbest / top-(G+1) with one
// slice per lane (decoding.py:522-531 and the candidate lists of 707-733)
// WT: the candidates are stored write-through (sc1), for the merge in the same launch
// cv_out / ci_out (WT false): where the row's candidates go instead of s.cand_val / cand_idx
template <int NS, bool WT>
__device__ __forceinline__ void lp_combine(const LPRec* rec, int r, const DecState& s, const DecOpts& o, int lane,
                                           float* cv_out, int* ci_out) {
  constexpr int TS = NS - 1;
  float m = -INFINITY;
  for (int j = 0; j < NS; ++j) m = fmaxf(m, rec[j].mx);
  bool text_killed = false;
  if (o.timestamps) {
    float st0 = 0.f, mx_tx = -INFINITY;
    for (int j = 0; j < NS; ++j)
      if (rec[j].mx > -INFINITY) st0 += rec[j].se * __expf(rec[j].mx - m);
    for (int j = 0; j < TS; ++j) mx_tx = fmaxf(mx_tx, rec[j].mx);
    const float lS0 = logf(st0), mx_ts = rec[TS].mx;
    const float mts = mx_ts > -INFINITY ? (mx_ts - m) - lS0 : -INFINITY;
    const float mtx = mx_tx > -INFINITY ? (mx_tx - m) - lS0 : -INFINITY;
    // sum over timestamps of exp(logprob - mts) = the timestamp slice's own sum
    const float ts_lp = mts > -INFINITY ? mts + logf(rec[TS].se) : -INFINITY;
    text_killed = ts_lp > mtx;
    if (text_killed) m = mx_ts;
  }
  const int j0 = text_killed ? TS : 0;
  float se = 0.f;
  for (int j = j0; j < NS; ++j)
    if (rec[j].mx > -INFINITY) se += rec[j].se * __expf(rec[j].mx - m);
  const float logS = logf(se);
  float* cv = cv_out ? cv_out : s.cand_val + (int64_t)r * KC;
  int* ci = ci_out ? ci_out : s.cand_idx + (int64_t)r * KC;
  // lane j holds slice j (NS <= 64): wave-level argbest rounds, the order of better()
  // (value desc, index asc) as in the slices themselves
  static_assert(NS <= 64 && NS <= LP_SLICES, "one lane per slice");
  const bool act = lane < NS && lane >= j0;
  if (!o.beam) {
    float bv = -INFINITY, bx = -INFINITY;
    int bi = 0x7fffffff;
    if (act) {
      if (o.temperature > 0.f) { bv = rec[lane].gv; bi = rec[lane].gi; bx = rec[lane].gx; }
      else { bv = rec[lane].bv; bi = rec[lane].bi; bx = bv; }
    }
    const int mine = bi;
    const float myx = bx;
    wave_argbest(bv, bi);
    const unsigned long long own = __ballot(mine == bi && bi != 0x7fffffff);
    const float wx = own ? __shfl(myx, __ffsll((long long)own) - 1, 64) : -INFINITY;
    if (lane == 0 && bi != 0x7fffffff) {
      if constexpr (WT) {
        wt_store1(wt_rsrc(ci), 0, __builtin_bit_cast(float, bi));
        wt_store1(wt_rsrc(cv), 0, (wx - m) - logS);
      } else {
        ci[0] = bi;
        cv[0] = (wx - m) - logS;
      }
    }
    return;
  }
  // beam: merge the kept slices' sorted top lists, one head per lane
  const int need = s.G + 1;
  int hd = 0;
  for (int q = 0; q < need; ++q) {
    float hv = -INFINITY;
    int hi = 0x7fffffff;
    if (act && hd < need) { hv = rec[lane].tv[hd]; hi = rec[lane].ti[hd]; }
    float bv = hv;
    int bi = hi;
    wave_argbest(bv, bi);
    if (bi == hi && bi != 0x7fffffff) ++hd;
    if (lane == 0) {
      if constexpr (WT) {
        wt_store1(wt_rsrc(cv), 4 * q, (bv - m) - logS);
        wt_store1(wt_rsrc(ci), 4 * q, __builtin_bit_cast(float, bi));
      } else {
        cv[q] = (bv - m) - logS;
        ci[q] = bi;
      }
    }
  }
}

template <int NS>
__global__ __launch_bounds__(64) void k_logit_combine(DecState s, DecOpts o) {
  const int r = blockIdx.x, w = r / s.G, lane = threadIdx.x;
  // the row's slice records -> LDS in one round trip, issued with the done flag's load
  // (the merge reads them serially; from global memory every read would be a dependent load)
  __shared__ __attribute__((aligned(16))) float recs[NS * LP_REC];
  {
    constexpr int N4 = NS * LP_REC / 4, PER = (N4 + 63) / 64;
    const float4_t* src = reinterpret_cast<const float4_t*>(s.lpart + (int64_t)r * LP_SLICES * LP_REC);
    float4_t* dst = reinterpret_cast<float4_t*>(recs);
    float4_t v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) v[k] = src[min(lane + 64 * k, N4 - 1)];
    if (s.done[w]) return;
#pragma unroll
    for (int k = 0; k < PER; ++k)
      if (lane + 64 * k < N4) dst[lane + 64 * k] = v[k];
  }
  __syncthreads();
  lp_combine<NS, false>(reinterpret_cast<const LPRec*>(recs), r, s, o, lane);
}

// the selection of one update; with `em` (launch_select_merge) the fused k_logit_part also
// runs each window's merge and this returns true
static bool select_rows(float* logits, int ldl, const DecState& s, const DecOpts& o, int nwin, hipStream_t st,
                        const MergeEmbed* em) {
  // the sliced selection (k_logit_part + k_logit_combine) unless WHISPER_HIP_LOGIT_SPLIT=0
  // (config 2, turbo one window: 0.380 -> 0.346 ms per token; config 3 unchanged)
  static const bool split = [] {
    const char* e = tune_env("WHISPER_HIP_LOGIT_SPLIT");
    return !(e && e[0] == '0');
  }();
  // the window's merge in the selection launch unless WHISPER_HIP_LP_MERGE=0 (tuning: k_merge
  // as its own launch)
  static const bool fold_merge = [] {
    const char* e = tune_env("WHISPER_HIP_LP_MERGE");
    return !(e && e[0] == '0');
  }();
  const int rows = nwin * s.G;
  const bool merge = em && fold_merge && s.lpw_cnt && s.G <= MG_MAXG;
  // the window-level arrival (k_logit_part<..., WIN>): tuning build only, WHISPER_HIP_LP_WIN=1.
  // Measured not faster (profiles/r06/ab_selection_window_arrival.txt: 100 rows 51.5 vs
  // 51.2 us, one turbo window 27.2 vs 28.5-28.9 us: the last slice's workgroup combining
  // every row after the last arrival costs what the row-then-window hand-off saved)
  static const bool win_on = [] {
    const char* e = tune_env("WHISPER_HIP_LP_WIN");
    return e && e[0] == '1';
  }();
  auto lp_win_fits = [&](int ns) {
    return win_on && (size_t)s.G * ns * LP_REC * 4 <= sizeof(MergeLds::oh) + sizeof(MergeLds::oa);
  };
  const bool sp = split && s.hctx <= LP_THREADS;  // k_logit_part: one history position per thread
  const MergeEmbed none;
  const MergeEmbed& e = em ? *em : none;
  // the records merged by the row's last slice (fused) unless WHISPER_HIP_LP_FUSED=0 (tuning:
  // k_logit_combine as its own launch)
  const char* fe = tune_env("WHISPER_HIP_LP_FUSED");
  const bool fused = !(fe && fe[0] == '0');
  // Every batch of >= 2 windows selects with 16 slices (15 text + timestamps, 8 elements
  // per lane): the per-slice normaliser sums, hence a row's log-probabilities to the last
  // bit, then do not depend on the batch size (batch invariance); at 100
  // rows 8 slices measured 3.5 us and 32 slices 10 us slower per step
  // (profiles/r03/step_tail_ab.txt).  One window keeps 32 slices (its latency path) —
  // the same window-count cut as the k_proj1 layers (wh_runtime.hip p1_active), so the
  // rule holds for greedy and small beams too.
  // Tuning: WHISPER_HIP_LP_NS=8 / 32 forces the other counts (A/B)
  const char* nse = tune_env("WHISPER_HIP_LP_NS");
  const int ns_force = nse ? atoi(nse) : 16;  // slices for >= 2 windows
  const bool one_win = nwin == 1;
  if (sp && fused && !one_win && ns_force == 16 && o.ts_begin > 0 &&
      (o.ts_begin + 14) / 15 <= LP_THREADS * 8 && o.V - o.ts_begin <= LP_THREADS * 8) {
    if (merge && lp_win_fits(16)) k_logit_part<16, 8, true, true, true><<<dim3(rows, 16), LP_THREADS, 0, st>>>(logits, ldl, s, o, e), wh_launched("k_logit_part<win>");
    else if (merge) k_logit_part<16, 8, true, true><<<dim3(rows, 16), LP_THREADS, 0, st>>>(logits, ldl, s, o, e), wh_launched("k_logit_part");
    else k_logit_part<16, 8, true><<<dim3(rows, 16), LP_THREADS, 0, st>>>(logits, ldl, s, o, e), wh_launched("k_logit_part");
    return merge;
  }
  if (sp && o.ts_begin > 0 && (one_win || ns_force == 32) && (o.ts_begin + 30) / 31 <= LP_THREADS * 4 &&
      o.V - o.ts_begin <= LP_THREADS * 4) {
    if (fused) {
      if (merge && lp_win_fits(32)) k_logit_part<32, 4, true, true, true><<<dim3(rows, 32), LP_THREADS, 0, st>>>(logits, ldl, s, o, e), wh_launched("k_logit_part<win>");
      else if (merge) k_logit_part<32, 4, true, true><<<dim3(rows, 32), LP_THREADS, 0, st>>>(logits, ldl, s, o, e), wh_launched("k_logit_part");
      else k_logit_part<32, 4, true><<<dim3(rows, 32), LP_THREADS, 0, st>>>(logits, ldl, s, o, e), wh_launched("k_logit_part");
      return merge;
    }
    k_logit_part<32, 4, false><<<dim3(rows, 32), LP_THREADS, 0, st>>>(logits, ldl, s, o, e), wh_launched("k_logit_part");
    k_logit_combine<32><<<rows, 64, 0, st>>>(s, o), wh_launched("k_logit_combine");
    return false;
  }
  if (sp && o.ts_begin > 0 && (o.ts_begin + 6) / 7 <= LP_THREADS * 16 && o.V - o.ts_begin <= LP_THREADS * 16) {
    if (fused) {
      if (merge) k_logit_part<8, 16, true, true><<<dim3(rows, 8), LP_THREADS, 0, st>>>(logits, ldl, s, o, e), wh_launched("k_logit_part");
      else k_logit_part<8, 16, true><<<dim3(rows, 8), LP_THREADS, 0, st>>>(logits, ldl, s, o, e), wh_launched("k_logit_part");
      return merge;
    }
    k_logit_part<8, 16, false><<<dim3(rows, 8), LP_THREADS, 0, st>>>(logits, ldl, s, o, e), wh_launched("k_logit_part");
    k_logit_combine<8><<<rows, 64, 0, st>>>(s, o), wh_launched("k_logit_combine");
    return false;
  }
  k_logit_rows<<<nwin * s.G, LR_THREADS, 0, st>>>(logits, ldl, s, o), wh_launched("k_logit_rows");
  return false;
}

void launch_logit_rows(float* logits, int ldl, const DecState& s, const DecOpts& o, int nwin, hipStream_t st) {
  select_rows(logits, ldl, s, o, nwin, st, nullptr);
}

// ------------------------------------------------------------ merge (one workgroup per window)
__global__ __launch_bounds__(256) void k_merge(DecState s, DecOpts o, MergeEmbed em) {
  __shared__ MergeLds L;
  merge_window<256, false>(s, o, em, blockIdx.x, threadIdx.x, L);
}

void launch_merge(const DecState& s, const DecOpts& o, int nwin, hipStream_t st, const MergeEmbed& em) {
  k_merge<<<nwin, 256, 0, st>>>(s, o, em), wh_launched("k_merge");
}

void launch_select_merge(float* logits, int ldl, const DecState& s, const DecOpts& o, int nwin, hipStream_t st,
                         const MergeEmbed& em) {
  if (!select_rows(logits, ldl, s, o, nwin, st, &em)) launch_merge(s, o, nwin, st, em);
}

// ------------------------------------------------------------ vocabulary + selection + merge, one window
// The single-window step's whole token tail in ONE launch (round 4): k_vocab1's balanced
// vocabulary projection (256 workgroups, 12-13 16-column tiles each, the final LayerNorm in
// the prologue, a ring of D weight tiles in flight), then, per workgroup and row, the
// selection of k_logit_part over the workgroup's own ~200 columns — filters, max, sum of
// exp, top-(G+1) / argbest / Gumbel best — as a record per (row, part): part 0 the text
// ids < timestamp_begin, part 1 the timestamp ids (only the workgroup straddling the
// boundary has both), stored write-through.  The workgroup whose arrival completes the
// launch merges every row's records (decoding.py:522-531: the timestamp-vs-text rule from
// the combined normaliser and the two maxima; top-(G+1) across the records' sorted lists)
// and then runs the window's candidate merge (merge_window) — no logits round trip, no
// selection or merge launch.  Same choices as the sliced selection; the normaliser is
// summed over other partitions, so log-probabilities can differ in the last bits.
struct LpMasks {
  int mlo[4], mhi[4], kid[5];
};
// the filters of decoding.py:450-532 for one row as four [lo, hi) masks and five ids
__device__ __forceinline__ LpMasks lp_masks(const DecOpts& o, bool last_ts, bool penult_ts, bool first, int ts_last) {
  const int tb = o.ts_begin, V = o.V;
  LpMasks f;
#pragma unroll
  for (int q = 0; q < 4; ++q) f.mlo[q] = f.mhi[q] = 0;
#pragma unroll
  for (int q = 0; q < 5; ++q) f.kid[q] = -1;
  if (o.timestamps) {
    if (last_ts) {
      if (penult_ts) { f.mlo[0] = tb; f.mhi[0] = V; }
      else { f.mlo[0] = 0; f.mhi[0] = o.eot; }
    }
    if (ts_last >= 0) {
      f.mlo[1] = tb;
      f.mhi[1] = (last_ts && !penult_ts) ? ts_last : ts_last + 1;
    }
    if (first) {
      f.mlo[2] = 0; f.mhi[2] = tb;
      if (o.max_initial >= 0) { f.mlo[3] = tb + o.max_initial + 1; f.mhi[3] = V; }
    }
    f.kid[4] = o.no_ts;
  }
  if (first && o.suppress_blank)
#pragma unroll
    for (int b = 0; b < 4; ++b)
      if (b < o.n_blank) f.kid[b] = o.blank[b];
  return f;
}

struct VsArgs {
  DecState s;
  DecOpts o;
  MergeEmbed em;
  float* rec;  // [VS_ROWS][2 parts][VS_NB workgroups][VS_REC]
  int* cnt;    // the launch's arrival counter (zero between launches)
};
constexpr int VS_ROWS = 8, VS_NB = 256, VS_REC = 32, VS_TMAX = 13;
// record words: 0 mx, 1 se, 2 bv, 3 bi, 4 gv, 5 gi, 6 gx, 8.. tv[KC], 20.. ti[KC] (the first
// 8 of each list 16-byte aligned: two b128 loads)
constexpr int VS_TV = 8, VS_TI = 20;
static_assert(VS_TI + KC <= VS_REC, "record size");

#if WH_TUNING
// tuning build: per-workgroup wall-clock marks of the last k_vocab_sel launch (100 MHz),
// read by wh_tune_vs_trace (profiles/vocab_sel_trace.py)
constexpr int VS_MARKS = 10;
__device__ unsigned long long g_vs_trace[VS_NB][VS_MARKS];
#define VS_MARK(k)                                                                          \
  do {                                                                                      \
    if (threadIdx.x == 0) g_vs_trace[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();    \
  } while (0)
#else
#define VS_MARK(k) \
  do {             \
  } while (0)
#endif

template <int D>
__global__ __launch_bounds__(512) void k_vocab_sel(GemmArgs a, VsArgs v) {
  constexpr int KW = 8, SW = 5, K = KW * SW * 32, TMAX = VS_TMAX;  // K 1280 (launcher)
  constexpr int XROW = K * 2 + 16;
  extern __shared__ __attribute__((aligned(16))) char vs_lds[];
  float4_t* red = reinterpret_cast<float4_t*>(vs_lds + 8 * XROW);  // [TMAX tiles][KW][64]
  float* lg = reinterpret_cast<float*>(vs_lds);                   // [8][TMAX * 16] logits (X dead)
  MergeLds& mlds = *reinterpret_cast<MergeLds*>(vs_lds + 8 * XROW);  // red's space, after the records
  __shared__ LpMasks fm[VS_ROWS];
  __shared__ int s_last;
  const DecState& s = v.s;
  const DecOpts& o = v.o;
  VS_MARK(0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const int nt = (a.N + 15) / 16, b = blockIdx.x, nb = gridDim.x;
  const int t0 = range_split(b, nt, nb), t1 = range_split(b + 1, nt, nb), ntl = t1 - t0;
  const half_t* W = reinterpret_cast<const half_t*>(a.W);
  const int kb = wave * SW * 32;
  // 1. the window's state first (its loads retire first), then the LayerNorm operands,
  // then the first D - 1 weight tiles
  const int done = s.done[0], len = s.len[0], sb = s.sample_begin[0];
  auto load_tile = [&](int tl, Frag<half_t> (&wf)[SW]) {
    const int tile = t0 + min(tl, ntl - 1);
    const half_t* wp = W + (int64_t)min(tile * 16 + r, a.N - 1) * K + kb + 8 * g;
#pragma unroll
    for (int s2 = 0; s2 < SW; ++s2) frag_load_stream(wf[s2], wp + s2 * 32);
  };
  constexpr int CPLM = 5;
  const int row = wave;
  const bool lnrow = row < a.M;
  float4_t xv[CPLM], gv[CPLM], bv[CPLM];
  if (lnrow) {
    const float* xr = a.xf32 + (int64_t)row * K;
#pragma unroll
    for (int i = 0; i < CPLM; ++i) {
      const int c = lane + 64 * i;
      xv[i] = load4f(xr + 4 * c);
      gv[i] = load4f(a.ln_g + 4 * c);
      bv[i] = load4f(a.ln_b + 4 * c);
    }
  }
  Frag<half_t> wf[D][SW];
#pragma unroll
  for (int t = 0; t < D - 1; ++t) load_tile(t, wf[t]);
  VS_MARK(1);
  // 2. this row's history facts (decoding.py:503-508), in flight during the projection
  const int tb = o.ts_begin, V = o.V;
  const int c0 = t0 * 16, c1 = min(t1 * 16, a.N);
  int hv[7], h1 = 0, h2 = 0;
  unsigned sw[4] = {0u, 0u, 0u, 0u};  // suppress words of this lane's columns
  unsigned long long seed = 0;
  if (lnrow) {
    const int* hist = s.hist + (int64_t)row * s.hctx;
#pragma unroll
    for (int i = 0; i < 7; ++i) hv[i] = hist[min(sb + lane + 64 * i, max(len - 1, 0))];
    h1 = hist[max(len - 1, 0)];
    h2 = hist[max(len - 2, 0)];
    if (o.suppress)
#pragma unroll
      for (int u = 0; u < 4; ++u) sw[u] = o.suppress[min(c0 + lane + 64 * u, c1 - 1) >> 5];
    seed = s.seed[0];
  }
  // 3. the final LayerNorm (k_vocab1's prologue) and the projection
  {
    half_t* dst = reinterpret_cast<half_t*>(vs_lds + row * XROW);
    if (!lnrow) {
      for (int c = lane; c < K / 4; c += 64) store4(dst + 4 * c, 0.f, 0.f, 0.f, 0.f);
    } else {
      float sm = 0.f;
#pragma unroll
      for (int i = 0; i < CPLM; ++i) sm += xv[i][0] + xv[i][1] + xv[i][2] + xv[i][3];
      const float mean = wave_sum(sm) / (float)K;
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < CPLM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = xv[i][e] - mean;
          q += d * d;
        }
      const float rstd = rsqrtf(wave_sum(q) / (float)K + a.ln_eps);
#pragma unroll
      for (int i = 0; i < CPLM; ++i) {
        const float4_t x4 = xv[i];
        store4(dst + 4 * (lane + 64 * i), (x4[0] - mean) * rstd * gv[i][0] + bv[i][0],
               (x4[1] - mean) * rstd * gv[i][1] + bv[i][1], (x4[2] - mean) * rstd * gv[i][2] + bv[i][2],
               (x4[3] - mean) * rstd * gv[i][3] + bv[i][3]);
      }
    }
  }
  __syncthreads();
  Frag<half_t> xf[SW];
#pragma unroll
  for (int s2 = 0; s2 < SW; ++s2)
    frag_load(xf[s2], reinterpret_cast<const half_t*>(vs_lds + min(r, 7) * XROW) + kb + s2 * 32 + 8 * g);
#pragma unroll
  for (int t = 0; t < TMAX; ++t) {
    if (t + D - 1 < TMAX) load_tile(t + D - 1, wf[(t + D - 1) % D]);
    float4_t acc = (float4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < SW; ++s2) mfma_step(acc, wf[t % D][s2], xf[s2]);
    if (t < ntl) red[(t * KW + wave) * 64 + lane] = acc;
  }
  VS_MARK(2);
  // a finished window (the decode's last no-op steps): no selection; its rows are
  // re-embedded (merge_window).  Checked only now, so that nothing of the projection's
  // load stream waits on the window state.
  if (done) {
    if (b == 0) {
      __syncthreads();  // every wave's X fragments are read: the merge scratch may overlap
      merge_window<512, false>(s, o, v.em, 0, tid, mlds);
    }
    return;
  }
  // the row's masks (its history loads have long landed)
  if (lnrow) {
    int pm = -1, pt = -1;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      const int p = sb + lane + 64 * i;
      if (p < len && hv[i] >= tb) { pm = p; pt = hv[i]; }
    }
#pragma unroll
    for (int o2 = 32; o2 > 0; o2 >>= 1) {
      const int op = __shfl_xor(pm, o2, 64), ot = __shfl_xor(pt, o2, 64);
      if (op > pm) { pm = op; pt = ot; }
    }
    const int nseq = len - sb;
    const bool last_ts = nseq >= 1 && h1 >= tb, penult_ts = nseq < 2 || h2 >= tb, first = len == sb;
    const LpMasks f = lp_masks(o, last_ts, penult_ts, first, pm >= 0 ? pt : -1);
    if (lane == 0) fm[row] = f;
  }
  __syncthreads();
  // 4. the logits of this workgroup's columns: the 8 eighths in wave order (k_vocab1)
  constexpr int LGW = TMAX * 16;
  for (int i = tid; i < ntl * 64; i += 512) {
    const int tl = i >> 6, ln = i & 63, rr = ln & 15;
    float4_t x4 = red[(tl * KW) * 64 + ln];
#pragma unroll
    for (int w2 = 1; w2 < KW; ++w2) x4 += red[(tl * KW + w2) * 64 + ln];
    if (rr < a.M) *reinterpret_cast<float4_t*>(lg + rr * LGW + tl * 16 + 4 * (ln >> 4)) = x4;
  }
  __syncthreads();
  VS_MARK(3);
  // 5. one wave per row: a record per part of this workgroup's columns
  const int need = s.G + 1;
  if (lnrow) {
    const LpMasks f = fm[row];
    const unsigned long long key =
        splitmix64(seed ^ ((unsigned long long)row << 40) ^ ((unsigned long long)len << 20));
#pragma unroll
    for (int part = 0; part < 2; ++part) {
      const int lo = part ? max(c0, tb) : c0, hi = part ? c1 : min(c1, tb);
      if (lo >= hi) continue;
      const auto rs = wt_rsrc(v.rec + ((int64_t)(row * 2 + part) * VS_NB + b) * VS_REC);
      float x[4];
      float mx = -INFINITY;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = c0 + lane + 64 * u;
        x[u] = -INFINITY;
        if (i >= lo && i < hi) {
          bool kill = (sw[u] >> (i & 31)) & 1u;
#pragma unroll
          for (int q = 0; q < 5; ++q) kill |= i == f.kid[q];
#pragma unroll
          for (int q = 0; q < 4; ++q) kill |= (i >= f.mlo[q] && i < f.mhi[q]);
          if (!kill) x[u] = lg[row * LGW + lane + 64 * u];
        }
        mx = fmaxf(mx, x[u]);
      }
      mx = wave_max(mx);
      float se = 0.f;
      if (mx > -INFINITY) {
#pragma unroll
        for (int u = 0; u < 4; ++u) se += __expf(x[u] - mx);
      }
      se = wave_sum(se);
      if (lane == 0) { wt_store1(rs, 0, mx); wt_store1(rs, 4, se); }
      if (!o.beam) {
        float bvv = -INFINITY, gvv = -INFINITY, gx = -INFINITY;
        int bi = 0x7fffffff, gi = 0x7fffffff;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i = c0 + lane + 64 * u;
          if (i < lo || i >= hi) continue;
          if (better(x[u], i, bvv, bi)) { bvv = x[u]; bi = i; }
          if (o.temperature > 0.f && x[u] != -INFINITY) {
            const unsigned long long z = splitmix64(key + (unsigned long long)i);
            const float uu = ((float)(z >> 40) + 0.5f) * (1.0f / 16777216.0f);
            const float gsc = x[u] / o.temperature - logf(-logf(uu));
            if (better(gsc, i, gvv, gi)) { gvv = gsc; gi = i; gx = x[u]; }
          }
        }
        wave_argbest(bvv, bi);
        const int mine = gi;
        const float myx = gx;
        wave_argbest(gvv, gi);
        const unsigned long long own = __ballot(mine == gi && gi != 0x7fffffff);
        const float gxw = own ? __shfl(myx, __ffsll((long long)own) - 1, 64) : -INFINITY;
        if (lane == 0) {
          wt_store1(rs, 8, bvv); wt_store1(rs, 12, __builtin_bit_cast(float, bi));
          wt_store1(rs, 16, gvv); wt_store1(rs, 20, __builtin_bit_cast(float, gi));
          wt_store1(rs, 24, gi != 0x7fffffff ? gxw : -INFINITY);
        }
      } else {
        unsigned taken = 0u;
        for (int q = 0; q < need; ++q) {
          float bvv = -INFINITY;
          int bi = 0x7fffffff;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int i = c0 + lane + 64 * u;
            if (i >= lo && i < hi && !((taken >> u) & 1u) && better(x[u], i, bvv, bi)) { bvv = x[u]; bi = i; }
          }
          const int mine = bi;
          wave_argbest(bvv, bi);
          if (mine == bi && bi != 0x7fffffff) taken |= 1u << ((bi - c0 - lane) / 64);
          if (lane == 0) {
            wt_store1(rs, 4 * (VS_TV + q), bvv);
            wt_store1(rs, 4 * (VS_TI + q), __builtin_bit_cast(float, bi));
          }
        }
      }
    }
  }
  // 6. arrival: every storing wave drains its records, one agent add per workgroup
  VS_MARK(4);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  VS_MARK(5);
  if (tid == 0) s_last = __hip_atomic_fetch_add(v.cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nb - 1;
  __syncthreads();
  VS_MARK(6);
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // no instruction: keeps the loads below the add
  if (tid == 0) __hip_atomic_store(v.cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // 7. the combine, one wave per row: text records of the workgroups with columns below
  // timestamp_begin (lane j: workgroups j, j + 64, ...), timestamp records of those above
  if (lnrow) {
    auto col0 = [&](int wb) { return range_split(wb, nt, nb) * 16; };
    auto col1 = [&](int wb) { return min(range_split(wb + 1, nt, nb) * 16, a.N); };
    const auto rsr = wt_rsrc(v.rec);
    auto ld = [&](int part, int wb, int word) -> float {
      return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                           rsr, (((row * 2 + part) * VS_NB + wb) * VS_REC + word) * 4, 0, 16));
    };
    // the first workgroup with timestamp columns (<= 64 of them: launcher)
    int bts = nb;
    for (int bb = lane; bb < nb; bb += 64)
      if (col1(bb) > tb) bts = min(bts, bb);
#pragma unroll
    for (int o2 = 32; o2 > 0; o2 >>= 1) bts = min(bts, __shfl_xor(bts, o2, 64));
    // record k of this lane: k < 4 text (workgroup lane + 64 k), k == 4 timestamps
    // (workgroup bts + lane); every word the combine reads is loaded here, in one round trip
    constexpr int NR = 5;
    auto rwb = [&](int k) { return k < 4 ? lane + 64 * k : bts + lane; };
    auto ld4 = [&](int part, int wb, int word) -> float4_t {
      return __builtin_bit_cast(float4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                              rsr, (((row * 2 + part) * VS_NB + wb) * VS_REC + word) * 4, 0, 16));
    };
    bool val[NR];
    float rmx[NR], rse[NR];
    float4_t w0[NR], w1[NR], tq0[NR], tq1[NR], iq0[NR], iq1[NR];
    float tv8[NR], ti8[NR];
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const int wb = rwb(k), part = k == 4;
      val[k] = wb < nb && (part ? col1(wb) > tb && col0(wb) < a.N : col0(wb) < min(tb, a.N));
      const int wc = val[k] ? wb : 0;
      w0[k] = ld4(part, wc, 0);
      if (o.beam) {
        tq0[k] = ld4(part, wc, VS_TV);
        tq1[k] = ld4(part, wc, VS_TV + 4);
        iq0[k] = ld4(part, wc, VS_TI);
        iq1[k] = ld4(part, wc, VS_TI + 4);
        tv8[k] = ld(part, wc, VS_TV + 8);
        ti8[k] = ld(part, wc, VS_TI + 8);
      } else {
        w1[k] = ld4(part, wc, 4);
      }
    }
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      rmx[k] = val[k] ? w0[k][0] : -INFINITY;
      rse[k] = w0[k][1];
    }
    float m = -INFINITY, mtx = -INFINITY, mts = -INFINITY;
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      m = fmaxf(m, rmx[k]);
      if (k < 4) mtx = fmaxf(mtx, rmx[k]);
      else mts = fmaxf(mts, rmx[k]);
    }
    m = wave_max(m);
    mtx = wave_max(mtx);
    mts = wave_max(mts);
    bool text_killed = false;
    if (o.timestamps) {
      float st0 = 0.f, sts = 0.f;
#pragma unroll
      for (int k = 0; k < NR; ++k)
        if (rmx[k] > -INFINITY) {
          st0 += rse[k] * __expf(rmx[k] - m);
          if (k == 4) sts += rse[k] * __expf(rmx[k] - mts);
        }
      st0 = wave_sum(st0);
      sts = wave_sum(sts);
      const float lS0 = logf(st0);
      const float lts = mts > -INFINITY ? (mts - m) - lS0 : -INFINITY;
      const float ltx = mtx > -INFINITY ? (mtx - m) - lS0 : -INFINITY;
      const float ts_lp = lts > -INFINITY ? lts + logf(sts) : -INFINITY;
      text_killed = ts_lp > ltx;
      if (text_killed) m = mts;
    }
    bool kept[NR];
#pragma unroll
    for (int k = 0; k < NR; ++k) kept[k] = val[k] && (!text_killed || k == 4);
    float se = 0.f;
#pragma unroll
    for (int k = 0; k < NR; ++k)
      if (kept[k] && rmx[k] > -INFINITY) se += rse[k] * __expf(rmx[k] - m);
    const float logS = logf(wave_sum(se));
    const auto rcv = wt_rsrc(s.cand_val + (int64_t)row * KC), rci = wt_rsrc(s.cand_idx + (int64_t)row * KC);
    if (!o.beam) {
      const bool samp = o.temperature > 0.f;
      float bvv = -INFINITY, bx = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        if (!kept[k]) continue;
        const float cv = samp ? w1[k][0] : w0[k][2];
        const int ci = __builtin_bit_cast(int, samp ? w1[k][1] : w0[k][3]);
        const float cx = samp ? w1[k][2] : cv;
        if (better(cv, ci, bvv, bi)) { bvv = cv; bi = ci; bx = cx; }
      }
      const int mine = bi;
      const float myx = bx;
      wave_argbest(bvv, bi);
      const unsigned long long own = __ballot(mine == bi && bi != 0x7fffffff);
      const float wx = own ? __shfl(myx, __ffsll((long long)own) - 1, 64) : -INFINITY;
      if (lane == 0 && bi != 0x7fffffff) {
        wt_store1(rci, 0, __builtin_bit_cast(float, bi));
        wt_store1(rcv, 0, (wx - m) - logS);
      }
    } else {
      // each lane's kept records' sorted lists; `need` rounds take the best head
      float tv[NR][KC];
      int ti[NR][KC];
#pragma unroll
      for (int k = 0; k < NR; ++k) {
#pragma unroll
        for (int q = 0; q < KC; ++q) {
          const float x = q < 4 ? tq0[k][q] : q < 8 ? tq1[k][q - 4] : tv8[k];
          const float xi = q < 4 ? iq0[k][q] : q < 8 ? iq1[k][q - 4] : ti8[k];
          const bool ok = kept[k] && q < need;
          tv[k][q] = ok ? x : -INFINITY;
          ti[k][q] = ok ? __builtin_bit_cast(int, xi) : 0x7fffffff;
        }
      }
      int hd[NR] = {0, 0, 0, 0, 0};
      for (int q = 0; q < need; ++q) {
        float hv2 = -INFINITY;
        int hi2 = 0x7fffffff, hk = -1;
#pragma unroll
        for (int k = 0; k < NR; ++k) {
          float cv = -INFINITY;
          int ci = 0x7fffffff;
#pragma unroll
          for (int qq = 0; qq < KC; ++qq)
            if (qq == hd[k]) { cv = tv[k][qq]; ci = ti[k][qq]; }
          if (hd[k] < need && better(cv, ci, hv2, hi2)) { hv2 = cv; hi2 = ci; hk = k; }
        }
        float bvv = hv2;
        int bi = hi2;
        wave_argbest(bvv, bi);
        if (bi == hi2 && bi != 0x7fffffff && hk >= 0) {
#pragma unroll
          for (int k = 0; k < NR; ++k)
            if (k == hk) ++hd[k];
        }
        if (lane == 0) {
          wt_store1(rcv, 4 * q, (bvv - m) - logS);
          wt_store1(rci, 4 * q, __builtin_bit_cast(float, bi));
        }
      }
    }
  }
  // 8. the window's candidate merge, with the candidates just written (sc1 loads)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  VS_MARK(7);
  merge_window<512, true>(s, o, v.em, 0, tid, mlds);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  VS_MARK(8);
}

#if WH_TUNING
extern "C" int wh_tune_vs_trace(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vs_trace), sizeof(g_vs_trace)) == hipSuccess ? 0 : -1;
}
#endif

// one window's tail in one launch; -1 when the shape is not the single-window fp16 step
bool vocab_select_on() {
  static const bool on = [] {  // tuning build only: WHISPER_HIP_VOCAB_SEL=1
    const char* e = tune_env("WHISPER_HIP_VOCAB_SEL");
    return e && e[0] == '1';
  }();
  return on;
}

int launch_vocab_select(const GemmArgs& a, const DecState& s, const DecOpts& o, const MergeEmbed& em, float* rec,
                        int* cnt, hipStream_t st) {
  const int nt = (a.N + 15) / 16;
  if (!vocab_select_on() || !rec || !cnt || !a.xf32 || a.K != 1280 || a.bias || a.M < 1 || a.M > VS_ROWS || a.M != s.G ||
      s.G > MG_MAXG || nt > VS_NB * VS_TMAX || nt < VS_NB || o.ts_begin <= 0 || o.ts_begin > a.N || a.N != o.V ||
      a.N - o.ts_begin > 64 * 16 * (nt / VS_NB) - 16)  // <= 64 workgroups hold timestamp columns
    return -1;
  constexpr int D = 6;
  const int lds = 8 * (1280 * 2 + 16) + VS_TMAX * 8 * 64 * 16;
  static_assert(sizeof(MergeLds) <= VS_TMAX * 8 * 64 * 16, "merge scratch inside the reduction space");
  // (the dynamic size itself: the kernel's static LDS counts against the 160 KB too)
  static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_vocab_sel<D>),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
  if (!attr) return -5;
  VsArgs v;
  v.s = s; v.o = o; v.em = em; v.rec = rec; v.cnt = cnt;
  k_vocab_sel<D><<<VS_NB, 512, lds, st>>>(a, v), wh_launched("k_vocab_sel");
  return 0;
}

// ------------------------------------------------------------ per-step ABI state updates
// wh_step: row r of window w takes token tok[r] at position len[w] (the token the host's
// decoder.update chose, decoding.py:730); the step then embeds hist[len - 1].
__global__ __launch_bounds__(64) void k_append_tokens(DecState s, const int* __restrict__ tok) {
  const int w = blockIdx.x, b = threadIdx.x;
  const int len = s.len[w];
  if (b < s.G) {
    s.hist[((int64_t)w * s.G + b) * s.hctx + len] = tok[w * s.G + b];
    // the step writes this position's K/V into the row's own slot
    if (len < s.ctx) s.anc[((int64_t)w * s.G + b) * s.ctx + len] = b;
  }
  __syncthreads();
  if (b == 0) s.len[w] = len + 1;
}
void launch_append_tokens(const DecState& s, const int* tok, int nwin, hipStream_t st) {
  k_append_tokens<<<nwin, 64, 0, st>>>(s, tok), wh_launched("k_append_tokens");
}

// wh_reorder_kv (rearrange_kv_cache, decoding.py:189-204; rearrange_mkv coreml.mm:251-277):
// row j of window w continues row src[j]'s sequence.  The cache itself is not copied:
// row j's ancestry (which beam slot holds each cached position) and history become
// src[j]'s (k_append_tokens recorded each stepped position in its row's own slot).
__global__ __launch_bounds__(256) void k_reorder_rows(DecState s, const int* __restrict__ src) {
  __shared__ int oh[MG_MAXG][MG_MAXCTX];
  __shared__ int oa[MG_MAXG][MG_MAXCTX];
  const int w = blockIdx.x, tid = threadIdx.x, G = s.G;
  const int len = s.len[w];
  int* hist = s.hist + (int64_t)w * G * s.hctx;
  int* anc = s.anc + (int64_t)w * G * s.ctx;
  for (int i = tid; i < G * len; i += 256) {
    const int b = i / len, p = i - b * len;
    oh[b][p] = hist[b * s.hctx + p];
    oa[b][p] = (p < s.ctx) ? anc[b * s.ctx + p] : 0;
  }
  __syncthreads();
  for (int i = tid; i < G * len; i += 256) {
    const int j = i / len, p = i - j * len;
    const int sj = src[w * G + j] - w * G;
    hist[j * s.hctx + p] = oh[sj][p];
    if (p < s.ctx) anc[j * s.ctx + p] = oa[sj][p];
  }
}
void launch_reorder_rows(const DecState& s, const int* src, int nwin, hipStream_t st) {
  k_reorder_rows<<<nwin, 256, 0, st>>>(s, src), wh_launched("k_reorder_rows");
}

// ------------------------------------------------------------ no_speech prob (decoding.py:716-720)
__global__ __launch_bounds__(256) void k_no_speech(const float* logits, int ldl, int V, int ns, float* out) {
  __shared__ BlockRed sm;
  const float* row = logits + (int64_t)blockIdx.x * ldl;
  float m = -INFINITY;
  for (int i = threadIdx.x; i < V; i += 256) m = fmaxf(m, row[i]);
  m = block_max(m, sm);
  float se = 0.f;
  for (int i = threadIdx.x; i < V; i += 256) se += __expf(row[i] - m);
  se = block_sum(se, sm);
  if (threadIdx.x == 0) out[blockIdx.x] = __expf(row[ns] - m) / se;
}
void launch_no_speech(const float* logits, int ldl, int rows, int V, int ns, float* out, hipStream_t st) {
  if (rows > 0) k_no_speech<<<rows, 256, 0, st>>>(logits, ldl, V, ns, out), wh_launched("k_no_speech");
}

__global__ void k_broadcast_rows(const float* src, int ld_src, const int* src_rows, float* dst, int ld_dst, int G,
                                 int V) {
  const int r = blockIdx.x, w = r / G;
  const float* s = src + (int64_t)src_rows[w] * ld_src;
  float* d = dst + (int64_t)r * ld_dst;
  for (int i = threadIdx.x; i < V; i += 256) d[i] = s[i];
}
void launch_broadcast_rows(const float* src, int ld_src, const int* src_rows, float* dst, int ld_dst, int G, int nwin,
                           int V, hipStream_t st) {
  k_broadcast_rows<<<nwin * G, 256, 0, st>>>(src, ld_src, src_rows, dst, ld_dst, G, V), wh_launched("k_broadcast_rows");
}

}  // namespace wh

#if WH_TUNING
WH_CT_READER(decode)
#endif
