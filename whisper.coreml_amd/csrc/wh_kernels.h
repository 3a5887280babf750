// Kernel launch declarations for libwhisper_hip.
#pragma once
#include "wh_common.h"

namespace wh {

constexpr int TKP = 1536;  // cross-KV keys per (window, head) block: 1500 padded to whole 64-key tiles
// cross-V (V^T) is tile-major: xv_index (wh_common.h)

template <typename T>
void launch_layernorm(const float* x, T* y, const float* g, const float* b, int rows, int n, float eps,
                      const int* rows_in, hipStream_t st);
// Split-K slabs of the decoder-step projections (k_proj EPI_PARTIAL) are fp32, or fp16 in
// fp16 contexts (GemmArgs::slab_half): `part` then points at half_t
// elements and slab_half is 1.  Strides count elements.
// Round 6: an L2 prefetch ridden by a latency-bound launch for the NEXT launch of the same
// stream.  Workgroup b of the carrying launch runs on XCD b % 8 (round-robin dispatch, as
// xcd_remap assumes; speed only), and the workgroups on XCD x pull bytes [lo[x], hi[x]) x
// unit of `base` into that XCD's L2 by LDS-DMA into a scratch block (no registers; the
// carrying workgroup waits for them before it ends, so its LDS is never reallocated under
// a transfer).  Used for the step cross-attention's W_q head slices (k_xattn_seg<qproj>):
// read by 25 workgroups per XCD at once, they missed the L2 together and streamed from
// memory at ~4 TB/s (profiles/r06/xattn_trace_xqv.txt).
struct L2Prefetch {
  const char* base = nullptr;
  int64_t unit = 0;  // bytes per index (a W_q head slice: 64 rows x n)
  int lo[8] = {0, 0, 0, 0, 0, 0, 0, 0}, hi[8] = {0, 0, 0, 0, 0, 0, 0, 0};
};
template <typename T>
void launch_resid_ln(float* x, const float* part, int nsplit, int64_t part_stride, const float* bias, T* y,
                     const float* g, const float* b, int rows, int n, float eps, hipStream_t st, int slab_half = 0,
                     const L2Prefetch* pf = nullptr);
// the per-XCD head ranges of k_xattn_seg<qproj>'s workgroups for a batch (same grid and
// xcd_remap as launch_cross_attn): pf->lo / hi in heads; false when the grid is too small
// for the per-XCD runs (fewer than 16 workgroups)
bool xattn_l2_ranges(int nwin, int H, int max_rows, L2Prefetch* pf);
template <typename T>
void launch_attn_enc(const T* qkv, int ld, int ns, int H, int Tlen, int nwin, int64_t wsi, const T* vt, int tkp, T* out,
                     int64_t wso, hipStream_t st);
template <typename T>
void launch_self_attn(const T* q, int ldq, const T* kc, const T* vc, const int* rw, const int* rs, const int* rp,
                      const int* anc, int anc_beams, int nbeam, int H, int ctx, T* out, int ldo, int rows,
                      hipStream_t st);
template <typename T>
int launch_self_attn_qkv(const float* part, int nsplit, int64_t part_stride, const float* bqkv, int ns, T* kc, T* vc,
                          const int* rw, const int* rs, const int* rp, const int* anc, int anc_beams, int nbeam, int H,
                          int ctx, T* out, int ldo, int rows, hipStream_t st, int slab_half = 0);
template <typename T>
void launch_reduce_store(const float* part, int nsplit, int64_t part_stride, const float* bias, T* out, int ldo, int M,
                         int N, int gelu, hipStream_t st, int slab_half = 0);
// decoder-step query given as split-K slabs: q = bias + sum_z part[z*stride + row*ldq + c]
// (part == nullptr: q is a T matrix); needs <= 16 rows per window and z in {4, 8, 10}
// (cross_attn_q_slabs(z)).
struct XQPart {
  const float* part = nullptr;  // half_t elements when part_half
  int part_half = 0;
  int64_t stride = 0;
  int z = 0;
  const float* bias = nullptr;
  int max_rows = 0;  // rows per window when known (decoder step: the beam group)
  // step cross-attention records of pairs cut between workgroups, [pair][segment][XREC],
  // one arrival counter per (window, head) pair (zero between launches), and the pair
  // capacity of both; null = the first-pass kernel
  float* split_rec = nullptr;
  int* split_cnt = nullptr;
  int max_pairs = 0;
  // round 6: the query projected inside the step kernel (xattn_fused_q): q = qx qw^T + bias
  // with qx the LayerNorm'd rows [rows][n] and qw = W_q [n][n] (T); q / part unused
  const void* qx = nullptr;
  const void* qw = nullptr;
  const void* qwf = nullptr;  // W_q in fragment order (launch_wq_frag), read instead of qw when set
  // the single-window step (k_proj1 layers): qx is the fp32 residual rows and the kernel
  // computes their LayerNorm (ln_g, ln_b, ln_eps) itself — no cross-q k_proj1 launch
  const float* ln_g = nullptr;
  const float* ln_b = nullptr;
  float ln_eps = 1e-5f;
  // ... with the projection split over the pair's workgroups (k_xattn_seg QV 6): the partial
  // queries [pair][XQ1_P][4][64] float4 and per pair {arrivals, departures} (zero between launches)
  float* q_part = nullptr;
  int* q_cnt = nullptr;
};
// the shapes the in-kernel query projection serves: fp16, n = 1280 (large-v3, turbo), <= 8
// rows per window; the choice depends on the model and the beam group only, never on the
// window count (a window's step stays batch-invariant)
inline bool xattn_fused_q(int n, int rows_per_window, int elem_size) {
  return elem_size == 2 && n == 1280 && rows_per_window >= 1 && rows_per_window <= 8;
}
// W_q [n][n] (fp16) -> the in-kernel query projection's fragment order: 16-B chunk
// ((((h * 4 + c) * 2 + kh) * (n / 64) + s) * 64 + lane) holds row h * 64 + 16 c + (lane & 15),
// columns kh * n / 2 + 32 s + 8 (lane >> 4) .. + 7 (a wave's k-step s is 1 KB contiguous)
void launch_wq_frag(const void* w, void* f, int n, hipStream_t st);
// round-6 probe (tuning build): pull a layer's cross K / V blocks of nwin windows (slots from
// win_slot, slot_bytes each, a multiple of 32 KB) through the memory side; nwg one-wave workgroups
void launch_kv_pull(const void* ck, const void* cv, const int* win_slot, int nwin, int64_t slot_bytes, int nwg,
                    unsigned* sink, hipStream_t st);
constexpr int XREC = 16 * 64 + 32;  // floats per segment record: O[16][64], m[16], l[16]
// step cross-attention (k_xattn_seg): one softmax partial per 64-key tile, at most
// XS_NSP tiles per (window, head) pair (Tk <= 1536), at most XS_QP pairs per workgroup
constexpr int XS_NSP = 24;
constexpr int XQ1_P = 8;  // workgroups per pair of the split single-window query projection (k_xattn_seg QV 6)
constexpr int XS_QP = 4;
int xattn_seg_grid(int npair, int nsp, int smax);
inline bool cross_attn_q_slabs(int z) { return z == 4 || z == 8 || z == 10; }
template <typename T>
void launch_cross_attn(const T* q, int ldq, const T* ck, const T* cv, int Tk, int H, int nsplit, int nwin,
                       const int* win_row0, const int* win_nrows, const int* win_slot, int64_t win_stride, float* po,
                       float* pm, float* pl, T* out, int ldo, int rows, float* qk_out, const int* qk_map, int qk_rows,
                       hipStream_t st, XQPart xq = XQPart());
template <typename T>
void launch_embed(const T* E, const T* P, int n, const int* row_tok, int* row_pos, const int* hist,
                  const int* cur_len, int G, int hctx, int pmax, float* x, int rows, hipStream_t st);
template <typename T>
void launch_mel_windows(const float* mel, int64_t ld_mel, int n_mels, const int64_t* seeks, const int* segs, T* melT,
                        int64_t win_stride, int rows_alloc, int nwin, hipStream_t st);
template <typename T>
void launch_zero_rows(T* buf, int64_t ws, int n, int ra, int rb, int nwin, hipStream_t st);

void launch_mel(const float* audio, int64_t n_real, int64_t n_padded, int64_t frame0, int64_t count,
                const float* filters, int n_mels, float* mel, int64_t ld, unsigned* gmax, hipStream_t st);
void launch_mel_norm(float* mel, int64_t count, int64_t ld, int n_mels, const unsigned* gmax, const float* ovr,
                     hipStream_t st);

// ------------------------------------------------------------ decode state (device)
// Per window slot w (capacity nw) with G rows (beams / samples) each.
struct DecState {
  int* hist;         // [nw][G][hctx]   token history (initial tokens + sampled)
  int* anc;          // [nw][G][ctx]    KV slot of each position (beam reorder by indirection)
  int* len;          // [nw]            current token count
  int* sample_begin; // [nw]
  int* step;         // [nw]            updates done
  int* done;         // [nw]
  float* sum_lp;     // [nw][G]
  int* fin_n;        // [nw]
  float* fin_score;  // [nw][maxc]
  int* fin_len;      // [nw][maxc]
  int* fin_tok;      // [nw][maxc][hctx]
  float* cand_val;   // [nw*G][KC]
  int* cand_idx;     // [nw*G][KC]
  float* lpart;      // [nw*G][LP_SLICES][LP_REC] per-slice token-selection partials
  int* lp_cnt;       // [nw*G] slice arrival counters of k_logit_part (zero between launches)
  int* lpw_cnt;      // [nw] row arrival counters of the merging k_logit_part (zero between launches)
  unsigned long long* seed;  // [1] sampling seed (device memory: not part of a captured graph)
  int nw, G, ctx, hctx, maxc;
};

struct DecOpts {
  int V, eot, ts_begin, no_ts;       // vocabulary facts
  int blank[4], n_blank;             // SuppressBlank ids (tokenizer.encode(" ") + eot)
  const unsigned* suppress;          // bitmask [ceil(V/32)] or null
  int suppress_blank, timestamps;    // flags
  int max_initial;                   // max_initial_timestamp index or -1
  int beam;                          // 1 = beam search, 0 = greedy/sampling
  int sample_len;                    // max updates
  int n_ctx;                         // text context (448): stop when len > n_ctx
  float temperature;                 // > 0: Gumbel-max sampling (greedy decoder)
};

constexpr int LP_SLICES = 32;  // vocabulary slices per row: 31 text slices + [timestamp_begin, V)
constexpr int LP_REC = 32;    // words per slice record
void launch_logit_rows(float* logits, int ldl, const DecState& s, const DecOpts& o, int nwin, hipStream_t st);
// k_merge also writes the NEXT step's decoder input rows (the embedding of each row's
// newest token, k_embed's arithmetic) when em.x is set: the step graph then starts with
// the first layer instead of a separate k_embed launch (round 4)
struct MergeEmbed {
  const void* E = nullptr;  // token embedding [V][n] (T)
  const void* P = nullptr;  // positional embedding [ctx][n] (T)
  float* x = nullptr;       // decoder input rows [rows][n] (fp32)
  int* row_pos = nullptr;   // position of each row's input token
  int n = 0, pmax = 0, half = 0;
};
void launch_merge(const DecState& s, const DecOpts& o, int nwin, hipStream_t st, const MergeEmbed& em = MergeEmbed());
// the single-window step's whole token tail (vocabulary projection with the final
// LayerNorm, selection, merge) in one launch; -1 when the shape does not fit it
struct GemmArgs;
bool vocab_select_on();
int self_attn_grp_mode();
bool self_attn_pipe_on();
bool self_attn_kco_on();  // the coalesced-K self-attention passes (round 6)
int self_attn_kco_min();   // ... from this many cached keys on
int launch_vocab_select(const GemmArgs& a, const DecState& s, const DecOpts& o, const MergeEmbed& em, float* rec,
                        int* cnt, hipStream_t st);
constexpr size_t VS_REC_FLOATS = 8 * 2 * 256 * 32;  // k_vocab_sel records [rows][part][workgroup][32]
// token selection + candidate merge of one update: one k_logit_part launch whose last
// row combiner of each window runs the merge (round 4), or k_logit_* then k_merge
void launch_select_merge(float* logits, int ldl, const DecState& s, const DecOpts& o, int nwin, hipStream_t st,
                         const MergeEmbed& em);
// per-step ABI (wh_step / wh_reorder_kv): append host-chosen tokens, reorder rows
void launch_append_tokens(const DecState& s, const int* tok, int nwin, hipStream_t st);
void launch_reorder_rows(const DecState& s, const int* src, int nwin, hipStream_t st);
void launch_no_speech(const float* logits, int ldl, int rows, int V, int no_speech, float* out, hipStream_t st);
void launch_broadcast_rows(const float* src, int ld_src, const int* src_rows, float* dst, int ld_dst, int G, int nwin,
                           int V, hipStream_t st);

}  // namespace wh
