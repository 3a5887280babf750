// libwhisper_hip runtime: context, weights, buffers, stage drivers and the C ABI
// declared in include/whisper_hip.h.  The reference counterpart is the
// Objective-C++ CoreML runner coreml/coreml.mm:18-463 (process-global state, one
// model per process, void returns); here everything lives in a context object,
// every entry point returns a status, and all stage data stays in HBM.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>
#include <chrono>

#include "whisper_hip.h"
#include "wh_align.h"
#include "wh_gemm.h"
#include "wh_kernels.h"

using namespace wh;

static thread_local std::string g_err;
static thread_local std::string g_release_error;  // a failed release in the last context destroy
static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                                  \
  do {                                                                                                \
    hipError_t e_ = (expr);                                                                           \
    if (e_ != hipSuccess) return fail(-100, std::string(#expr) + ": " + hipGetErrorString(e_));       \
  } while (0)

// A launch error (or any HIP error left pending) surfaces at the next hipGetLastError():
// report it with the launch that raised it (tuning build: wh_launched checked every launch)
// or, in the shipped build, the last launch before the check (wh_common.h)
static int launch_status(const char* where) {
  const hipError_t e = hipGetLastError();
  std::string& first = wh_first_launch_error();
  if (e == hipSuccess && first.empty()) return 0;
  std::string msg = std::string(where) + ": ";
  if (!first.empty()) msg += first;
  else msg += std::string(hipGetErrorString(e)) + " (raised at or before the launch of " + wh_last_launch() + ")";
  first.clear();
  return fail(-100, msg);
}

static int enter(wh_ctx* ctx, const char* entry);

#define TRY(expr)                  \
  do {                             \
    int rc_ = (expr);              \
    if (rc_ != 0) return rc_;      \
  } while (0)

namespace {

constexpr int CTX = 448;          // text positions (decoder.py:243, decoding.py:173)
constexpr int HCTX = CTX + 1;     // history capacity (tokens.shape[-1] may reach n_ctx + 1)
constexpr int NSPLIT = 8;         // cross-attention key splits (1500 / 8 = 188 keys)
// encoder windows per pass (WHISPER_HIP_ENC_CHUNK overrides; activations scale with it)
static int enc_chunk() {
  static const int v = [] {
    const char* e = tune_env("WHISPER_HIP_ENC_CHUNK");
    const int c = e ? atoi(e) : 16;
    return c >= 1 && c <= 64 ? c : 16;
  }();
  return v;
}
constexpr int PRE_ROWS = 1024;    // min prefill rows per pass (the context sizes it to ~240 per window)
constexpr int MROWS = 3008;       // melT rows per window (1 pad + 3000 + slack for padded conv1 K)
constexpr int H1ROWS = 3002;      // conv1 output rows per window (zero rows 0 and 3001)
constexpr int KC = 9;
// 128 x 64 tiles of a single window's n-wide encoder GEMMs (1500 rows: 12 row tiles)
constexpr int EKZ_TILES(int n) { return 12 * (n / 64); }
constexpr int RSPLIT = 16;      // max split-K slabs of the residual projections (decode rows <= 128)

struct Arena {
  char* base = nullptr;
  size_t cap = 0, off = 0;
  void* take(size_t bytes) {
    off = (off + 255) & ~size_t(255);
    void* p = base + off;
    off += bytes;
    return off <= cap ? p : nullptr;
  }
};

template <typename T>
struct EncLayer {
  float *ln1_g, *ln1_b, *bqkv, *bo, *ln2_g, *ln2_b, *b1, *b2;
  T *wqkv, *wo, *w1, *w2;
};
template <typename T>
struct DecLayer {
  float *ln1_g, *ln1_b, *bqkv, *bo, *lnx_g, *lnx_b, *bqx, *box, *ln2_g, *ln2_b, *b1, *b2;
  T *wqkv, *wo, *wqx, *wox, *w1, *w2;
  // round 6: W_q in the in-kernel query projection's fragment order (xq_project: each wave's
  // 16 B-per-lane loads are 1 KB contiguous), fp16 contexts whose shape xattn_fused_q serves
  T* wqx_f = nullptr;
};

struct Timer {
  hipEvent_t a = nullptr, b = nullptr;
  void create() { hipEventCreate(&a); hipEventCreate(&b); }
  ~Timer() {
    if (a) hipEventDestroy(a);
    if (b) hipEventDestroy(b);
  }
};

}  // namespace

struct wh_ctx {
  virtual std::string step_kernels(int n_win, int group) const = 0;
  virtual ~wh_ctx() {}
  virtual int load(const std::string& name, const float* data, const int64_t* shape, int ndim) = 0;
  virtual int finalize() = 0;
  virtual int log_mel(const float* audio, int64_t n, int64_t pad, int n_mels, int normalize, int64_t* nf) = 0;
  virtual int log_mel_frames(const float* audio, int64_t n, int64_t pad, int n_mels, int64_t frame0, int64_t count,
                             int normalize, int64_t* total_frames) = 0;
  virtual int audio_upload(const float* audio, int64_t n) = 0;
  virtual int mel_max(float* g) = 0;
  virtual int mel_normalize(float g) = 0;
  virtual int mel_read(float* out, int64_t f0, int64_t nf) = 0;
  virtual int mel_write(const float* mel, int64_t nf) = 0;
  virtual int encode(int n_win, const int64_t* seeks, const int* segs) = 0;
  virtual int read_xa(int slot, float* out) = 0;
  virtual int read_ckv(int slot, int layer, float* k, float* v) = 0;
  virtual int decode_begin(int n_win, const wh_decode_opts* o, const int* init, const int* n_init, int max_init,
                           const int* sot_index, const int* slots) = 0;
  virtual int decode_steps(int max_steps, int* n_done) = 0;
  virtual int step_prefill(int n_win, int G, const int* init, const int* n_init, int max_init, const int* sot_index,
                           float* lg) = 0;
  virtual int step_tokens(const int* tok, const int* offsets, float* lg) = 0;
  virtual int reorder_kv(const int* src) = 0;
  virtual int decode_read(int slot, int* tokens, float* slp, int* len, int* fin_n, int* fin_tok, int* fin_len,
                          float* fin_score, float* nsp) = 0;
  virtual int prefill_logits(int slot, const int* tokens, int n, float* logits, const int* ah, int na, float* aqk) = 0;
  virtual int align(int slot, const int* tokens, int n, int n_sot, int num_frames, const int* ah, int na, int medfilt,
                    float* probs, int* path, int* plen) = 0;
  virtual int align_batch(int n_win, const int* slots, const int* tokens, const int* n_tokens, int n_sot,
                          const int* num_frames, const int* ah, int na, int medfilt, float* probs, int* paths,
                          int* plens) = 0;
  virtual int dtw(const float* x, int N, int M, int* path, int* plen) = 0;
  virtual int time_stage(int what, int iters, double* ms) = 0;
  // tuning builds only (wh_tune_share_weights): read the weights of another context of the
  // same dims and dtype instead of this one's (probes of two window groups, one weight copy)
  virtual int share_weights_from(wh_ctx* src) = 0;
  // weight sharing (tuning builds): the contexts reading this one's weights, and the
  // context this one reads from; wh_destroy refuses a context others still read from
  int sharers = 0;
  wh_ctx* shares_from = nullptr;
  std::vector<float> token_ms;  // per-token wall ms of each decode_steps chunk
  double stats[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int maxc = 5;
  int maxc_stride = 1;
  int device = 0;
};

namespace {

template <typename T>
struct Ctx : public wh_ctx {
  wh_dims d;
  int ns, nh, La, Ld, V, nm, K1p;
  int Wcap, Gcap;
  hipStream_t st = nullptr;
  Arena wa;  // weights
  Arena aa;  // activations / state
  void* wbase = nullptr;
  void* abase = nullptr;
  std::set<std::string> loaded;
  size_t expected = 0;
  bool finalized = false;

  // weights
  T *conv1_w, *conv2_w, *E, *Pdec, *ckv_w;
  float *conv1_b, *conv2_b, *pos_enc, *lnp_g, *lnp_b, *ln_g, *ln_b, *ckv_b;
  std::vector<EncLayer<T>> enc;
  std::vector<DecLayer<T>> dec;

  // mel
  float* d_audio = nullptr;
  size_t audio_cap = 0;
  float* d_mel = nullptr;
  size_t mel_cap = 0;
  int64_t mel_frames = 0;
  int64_t mel_f0 = 0;  // absolute index of the first stored frame
  std::vector<int64_t> h_seeks;
  int mel_nm = 0;
  unsigned* d_gmax = nullptr;
  float* d_gmax_f = nullptr;
  std::map<int, float*> d_filters;

  // encoder buffers
  T *melT, *h1, *xn_e, *qkv_e, *vt_e, *att_e, *hm_e, *xa, *ckv;
  float* x_e;
  int64_t* d_seeks;
  int* d_segs;
  // self KV per layer
  std::vector<T*> kc, vc;
  // decoder buffers
  int RD;
  int PRE = PRE_ROWS;
  float *x_d, *po, *pm, *pl, *logits, *logits2, *nsp, *part;
  T *xn_d, *q_d, *att_d, *hm_d;
  int *row_tok, *row_pos, *row_win, *row_slot, *win_row0, *win_nrows, *win_slot, *rows_in, *src_rows;
  int *st_row_win, *st_row_slot, *st_win_row0, *st_win_nrows, *st_win_slot;
  int* fp_anc = nullptr;
  static constexpr int P1_SLABS = 2048;  // k_proj1 split-K slabs: zs x 16-column tiles <= 16 x 80 at n = 1280
  float* p1_slab = nullptr;  // k_proj1 in-launch split-K slabs [zs][N/16][256]
  float* vs_rec = nullptr;   // k_vocab_sel records
  int* vs_cnt = nullptr;     // and its arrival counter (zero between launches)
  int* p1_cnt = nullptr;     // and arrival counters [4n/16] (zero between launches)
  // single-window encoder: the residual GEMMs' K halves (k_gemm_tile KZ = 2) meet through
  // these fp32 slabs (64 KB per 128 x 64 tile, 12 x n/64 tiles at 1500 rows) and
  // per-(tile, wave) arrival counters (zero between launches)
  float* ekz_slab = nullptr;
  int* ekz_cnt = nullptr;
  float* xs_rec = nullptr;   // step cross-attention segment records [pair][XS_NSP][XREC]
  float* x2_d = nullptr;     // k_proj1 path: second residual buffer (deferred residual ping-pong)
  int* xs_cnt = nullptr;     // and (window, head) arrival counters
  float* xq1_part = nullptr; // single-window split query projection: partials [head][8][4][64] float4
  int* xq1_cnt = nullptr;    // and {arrivals, departures} per head (zero between launches)

  // the step cross-attention's query / split arguments
  XQPart step_xq(int rows_per_window) const {
    XQPart xq;
    xq.max_rows = rows_per_window;
    xq.split_rec = xs_rec;
    xq.split_cnt = xs_cnt;
    xq.max_pairs = Wcap * nh;
    return xq;
  }
  int* qk_map;  // [Ld][nh]
  unsigned* suppress;
  DecState S;
  DecOpts O;
  int cur_nwin = 0, cur_G = 1;
  // graph cache
  hipGraph_t graph = nullptr;
  hipGraphExec_t gexec = nullptr;
  std::vector<char> graph_key;
  int* h_done = nullptr;
  hipEvent_t poll_ev[2] = {nullptr, nullptr};

  Timer tm;
  std::vector<hipEvent_t> proj_ev;  // time_stage(7) event pairs, empty otherwise
  int proj_ev_n = 0;

  int share_weights_from(wh_ctx* src_) override {
    auto* src = dynamic_cast<Ctx<T>*>(src_);
    if (!src || src->ns != ns || src->Ld != Ld || src->La != La || src->V != V || !src->finalized)
      return fail(-2, "share_weights: a finalized context of the same dims and dtype is needed");
    conv1_w = src->conv1_w; conv2_w = src->conv2_w; E = src->E; Pdec = src->Pdec; ckv_w = src->ckv_w;
    conv1_b = src->conv1_b; conv2_b = src->conv2_b; pos_enc = src->pos_enc; lnp_g = src->lnp_g; lnp_b = src->lnp_b;
    ln_g = src->ln_g; ln_b = src->ln_b; ckv_b = src->ckv_b;
    enc = src->enc;
    dec = src->dec;
    finalized = true;
    if (shares_from) --shares_from->sharers;
    shares_from = src;
    ++src->sharers;  // src's weight arena must outlive this context (wh_destroy checks)
    return 0;
  }

  // every release checked: the first failure is kept (release_error) and reported by
  // wh_destroy instead of staying pending for the next context's first call
  std::string release_error;
  void rel(hipError_t e, const char* what) {
    if (e != hipSuccess && release_error.empty()) release_error = std::string(what) + ": " + hipGetErrorString(e);
  }
  ~Ctx() override {
    if (st) rel(hipStreamSynchronize(st), "hipStreamSynchronize");
    if (gexec) rel(hipGraphExecDestroy(gexec), "hipGraphExecDestroy");
    if (graph) rel(hipGraphDestroy(graph), "hipGraphDestroy");
    if (st) rel(hipStreamDestroy(st), "hipStreamDestroy");
    if (pst) {  // the tuning build's KV pull stream (kv_pull_setup)
      rel(hipStreamSynchronize(pst), "hipStreamSynchronize(pull)");
      rel(hipStreamDestroy(pst), "hipStreamDestroy(pull)");
      for (auto& e : kv_ev) rel(hipEventDestroy(e), "hipEventDestroy(pull)");
      rel(hipFree(kv_sink), "hipFree(pull sink)");
    }
    if (wbase) rel(hipFree(wbase), "hipFree(weights)");
    if (abase) rel(hipFree(abase), "hipFree(activations)");
    if (d_audio) rel(hipFree(d_audio), "hipFree(audio)");
    if (d_mel) rel(hipFree(d_mel), "hipFree(mel)");
    for (auto& kv : d_filters) rel(hipFree(kv.second), "hipFree(mel filters)");
    if (d_gmax) rel(hipFree(d_gmax), "hipFree(mel max)");
    if (scratch) rel(hipFree(scratch), "hipFree(scratch)");
    if (h_done) rel(hipHostFree(h_done), "hipHostFree(done flags)");
    for (auto& e : poll_ev)
      if (e) rel(hipEventDestroy(e), "hipEventDestroy(poll)");
    (void)hipGetLastError();  // what failed above is in release_error, not left pending
    if (!release_error.empty()) g_release_error = release_error;
  }

  int init(int device_, const wh_dims& dims, int Wcap_, int Gcap_) {
    device = device_;
    d = dims;
    ns = d.n_text_state;
    nh = d.n_text_head;
    La = d.n_audio_layer;
    Ld = d.n_text_layer;
    V = d.n_vocab;
    nm = d.n_mels;
    if (d.n_audio_state != ns || d.n_audio_head != nh) return fail(-2, "audio/text state or head mismatch unsupported");
    if (ns != nh * 64) return fail(-2, "head dim must be 64 (decoder.py:62-64)");
    if (d.n_audio_ctx != 1500 || d.n_text_ctx != CTX) return fail(-2, "n_audio_ctx must be 1500, n_text_ctx 448");
    if (ns % 128 || ns > 2048) return fail(-2, "n_state must be a multiple of 128 and <= 2048");
    if (V > 57344) return fail(-2, "n_vocab too large");
    Wcap = Wcap_;
    Gcap = Gcap_;
    if (Wcap < 1 || Gcap < 1 || Gcap > 8) return fail(-2, "bad max_windows / max_group");
    const int kb = 128 / (int)sizeof(T);
    K1p = ((3 * nm + kb - 1) / kb) * kb;
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    tm.create();
    HIPCHK(hipHostMalloc((void**)&h_done, sizeof(int) * 2 * Wcap));  // two poll buffers
    for (auto& e : poll_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    // ---------------- weights
    const size_t n = ns;
    size_t wb = 0;
    auto add = [&](size_t elems, size_t esz) { wb += ((elems * esz + 255) & ~size_t(255)) + 256; };
    add(n * K1p, sizeof(T)); add(n, 4); add(n * 3 * n, sizeof(T)); add(n, 4); add(1500 * n, 4);
    for (int l = 0; l < La; ++l) {
      add(n, 4); add(n, 4); add(3 * n * n, sizeof(T)); add(3 * n, 4); add(n * n, sizeof(T)); add(n, 4);
      add(n, 4); add(n, 4); add(4 * n * n, sizeof(T)); add(4 * n, 4); add(4 * n * n, sizeof(T)); add(n, 4);
    }
    add(n, 4); add(n, 4);
    add((size_t)V * n, sizeof(T)); add(CTX * n, sizeof(T));
    for (int l = 0; l < Ld; ++l) {
      add(n, 4); add(n, 4); add(3 * n * n, sizeof(T)); add(3 * n, 4); add(n * n, sizeof(T)); add(n, 4);
      add(n, 4); add(n, 4); add(n * n, sizeof(T)); add(n, 4); add(n * n, sizeof(T)); add(n, 4);
      add(n, 4); add(n, 4); add(4 * n * n, sizeof(T)); add(4 * n, 4); add(4 * n * n, sizeof(T)); add(n, 4);
    }
    add(n, 4); add(n, 4);
    add(2 * Ld * n * n, sizeof(T)); add(2 * Ld * n, 4);
    const bool wq_frag = xattn_fused_q(n, 1, (int)sizeof(T));
    if (wq_frag)
      for (int l = 0; l < Ld; ++l) add(n * n, sizeof(T));
    HIPCHK(hipMalloc(&wbase, wb));
    HIPCHK(hipMemset(wbase, 0, wb));
    wa.base = (char*)wbase;
    wa.cap = wb;
    auto tk = [&](size_t elems) { return (T*)wa.take(elems * sizeof(T)); };
    auto fk = [&](size_t elems) { return (float*)wa.take(elems * 4); };
    conv1_w = tk(n * K1p); conv1_b = fk(n); conv2_w = tk(n * 3 * n); conv2_b = fk(n); pos_enc = fk(1500 * n);
    enc.resize(La);
    for (auto& e : enc) {
      e.ln1_g = fk(n); e.ln1_b = fk(n); e.wqkv = tk(3 * n * n); e.bqkv = fk(3 * n); e.wo = tk(n * n); e.bo = fk(n);
      e.ln2_g = fk(n); e.ln2_b = fk(n); e.w1 = tk(4 * n * n); e.b1 = fk(4 * n); e.w2 = tk(4 * n * n); e.b2 = fk(n);
    }
    lnp_g = fk(n); lnp_b = fk(n);
    E = tk((size_t)V * n); Pdec = tk(CTX * n);
    dec.resize(Ld);
    for (auto& e : dec) {
      e.ln1_g = fk(n); e.ln1_b = fk(n); e.wqkv = tk(3 * n * n); e.bqkv = fk(3 * n); e.wo = tk(n * n); e.bo = fk(n);
      e.lnx_g = fk(n); e.lnx_b = fk(n); e.wqx = tk(n * n); e.bqx = fk(n); e.wox = tk(n * n); e.box = fk(n);
      e.ln2_g = fk(n); e.ln2_b = fk(n); e.w1 = tk(4 * n * n); e.b1 = fk(4 * n); e.w2 = tk(4 * n * n); e.b2 = fk(n);
    }
    ln_g = fk(n); ln_b = fk(n);
    ckv_w = tk(2 * Ld * n * n); ckv_b = fk(2 * Ld * n);
    if (wq_frag)
      for (auto& e : dec) e.wqx_f = tk(n * n);
    if (!ckv_b || (wq_frag && !dec.back().wqx_f)) return fail(-3, "weight arena overflow");
    expected = 5 + La * 15 + 2 + 2 + Ld * 24 + 2;
    // ---------------- activations
    const int WE = std::min(Wcap, enc_chunk());
    // first-pass rows per pass: every window's word-timestamp alignment (<= ~230 tokens)
    // fits one pass, so its GEMMs run at M in the thousands
    PRE = std::max(PRE_ROWS, std::min(Wcap * 240, 8192));
    RD = std::max(Wcap * Gcap, PRE);
    const int LR = std::max(Wcap * Gcap, 2 * Wcap);
    size_t ab = 0;
    auto addA = [&](size_t bytes) { ab += ((bytes + 255) & ~size_t(255)) + 256; };
    addA((size_t)WE * MROWS * nm * sizeof(T)); addA((size_t)WE * H1ROWS * n * sizeof(T));
    addA((size_t)WE * 1500 * n * 4); addA((size_t)WE * 1500 * n * sizeof(T)); addA((size_t)WE * 1500 * 3 * n * sizeof(T));
    addA((size_t)WE * 1500 * n * sizeof(T)); addA((size_t)WE * 1500 * 4 * n * sizeof(T));
    addA(((size_t)WE * nh * 64 * TKP + 64) * sizeof(T));  // encoder V^T (padding keys stay zero)
    addA((size_t)Wcap * 1500 * n * sizeof(T));
    addA((size_t)2 * Ld * Wcap * TKP * n * sizeof(T) + 65536);  // + slack: last key tile reads past TKP
    // the self-attention kernels address one layer's self-K / V cache with 32-bit byte
    // offsets (buffer loads, wh_kernels.hip k_self_attn / k_self_attn_qkv)
    if ((int64_t)Wcap * Gcap * CTX * n * (int64_t)sizeof(T) >= ((int64_t)1 << 31) - 4096)
      return fail(-3, "self-KV cache of one layer exceeds 2 GiB: lower max_windows or max_group");
    for (int l = 0; l < Ld; ++l) { addA((size_t)Wcap * Gcap * CTX * n * sizeof(T)); addA((size_t)Wcap * Gcap * CTX * n * sizeof(T)); }
    addA((size_t)RD * n * 4); addA((size_t)RD * n * sizeof(T)); addA((size_t)RD * n * sizeof(T)); addA((size_t)RD * n * sizeof(T));
    addA((size_t)RD * 4 * n * sizeof(T));
    addA((size_t)RD * nh * NSPLIT * 64 * 4); addA((size_t)RD * nh * NSPLIT * 4); addA((size_t)RD * nh * NSPLIT * 4);
    addA((size_t)LR * V * 4); addA((size_t)2 * Wcap * V * 4); addA(Wcap * 4); addA((size_t)RSPLIT * RD * n * 4);
    for (int i = 0; i < 9; ++i) addA(RD * 4);
    for (int i = 0; i < 5; ++i) addA(RD * 4);
    addA(Ld * nh * 4);
    addA(((V + 31) / 32) * 4);
    addA(Wcap * 8); addA(Wcap * 4);
    // state
    addA((size_t)Wcap * Gcap * HCTX * 4); addA((size_t)Wcap * Gcap * CTX * 4);
    addA((size_t)Wcap * CTX * 4);  // fp_anc
    for (int i = 0; i < 5; ++i) addA(Wcap * 4);
    addA(Wcap * Gcap * 4);
    addA(Wcap * 16 * 4); addA(Wcap * 16 * 4); addA((size_t)Wcap * 16 * HCTX * 4);
    addA((size_t)Wcap * Gcap * KC * 4); addA((size_t)Wcap * Gcap * KC * 4);
    addA((size_t)Wcap * Gcap * LP_SLICES * LP_REC * 4); addA((size_t)Wcap * Gcap * 4);
    addA((size_t)Wcap * 4);  // window arrival counters of the merging selection
    addA(VS_REC_FLOATS * 4); addA(64);  // single-window tail records + arrival counter
    addA(64);
    addA(64);
    addA((size_t)P1_SLABS * 256 * 4); addA((size_t)(4 * n / 16) * 4);  // k_proj1 split-K slabs + counters
    addA((size_t)Wcap * nh * XS_NSP * XREC * 4); addA((size_t)Wcap * nh * 4);  // cross-attention segment records
    addA((size_t)8 * n * 4);  // k_proj1 path (<= 8 rows, wh_proj.h P1_RMAX): the second residual buffer
    addA((size_t)nh * XQ1_P * 4 * 64 * 16); addA((size_t)nh * 2 * 4);  // split query partials + counters
    addA((size_t)EKZ_TILES(n) * 65536); addA((size_t)EKZ_TILES(n) * 4 * 4);  // single-window encoder K halves
    HIPCHK(hipMalloc(&abase, ab));
    HIPCHK(hipMemset(abase, 0, ab));
    aa.base = (char*)abase;
    aa.cap = ab;
    auto ta = [&](size_t elems) { return (T*)aa.take(elems * sizeof(T)); };
    auto fa = [&](size_t elems) { return (float*)aa.take(elems * 4); };
    auto ia = [&](size_t elems) { return (int*)aa.take(elems * 4); };
    melT = ta((size_t)WE * MROWS * nm); h1 = ta((size_t)WE * H1ROWS * n);
    x_e = fa((size_t)WE * 1500 * n); xn_e = ta((size_t)WE * 1500 * n); qkv_e = ta((size_t)WE * 1500 * 3 * n);
    att_e = ta((size_t)WE * 1500 * n); hm_e = ta((size_t)WE * 1500 * 4 * n);
    vt_e = ta((size_t)WE * nh * 64 * TKP + 64);  // + the last key tile's read past TKP
    xa = ta((size_t)Wcap * 1500 * n);
    ckv = ta((size_t)2 * Ld * Wcap * TKP * n + 32768 / sizeof(T));
    kc.resize(Ld); vc.resize(Ld);
    for (int l = 0; l < Ld; ++l) { kc[l] = ta((size_t)Wcap * Gcap * CTX * n); vc[l] = ta((size_t)Wcap * Gcap * CTX * n); }
    x_d = fa((size_t)RD * n); xn_d = ta((size_t)RD * n); q_d = ta((size_t)RD * n); att_d = ta((size_t)RD * n);
    hm_d = ta((size_t)RD * 4 * n);
    po = fa((size_t)RD * nh * NSPLIT * 64); pm = fa((size_t)RD * nh * NSPLIT); pl = fa((size_t)RD * nh * NSPLIT);
    logits = fa((size_t)LR * V); logits2 = fa((size_t)2 * Wcap * V); nsp = fa(Wcap); part = fa((size_t)RSPLIT * RD * n);
    row_tok = ia(RD); row_pos = ia(RD); row_win = ia(RD); row_slot = ia(RD); win_row0 = ia(RD); win_nrows = ia(RD);
    win_slot = ia(RD); rows_in = ia(RD); src_rows = ia(RD);
    st_row_win = ia(RD); st_row_slot = ia(RD); st_win_row0 = ia(RD); st_win_nrows = ia(RD); st_win_slot = ia(RD);
    qk_map = ia(Ld * nh);
    suppress = (unsigned*)ia((V + 31) / 32);
    d_seeks = (int64_t*)aa.take(Wcap * 8); d_segs = ia(Wcap);
    S.hist = ia((size_t)Wcap * Gcap * HCTX); S.anc = ia((size_t)Wcap * Gcap * CTX);
    fp_anc = ia((size_t)Wcap * CTX);  // first passes' ancestry: all zero (beam slot 0), never written
    S.len = ia(Wcap); S.sample_begin = ia(Wcap); S.step = ia(Wcap); S.done = ia(Wcap); S.fin_n = ia(Wcap);
    S.sum_lp = fa(Wcap * Gcap);
    S.fin_score = fa(Wcap * 16); S.fin_len = ia(Wcap * 16); S.fin_tok = ia((size_t)Wcap * 16 * HCTX);
    S.cand_val = fa((size_t)Wcap * Gcap * KC); S.cand_idx = ia((size_t)Wcap * Gcap * KC);
    S.lpart = fa((size_t)Wcap * Gcap * LP_SLICES * LP_REC); S.lp_cnt = ia((size_t)Wcap * Gcap);  // zeroed with the arena
    S.lpw_cnt = ia((size_t)Wcap);
    vs_rec = fa(VS_REC_FLOATS); vs_cnt = ia(16);  // zeroed with the arena
    S.seed = (unsigned long long*)aa.take(64);
    p1_slab = fa((size_t)P1_SLABS * 256); p1_cnt = ia(4 * n / 16);  // zeroed with the arena
    xs_rec = fa((size_t)Wcap * nh * XS_NSP * XREC); xs_cnt = ia((size_t)Wcap * nh);
    x2_d = fa((size_t)8 * n);
    xq1_part = fa((size_t)nh * XQ1_P * 4 * 64 * 4); xq1_cnt = ia((size_t)nh * 2);  // zeroed with the arena
    ekz_slab = fa((size_t)EKZ_TILES(n) * 16384); ekz_cnt = ia((size_t)EKZ_TILES(n) * 4);  // zeroed with the arena
    if (!fp_anc || !S.seed || !S.cand_idx || !S.lp_cnt || !S.lpw_cnt || !vs_cnt || !p1_cnt || !xs_cnt || !x2_d || !ekz_cnt ||
        !xq1_cnt)
      return fail(-3, "activation arena overflow");
    S.nw = Wcap; S.G = 1; S.ctx = CTX; S.hctx = HCTX; S.maxc = 16;
    HIPCHK(hipMalloc(&d_gmax, 64));
    d_gmax_f = (float*)(d_gmax + 4);
    return 0;
  }

  // ------------------------------------------------------------ weights
  int up(void* dst, const std::vector<T>& h) {
    HIPCHK(hipMemcpy(dst, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return 0;
  }
  int upf(float* dst, const float* src, size_t cnt, float scale = 1.f) {
    if (scale == 1.f) {
      HIPCHK(hipMemcpy(dst, src, cnt * 4, hipMemcpyHostToDevice));
      return 0;
    }
    std::vector<float> t(src, src + cnt);
    for (auto& v : t) v *= scale;
    HIPCHK(hipMemcpy(dst, t.data(), cnt * 4, hipMemcpyHostToDevice));
    return 0;
  }
  int upT(T* dst, const float* src, size_t cnt, float scale = 1.f) {
    std::vector<T> t(cnt);
    for (size_t i = 0; i < cnt; ++i) t[i] = (T)(src[i] * scale);
    return up(dst, t);
  }

  int load(const std::string& name, const float* data, const int64_t* shape, int ndim) override {
    auto numel = [&]() { int64_t c = 1; for (int i = 0; i < ndim; ++i) c *= shape[i]; return (size_t)c; };
    auto need = [&](std::initializer_list<int64_t> want) -> int {
      if ((int)want.size() != ndim) return fail(-4, name + ": bad rank");
      int i = 0;
      for (auto w : want)
        if (shape[i++] != w) return fail(-4, name + ": bad shape");
      return 0;
    };
    const size_t n = ns;
    const float kscale = 0.125f;  // (64)^-0.5: encoder key (encoder.py:38), decoder query (decoder.py:20)
    int rc = 0;
    if (name == "encoder.conv1.weight") {
      TRY(need({(int64_t)n, nm, 3}));
      std::vector<float> t(n * K1p, 0.f);  // [o][j*nm + c] = w[o][c][j]
      for (size_t o = 0; o < n; ++o)
        for (int c = 0; c < nm; ++c)
          for (int j = 0; j < 3; ++j) t[o * K1p + j * nm + c] = data[(o * nm + c) * 3 + j];
      rc = upT(conv1_w, t.data(), t.size());
    } else if (name == "encoder.conv1.bias") { TRY(need({(int64_t)n})); rc = upf(conv1_b, data, n); }
    else if (name == "encoder.conv2.weight") {
      TRY(need({(int64_t)n, (int64_t)n, 3}));
      std::vector<float> t(n * 3 * n);
      for (size_t o = 0; o < n; ++o)
        for (size_t c = 0; c < n; ++c)
          for (int j = 0; j < 3; ++j) t[o * 3 * n + j * n + c] = data[(o * n + c) * 3 + j];
      rc = upT(conv2_w, t.data(), t.size());
    } else if (name == "encoder.conv2.bias") { TRY(need({(int64_t)n})); rc = upf(conv2_b, data, n); }
    else if (name == "encoder.positional_embedding") { TRY(need({1500, (int64_t)n})); rc = upf(pos_enc, data, 1500 * n); }
    else if (name == "encoder.ln_post.weight") { TRY(need({(int64_t)n})); rc = upf(lnp_g, data, n); }
    else if (name == "encoder.ln_post.bias") { TRY(need({(int64_t)n})); rc = upf(lnp_b, data, n); }
    else if (name == "decoder.token_embedding.weight") { TRY(need({V, (int64_t)n})); rc = upT(E, data, (size_t)V * n); }
    else if (name == "decoder.positional_embedding") { TRY(need({CTX, (int64_t)n})); rc = upT(Pdec, data, CTX * n); }
    else if (name == "decoder.ln.weight") { TRY(need({(int64_t)n})); rc = upf(ln_g, data, n); }
    else if (name == "decoder.ln.bias") { TRY(need({(int64_t)n})); rc = upf(ln_b, data, n); }
    else {
      int l = -1;
      char part[128];
      const bool is_enc = sscanf(name.c_str(), "encoder.blocks.%d.%127s", &l, part) == 2;
      const bool is_dec = !is_enc && sscanf(name.c_str(), "decoder.blocks.%d.%127s", &l, part) == 2;
      if (!is_enc && !is_dec) return fail(-5, "unknown tensor " + name);
      const std::string p(part);
      if (is_enc) {
        if (l < 0 || l >= La) return fail(-5, "layer out of range " + name);
        auto& e = enc[l];
        if (p == "attn.query.weight") { TRY(need({(int64_t)n, (int64_t)n})); rc = upT(e.wqkv, data, n * n); }
        else if (p == "attn.query.bias") { TRY(need({(int64_t)n})); rc = upf(e.bqkv, data, n); }
        else if (p == "attn.key.weight") { TRY(need({(int64_t)n, (int64_t)n})); rc = upT(e.wqkv + n * n, data, n * n, kscale); }
        else if (p == "attn.value.weight") { TRY(need({(int64_t)n, (int64_t)n})); rc = upT(e.wqkv + 2 * n * n, data, n * n); }
        else if (p == "attn.value.bias") { TRY(need({(int64_t)n})); rc = upf(e.bqkv + 2 * n, data, n); }
        else if (p == "attn.out.weight") { TRY(need({(int64_t)n, (int64_t)n})); rc = upT(e.wo, data, n * n); }
        else if (p == "attn.out.bias") { TRY(need({(int64_t)n})); rc = upf(e.bo, data, n); }
        else if (p == "attn_ln.weight") { TRY(need({(int64_t)n})); rc = upf(e.ln1_g, data, n); }
        else if (p == "attn_ln.bias") { TRY(need({(int64_t)n})); rc = upf(e.ln1_b, data, n); }
        else if (p == "mlp_ln.weight") { TRY(need({(int64_t)n})); rc = upf(e.ln2_g, data, n); }
        else if (p == "mlp_ln.bias") { TRY(need({(int64_t)n})); rc = upf(e.ln2_b, data, n); }
        else if (p == "mlp.0.weight") { TRY(need({4 * (int64_t)n, (int64_t)n})); rc = upT(e.w1, data, 4 * n * n); }
        else if (p == "mlp.0.bias") { TRY(need({4 * (int64_t)n})); rc = upf(e.b1, data, 4 * n); }
        else if (p == "mlp.2.weight") { TRY(need({(int64_t)n, 4 * (int64_t)n})); rc = upT(e.w2, data, 4 * n * n); }
        else if (p == "mlp.2.bias") { TRY(need({(int64_t)n})); rc = upf(e.b2, data, n); }
        else return fail(-5, "unknown tensor " + name);
      } else {
        if (l < 0 || l >= Ld) return fail(-5, "layer out of range " + name);
        auto& e = dec[l];
        T* ck = ckv_w + (size_t)(2 * l) * n * n;
        if (p == "attn.query.weight") { TRY(need({(int64_t)n, (int64_t)n})); rc = upT(e.wqkv, data, n * n, kscale); }
        else if (p == "attn.query.bias") { TRY(need({(int64_t)n})); rc = upf(e.bqkv, data, n, kscale); }
        else if (p == "attn.key.weight") { TRY(need({(int64_t)n, (int64_t)n})); rc = upT(e.wqkv + n * n, data, n * n); }
        else if (p == "attn.value.weight") { TRY(need({(int64_t)n, (int64_t)n})); rc = upT(e.wqkv + 2 * n * n, data, n * n); }
        else if (p == "attn.value.bias") { TRY(need({(int64_t)n})); rc = upf(e.bqkv + 2 * n, data, n); }
        else if (p == "attn.out.weight") { TRY(need({(int64_t)n, (int64_t)n})); rc = upT(e.wo, data, n * n); }
        else if (p == "attn.out.bias") { TRY(need({(int64_t)n})); rc = upf(e.bo, data, n); }
        else if (p == "attn_ln.weight") { TRY(need({(int64_t)n})); rc = upf(e.ln1_g, data, n); }
        else if (p == "attn_ln.bias") { TRY(need({(int64_t)n})); rc = upf(e.ln1_b, data, n); }
        else if (p == "cross_attn.query.weight") { TRY(need({(int64_t)n, (int64_t)n})); rc = upT(e.wqx, data, n * n, kscale); }
        else if (p == "cross_attn.query.bias") { TRY(need({(int64_t)n})); rc = upf(e.bqx, data, n, kscale); }
        else if (p == "cross_attn.key.weight") { TRY(need({(int64_t)n, (int64_t)n})); rc = upT(ck, data, n * n); }
        else if (p == "cross_attn.value.weight") { TRY(need({(int64_t)n, (int64_t)n})); rc = upT(ck + n * n, data, n * n); }
        else if (p == "cross_attn.value.bias") { TRY(need({(int64_t)n})); rc = upf(ckv_b + (2 * l + 1) * n, data, n); }
        else if (p == "cross_attn.out.weight") { TRY(need({(int64_t)n, (int64_t)n})); rc = upT(e.wox, data, n * n); }
        else if (p == "cross_attn.out.bias") { TRY(need({(int64_t)n})); rc = upf(e.box, data, n); }
        else if (p == "cross_attn_ln.weight") { TRY(need({(int64_t)n})); rc = upf(e.lnx_g, data, n); }
        else if (p == "cross_attn_ln.bias") { TRY(need({(int64_t)n})); rc = upf(e.lnx_b, data, n); }
        else if (p == "mlp_ln.weight") { TRY(need({(int64_t)n})); rc = upf(e.ln2_g, data, n); }
        else if (p == "mlp_ln.bias") { TRY(need({(int64_t)n})); rc = upf(e.ln2_b, data, n); }
        else if (p == "mlp.0.weight") { TRY(need({4 * (int64_t)n, (int64_t)n})); rc = upT(e.w1, data, 4 * n * n); }
        else if (p == "mlp.0.bias") { TRY(need({4 * (int64_t)n})); rc = upf(e.b1, data, 4 * n); }
        else if (p == "mlp.2.weight") { TRY(need({(int64_t)n, 4 * (int64_t)n})); rc = upT(e.w2, data, 4 * n * n); }
        else if (p == "mlp.2.bias") { TRY(need({(int64_t)n})); rc = upf(e.b2, data, n); }
        else return fail(-5, "unknown tensor " + name);
      }
    }
    if (rc) return rc;
    (void)numel;
    loaded.insert(name);
    return 0;
  }

  int finalize() override {
    if (loaded.size() != expected)
      return fail(-6, "loaded " + std::to_string(loaded.size()) + " of " + std::to_string(expected) + " tensors");
    // the fragment-ordered W_q copies (after the 0.125 query scale was folded in at load)
    for (auto& e : dec)
      if (e.wqx_f) launch_wq_frag(e.wqx, e.wqx_f, ns, st);
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipGetLastError());
    HIPCHK(hipDeviceSynchronize());
    finalized = true;
    return 0;
  }

  // ------------------------------------------------------------ GEMM helper
  int gemm(const void* X, int ldx, const T* W, const float* bias, int M, int N, int K, int epi, GemmArgs a) {
    a.X = X; a.ldx = ldx; a.W = W; a.bias = bias; a.M = M; a.N = N; a.K = K;
    if (a.x_group_rows == (1 << 30)) a.x_group_rows = std::max(M, 1);
    const int rc = launch_gemm<T>(a, epi, st);
    if (rc) return fail(-20, "gemm launch failed code " + std::to_string(rc) + " M=" + std::to_string(M) +
                                 " N=" + std::to_string(N) + " K=" + std::to_string(K));
    return 0;
  }

  // ------------------------------------------------------------ mel
  int64_t audio_n = 0;
  int audio_upload(const float* audio, int64_t n) override {
    if ((size_t)n > audio_cap) {
      if (d_audio) HIPCHK(hipFree(d_audio));
      d_audio = nullptr;
      audio_cap = std::max<size_t>(n, 16000);
      HIPCHK(hipMalloc(&d_audio, audio_cap * 4));
    }
    HIPCHK(hipMemcpyAsync(d_audio, audio, n * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
    audio_n = n;
    return 0;
  }
  // audio == nullptr: use the resident buffer of wh_audio_upload (n must match)
  int log_mel(const float* audio, int64_t n, int64_t pad, int n_mels, int normalize, int64_t* nf) override {
    int64_t total = 0;
    TRY(log_mel_frames(audio, n, pad, n_mels, 0, -1, normalize, &total));
    *nf = total;
    return 0;
  }
  // frames [frame0, frame0 + count) of the padded signal's log-mel (count < 0: to the
  // end); the context keeps them with their absolute frame offset (mel_f0), so window
  // seeks stay absolute.  A rank of a sharded file computes only its own frames.
  int log_mel_frames(const float* audio, int64_t n, int64_t pad, int n_mels, int64_t frame0, int64_t count,
                     int normalize, int64_t* total_frames) override {
    if (!h_filters.count(n_mels)) return fail(-7, "mel filters for n_mels=" + std::to_string(n_mels) + " not set");
    if (n + pad <= 200 || n < 1) return fail(-7, "audio too short for reflect padding");
    if (!audio && n != audio_n) return fail(-7, "no resident audio of that length");
    const int64_t total = (n + pad) / 160;
    if (count < 0) count = total - frame0;
    if (frame0 < 0 || count < 1 || frame0 + count > total) return fail(-7, "mel frame range out of bounds");
    if (audio && (size_t)n > audio_cap) {
      if (d_audio) HIPCHK(hipFree(d_audio));
      d_audio = nullptr;
      audio_cap = std::max<size_t>(n, 16000);
      HIPCHK(hipMalloc(&d_audio, audio_cap * 4));
    }
    const size_t need = (size_t)n_mels * count;
    if (need > mel_cap) {
      if (d_mel) HIPCHK(hipFree(d_mel));
      d_mel = nullptr;
      mel_cap = need;
      HIPCHK(hipMalloc(&d_mel, mel_cap * 4));
    }
    HIPCHK(hipEventRecord(tm.a, st));
    if (audio) {
      HIPCHK(hipMemcpyAsync(d_audio, audio, n * 4, hipMemcpyHostToDevice, st));
      audio_n = n;
    }
    HIPCHK(hipMemsetAsync(d_gmax, 0, 16, st));
    launch_mel(d_audio, n, n + pad, frame0, count, d_filters[n_mels], n_mels, d_mel, count, d_gmax, st);
    if (normalize) launch_mel_norm(d_mel, count, count, n_mels, d_gmax, nullptr, st);
    HIPCHK(hipEventRecord(tm.b, st));
    HIPCHK(hipStreamSynchronize(st));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, tm.a, tm.b));
    stats[0] += ms;
    mel_frames = count;
    mel_f0 = frame0;
    mel_nm = n_mels;
    *total_frames = total;
    return 0;
  }
  std::map<int, std::vector<float>> h_filters;
  int mel_max(float* g) override {
    unsigned u = 0;
    HIPCHK(hipMemcpy(&u, d_gmax, 4, hipMemcpyDeviceToHost));
    const unsigned v = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
    memcpy(g, &v, 4);
    return 0;
  }
  int mel_normalize(float g) override {
    HIPCHK(hipMemcpyAsync(d_gmax_f, &g, 4, hipMemcpyHostToDevice, st));
    launch_mel_norm(d_mel, mel_frames, mel_frames, mel_nm, d_gmax, d_gmax_f, st);
    HIPCHK(hipStreamSynchronize(st));
    return 0;
  }
  int mel_read(float* out, int64_t f0, int64_t nf) override {
    f0 -= mel_f0;  // absolute frame -> stored frame
    if (f0 < 0 || nf < 0 || f0 + nf > mel_frames) return fail(-8, "mel_read out of range");
    HIPCHK(hipMemcpy2D(out, nf * 4, d_mel + f0, mel_frames * 4, nf * 4, mel_nm, hipMemcpyDeviceToHost));
    return 0;
  }
  int mel_write(const float* mel, int64_t nf) override {
    const size_t need = (size_t)nm * nf;
    if (need > mel_cap) {
      if (d_mel) HIPCHK(hipFree(d_mel));
      d_mel = nullptr;
      mel_cap = need;
      HIPCHK(hipMalloc(&d_mel, mel_cap * 4));
    }
    HIPCHK(hipMemcpy(d_mel, mel, need * 4, hipMemcpyHostToDevice));
    mel_frames = nf;
    mel_f0 = 0;
    mel_nm = nm;
    return 0;
  }

  // ------------------------------------------------------------ encoder
  // single: the encode is ONE window (its decode batch runs the single-window path too):
  // the residual GEMMs (conv2, out, fc2) split K in two halves inside the launch — within
  // the fp16 bound of the multi-window encoder, not bit-equal to it, as k_proj1 in the step
  int encode_chunk(int s0, int we, bool single = false) {
    const int n = ns;
    GemmArgs g;
    const bool kz = single && we == 1 && sizeof(T) == 2 && !(tune_env("WHISPER_HIP_ENC_KZ") && tune_env("WHISPER_HIP_ENC_KZ")[0] == '0');
    auto kz_on = [&](GemmArgs& ga) {
      if (!kz) return;
      ga.p1_slab = ekz_slab;
      ga.p1_cnt = ekz_cnt;
      ga.p1_slabs = EKZ_TILES(n) * 64;
    };
    // mel windows -> time-major (T), conv1 as overlapping-row GEMM (lda = n_mels)
    launch_mel_windows<T>(d_mel, mel_frames, nm, d_seeks + s0, d_segs + s0, melT, (int64_t)MROWS * nm, MROWS, we, st);
    g = GemmArgs();
    g.x_group_rows = 3000; g.x_group_stride = (int64_t)MROWS * nm;
    g.out = h1; g.ldo = n; g.out_group_stride = (int64_t)H1ROWS * n; g.out_row_off = 1;
    TRY(gemm(melT, nm, conv1_w, conv1_b, we * 3000, n, K1p, EPI_STORE_GELU, g));
    launch_zero_rows<T>(h1, (int64_t)H1ROWS * n, n, 0, H1ROWS - 1, we, st);
    // conv2 (stride 2): row t reads padded rows 2t..2t+2 -> lda = 2n; + GELU + positional embedding
    g = GemmArgs();
    g.x_group_rows = 1500; g.x_group_stride = (int64_t)H1ROWS * n;
    g.out_f32 = x_e; g.ldo = n; g.pos = pos_enc;
    kz_on(g);
    TRY(gemm(h1, 2 * n, conv2_w, conv2_b, we * 1500, n, 3 * n, EPI_GELU_POS, g));
    const int M = we * 1500;
    for (int l = 0; l < La; ++l) {
      auto& e = enc[l];
      launch_layernorm<T>(x_e, xn_e, e.ln1_g, e.ln1_b, M, n, 1e-7f, nullptr, st);
      // q, k -> qkv_e; v -> vt_e as per-(window, head) V^T with permuted keys
      g = GemmArgs(); g.out = qkv_e; g.ldo = 3 * n;
      g.x_group_rows = 1500; g.x_group_stride = (int64_t)1500 * n; g.out_group_stride = (int64_t)1500 * 3 * n;
      g.hs_state = n; g.hs_heads = nh; g.hs_T = TKP; g.vc = vt_e;
      TRY(gemm(xn_e, n, e.wqkv, e.bqkv, M, 3 * n, n, EPI_QKV_ENC, g));
      launch_attn_enc<T>(qkv_e, 3 * n, n, nh, 1500, we, (int64_t)1500 * 3 * n, vt_e, TKP, att_e, (int64_t)1500 * n, st);
      g = GemmArgs(); g.out_f32 = x_e; g.ldo = n;
      kz_on(g);
      TRY(gemm(att_e, n, e.wo, e.bo, M, n, n, EPI_RESID, g));
      launch_layernorm<T>(x_e, xn_e, e.ln2_g, e.ln2_b, M, n, 1e-7f, nullptr, st);
      g = GemmArgs(); g.out = hm_e; g.ldo = 4 * n;
      TRY(gemm(xn_e, n, e.w1, e.b1, M, 4 * n, n, EPI_STORE_GELU, g));
      g = GemmArgs(); g.out_f32 = x_e; g.ldo = n;
      kz_on(g);
      TRY(gemm(hm_e, 4 * n, e.w2, e.b2, M, n, 4 * n, EPI_RESID, g));
    }
    T* xa_s = xa + (size_t)s0 * 1500 * n;
    launch_layernorm<T>(x_e, xa_s, lnp_g, lnp_b, M, n, 1e-7f, nullptr, st);
    // cross-KV for every decoder layer in one GEMM, written head-split [l2][slot][h][t][64]
    g = GemmArgs();
    g.x_group_rows = 1500; g.x_group_stride = (int64_t)1500 * n;
    g.out = ckv; g.hs_state = n; g.hs_heads = nh; g.hs_T = TKP; g.hs_nslots = Wcap; g.hs_slot0 = s0;
    TRY(gemm(xa_s, n, ckv_w, ckv_b, M, 2 * Ld * n, n, EPI_HEADSPLIT, g));
    return 0;
  }

  int encode(int n_win, const int64_t* seeks, const int* segs) override {
    if (!finalized) return fail(-9, "weights not finalized");
    if (n_win < 1 || n_win > Wcap) return fail(-9, "n_win out of range");
    if (!d_mel || mel_nm != nm) return fail(-9, "no mel of the model's n_mels in the context");
    // seeks are absolute frames; the stored mel starts at mel_f0
    h_seeks.resize(n_win);
    for (int i = 0; i < n_win; ++i) {
      const int64_t s = seeks[i] - mel_f0;
      if (s < 0 || segs[i] < 1 || s + std::min(segs[i], 3000) > mel_frames) return fail(-9, "bad window");
      h_seeks[i] = s;
    }
    HIPCHK(hipEventRecord(tm.a, st));
    HIPCHK(hipMemcpyAsync(d_seeks, h_seeks.data(), n_win * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_segs, segs, n_win * 4, hipMemcpyHostToDevice, st));
    const int WE = std::min(Wcap, enc_chunk());
    for (int s0 = 0; s0 < n_win; s0 += WE) TRY(encode_chunk(s0, std::min(WE, n_win - s0), n_win == 1));
    HIPCHK(hipEventRecord(tm.b, st));
    HIPCHK(hipStreamSynchronize(st));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, tm.a, tm.b));
    stats[1] += ms;
    stats[5] += n_win;
    TRY(launch_status(__func__));
    return 0;
  }

  int read_xa(int slot, float* out) override {
    if (slot < 0 || slot >= Wcap) return fail(-10, "slot");
    const size_t cnt = (size_t)1500 * ns;
    std::vector<T> h(cnt);
    HIPCHK(hipMemcpy(h.data(), xa + (size_t)slot * cnt, cnt * sizeof(T), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < cnt; ++i) out[i] = (float)h[i];
    return 0;
  }
  int read_ckv(int slot, int layer, float* k, float* v) override {
    if (slot < 0 || slot >= Wcap || layer < 0 || layer >= Ld) return fail(-10, "slot/layer");
    const size_t per = (size_t)nh * TKP * 64;
    std::vector<T> h(per);
    for (int kv = 0; kv < 2; ++kv) {
      const T* src = ckv + ((size_t)(2 * layer + kv) * Wcap + slot) * per;
      HIPCHK(hipMemcpy(h.data(), src, per * sizeof(T), hipMemcpyDeviceToHost));
      float* o = kv ? v : k;
      for (int hh = 0; hh < nh; ++hh)
        for (int t = 0; t < 1500; ++t) {
          // K: [H][TKP][64]; V: transposed, tile-major with the 32-key permutation (xv_index)
          for (int dd = 0; dd < 64; ++dd)
            o[((size_t)hh * 1500 + t) * 64 + dd] =
                kv ? (float)h[(size_t)hh * 64 * TKP + xv_index(dd, t)] : (float)h[((size_t)hh * TKP + t) * 64 + dd];
        }
    }
    return 0;
  }

  // ------------------------------------------------------------ decoder layers
  // R rows of x_d (f32 residual); rw/rs/rp: row window / beam slot / position
  // ancG: beams per window in the anc table layout [w][ancG][ctx]; KV slots use Gcap
  // residual projection x += X W^T + b, then xn = LayerNorm(x) with the NEXT norm's
  // parameters.  Up to 128 rows: split-K weight streaming into fp32 partial slabs,
  // summed in fixed order by k_resid_ln (deterministic, no atomics).  More rows:
  // tile GEMM with an in-place residual epilogue.
  // how many [R][N] fp32 slabs fit in the partial buffer
  int part_slabs(int R, int N) const { return (int)std::min<int64_t>(16, (int64_t)RSPLIT * RD * ns / ((int64_t)R * N)); }

  // X[R][K] W^T into the split-K partial slabs part[z][R][N]: k_proj where a tile
  // configuration fits (decode rows <= 112), the k_gemv path otherwise; *ks = z
  // fp16 contexts store the slabs as fp16 (slab_h = 1 after such a partial(); the QKV
  // projection's too when the self-attention is the pipelined fp16 form): half the bytes
  // written by every k_proj and read by k_resid_ln / k_reduce_store / k_xattn_seg.  Round 4
  // measured 0.3 % and kept fp32; after round 5's issue-side fixes the 20-window step graph
  // is 3.378 -> 3.276 ms (early) and 3.661 -> 3.559 ms (150 tokens) with it
  // (profiles/r05/ab_slab16.txt), the fp16 teacher-forced / invariance tests unchanged.
  // Partial sums rounded to fp16 (the reference's CoreML path is fp16 end to end; the
  // residual stream here stays fp32).  Tuning build: WHISPER_HIP_SLAB16=0 keeps fp32 slabs.
  int slab_h = 0;
  static bool slab16_enabled() {
    static const bool on = [] {
      const char* e = tune_env("WHISPER_HIP_SLAB16");
      return !(e && e[0] == '0');
    }();
    return on;
  }
  // the QKV projection's slabs (read by k_self_attn_qkv's fp16 pipelined form) fp16 too:
  // 20-window step graph 3.261 / 3.258 -> 3.255 / 3.246 ms, 3.557 -> 3.546 at 150 tokens
  // (profiles/r05/ab_slab16_qkv.txt).  Tuning build: WHISPER_HIP_SLAB16_QKV=0 keeps them fp32
  static bool slab16_qkv() {
    static const bool on = [] {
      const char* e = tune_env("WHISPER_HIP_SLAB16_QKV");
      return !(e && e[0] == '0');
    }();
    return on;
  }
  int partial(const void* X, int ldx, const T* W, int R, int N, int K, int* ks, bool half_ok = true) {
    GemmArgs g;
    g.X = X; g.ldx = ldx; g.W = W; g.M = R; g.N = N; g.K = K; g.x_group_rows = R;
    g.out_f32 = part; g.ldo = N;
    g.slab_half = half_ok && sizeof(T) == 2 && slab16_enabled();
    slab_h = g.slab_half;
    const int maxz = part_slabs(R, N);
    // time_stage(7): each k_proj of an eager step timed by its own dispatch events
    const bool tev = proj_ev_n < (int)proj_ev.size() / 2;
    const int rc = tev ? launch_proj_partial<T>(g, maxz, st, ks, proj_ev[2 * proj_ev_n], proj_ev[2 * proj_ev_n + 1])
                       : launch_proj_partial<T>(g, maxz, st, ks);
    if (tev && rc == 0) ++proj_ev_n;
    if (rc == 0) return 0;
    if (rc != -1) return fail(-20, "k_proj launch failed code " + std::to_string(rc));
    slab_h = 0;
    *ks = gemv_ksplit(R, N, K, maxz);
    g = GemmArgs();
    g.out_f32 = part; g.ldo = N; g.ksplit = *ks;
    return gemm(X, ldx, W, nullptr, R, N, K, EPI_PARTIAL, g);
  }

  // pf: an L2 prefetch for the next launch, carried by the split-K reduction (round 6)
  int resid(const T* X, int K, const T* W, const float* b, int R, const float* lg, const float* lb,
            const L2Prefetch* pf = nullptr) {
    const int n = ns;
    GemmArgs g;
    if (R > 128) {
      g.out_f32 = x_d; g.ldo = n;
      TRY(gemm(X, K, W, b, R, n, K, EPI_RESID, g));
      launch_resid_ln<T>(x_d, nullptr, 0, 0, nullptr, xn_d, lg, lb, R, n, 1e-5f, st);
    } else {
      int ks = 0;
      TRY(partial(X, K, W, R, n, K, &ks));
      launch_resid_ln<T>(x_d, part, ks, (int64_t)R * n, b, xn_d, lg, lb, R, n, 1e-5f, st, slab_h, pf);
    }
    return 0;
  }
  // the step cross-attention's W_q head slices into the L2 of the XCDs whose k_xattn_seg
  // workgroups read them, by the k_resid_ln before it: tuning build only, WHISPER_HIP_XQ_PF=1.
  // Measured slower (profiles/r06/ab_xq_l2_prefetch.txt: the k_resid_ln 1.4 us longer, the
  // cross-attention not shorter — its query phase does not wait on L2 misses)
  static bool xq_pf_on() {
    static const bool on = [] {
      const char* e = tune_env("WHISPER_HIP_XQ_PF");
      return e && e[0] == '1';
    }();
    return on;
  }

  // round-6 probe, tuning build only: WHISPER_HIP_XKV_PF=<workgroups> pulls each layer's
  // cross K / V through the memory side on a second stream (k_kv_pull), forked after the
  // previous layer's cross-attention, joined at the end of the layers
  static int xkv_pf_wg() {
    static const int v = [] {
      const char* e = tune_env("WHISPER_HIP_XKV_PF");
      return e ? atoi(e) : 0;
    }();
    return v;
  }
  hipStream_t pst = nullptr;
  std::vector<hipEvent_t> kv_ev;
  unsigned* kv_sink = nullptr;
  int kv_pull_setup() {
    if (pst) return 0;
    // WHISPER_HIP_XKV_PRIO=1: the pull stream at the device's greatest priority
    const char* pe = tune_env("WHISPER_HIP_XKV_PRIO");
    if (pe && pe[0] == '1') {
      int lo = 0, hi = 0;
      HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
      HIPCHK(hipStreamCreateWithPriority(&pst, hipStreamNonBlocking, hi));
    } else {
      HIPCHK(hipStreamCreateWithFlags(&pst, hipStreamNonBlocking));
    }
    kv_ev.resize(Ld + 1);
    for (auto& e : kv_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(hipMalloc((void**)&kv_sink, 256));
    return 0;
  }
  int kv_pull(int l, int nwin, const int* wsl) {
    HIPCHK(hipEventRecord(kv_ev[l], st));
    HIPCHK(hipStreamWaitEvent(pst, kv_ev[l], 0));
    const size_t n = ns;
    launch_kv_pull(ckv + (size_t)(2 * l) * Wcap * TKP * n, ckv + (size_t)(2 * l + 1) * Wcap * TKP * n, wsl, nwin,
                   (int64_t)TKP * n * sizeof(T), xkv_pf_wg(), kv_sink, pst);
    return 0;
  }
  int kv_join() {
    HIPCHK(hipEventRecord(kv_ev[Ld], pst));
    HIPCHK(hipStreamWaitEvent(st, kv_ev[Ld], 0));
    return 0;
  }

  // out = act(xn W^T + b) for R rows (cross-attention query, MLP fc1): split-K
  // partial slabs + fixed-order reduce in step mode, the direct GEMM otherwise
  int proj(const T* W, const float* b, int R, int N, T* out, int gelu, bool skinny) {
    GemmArgs g;
    if (skinny) {
      int ks = 0;
      TRY(partial(xn_d, ns, W, R, N, ns, &ks));
      launch_reduce_store<T>(part, ks, (int64_t)R * N, b, out, N, R, N, gelu, st, slab_h);
    } else {
      g.out = out; g.ldo = N;
      TRY(gemm(xn_d, ns, W, b, R, N, ns, gelu ? EPI_STORE_GELU : EPI_STORE, g));
    }
    return 0;
  }

  // R rows of x_d (embeddings in, residual stream out); on exit xn_d holds the final
  // decoder LayerNorm of every row (decoder.py:316) — except on the k_proj1 path
  // (dec_layers_p1), which leaves final_x set instead: vocab() computes that LayerNorm
  // in its prologue.
  // anc: the ancestry table the self-attention reads ([w][ancG][CTX]); the decode's S.anc
  // unless a first pass (alignment / prefill logits) gives its own (fp_anc: all zeros)
  int sa_probe_ks = 1;  // the QKV projection's split count (time_stage 8 / 9)
  int sa_probe_half = 0;  // and whether its slabs were fp16
  int dec_layers(int R, const int* rw, const int* rs, const int* rp, int ancG, int nwin, const int* wr0, const int* wnr,
                 const int* wsl, float* aqk, const int* qkmap, int qkrows, bool step = false,
                 const int* anc = nullptr) {
    const int* A = anc ? anc : S.anc;
    const int n = ns;
    // step mode (one row per beam, rows independent): the skinny projections run
    // split-K into fp32 partial slabs; QKV's reduction is fused into self-attention
    const bool skinny = step && R <= 128;
    GemmArgs g;
    final_x = nullptr;
    if (step && !qkmap && p1_active(R, nwin))
      return dec_layers_p1(R, rw, rs, rp, ancG, nwin, wr0, wnr, wsl, A);
    launch_layernorm<T>(x_d, xn_d, dec[0].ln1_g, dec[0].ln1_b, R, n, 1e-5f, nullptr, st);
    const bool kvpf = skinny && nwin >= 2 && xkv_pf_wg() > 0;
    if (kvpf) {
      TRY(kv_pull_setup());
      TRY(kv_pull(0, nwin, wsl));
    }
    for (int l = 0; l < Ld; ++l) {
      auto& e = dec[l];
      if (skinny) {
        int ks = 0;
        TRY(partial(xn_d, n, e.wqkv, R, 3 * n, n, &ks, slab16_qkv() && self_attn_pipe_on() && !self_attn_grp_mode()));
        sa_probe_ks = ks;
        sa_probe_half = slab_h;
        if (launch_self_attn_qkv<T>(part, ks, (int64_t)R * 3 * n, e.bqkv, n, kc[l], vc[l], rw, rs, rp, A, ancG,
                                    Gcap, nh, CTX, att_d, n, R, st, slab_h))
          return fail(-20, "self-attention rows are not a whole number of beam groups");
      } else {
        g = GemmArgs();
        g.out = q_d; g.ldo = n; g.hs_state = n; g.hs_heads = nh;
        g.row_win = rw; g.row_slot = rs; g.row_pos = rp; g.kc = kc[l]; g.vc = vc[l]; g.kv_beams = Gcap; g.kv_ctx = CTX;
        TRY(gemm(xn_d, n, e.wqkv, e.bqkv, R, 3 * n, n, EPI_QKV_DEC, g));
        launch_self_attn<T>(q_d, n, kc[l], vc[l], rw, rs, rp, A, ancG, Gcap, nh, CTX, att_d, n, R, st);
      }
      L2Prefetch pf;
      const bool use_pf = skinny && xq_proj_active(ancG) && xq_pf_on() && xattn_l2_ranges(nwin, nh, ancG, &pf);
      if (use_pf) {
        pf.base = reinterpret_cast<const char*>(e.wqx);
        pf.unit = (int64_t)64 * n * sizeof(T);
      }
      TRY(resid(att_d, n, e.wo, e.bo, R, e.lnx_g, e.lnx_b, use_pf ? &pf : nullptr));
      // cross-attention query: in step mode its split-K slabs are reduced inside
      // k_cross_attn (rows per window <= Gcap <= 8), otherwise projected directly
      XQPart xq;
      if (skinny) xq = step_xq(ancG);
      if (skinny && xq_proj_active(ancG)) {
        // round 6: no cross-q launch; k_xattn_seg projects the LayerNorm'd rows itself
        xq.qx = xn_d; xq.qw = e.wqx; xq.bias = e.bqx;
        if (xq_frag_on()) xq.qwf = e.wqx_f;
      } else if (skinny && xq_fused) {
        int ks = 0;
        TRY(partial(xn_d, n, e.wqx, R, n, n, &ks));
        if (cross_attn_q_slabs(ks)) {
          xq.part = part; xq.part_half = slab_h; xq.stride = (int64_t)R * n; xq.z = ks; xq.bias = e.bqx;
        } else {
          launch_reduce_store<T>(part, ks, (int64_t)R * n, e.bqx, q_d, n, R, n, 0, st, slab_h);
        }
      } else {
        TRY(proj(e.wqx, e.bqx, R, n, q_d, 0, skinny));
      }
      const T* ck = ckv + (size_t)(2 * l) * Wcap * TKP * n;
      const T* cv = ckv + (size_t)(2 * l + 1) * Wcap * TKP * n;
      launch_cross_attn<T>(q_d, n, ck, cv, 1500, nh, NSPLIT, nwin, wr0, wnr, wsl, (int64_t)TKP * n, po, pm, pl, att_d,
                           n, R, aqk, qkmap ? qkmap + l * nh : nullptr, qkrows, st, xq);
      if (kvpf && l + 1 < Ld) TRY(kv_pull(l + 1, nwin, wsl));
      TRY(resid(att_d, n, e.wox, e.box, R, e.ln2_g, e.ln2_b));
      TRY(proj(e.w1, e.b1, R, 4 * n, hm_d, 1, skinny));
      const bool last = l + 1 == Ld;
      TRY(resid(hm_d, 4 * n, e.w2, e.b2, R, last ? ln_g : dec[l + 1].ln1_g, last ? ln_b : dec[l + 1].ln1_b));
    }
    if (kvpf) TRY(kv_join());
    return 0;
  }

  // Decoder step at <= P1_RMAX rows (one window's beams: the per-token latency path):
  // every projection is one k_proj1 launch over the whole K with its epilogue fused
  // (QKV scatter, residual add, GELU) and the LayerNorm before it recomputed in its
  // prologue, so a layer is 8 launches: qkv, self-attn, out, cross-q, cross-attn,
  // cross-out, fc1, fc2 (12 on the split-K path: + 3 resid+LN, + reduce+GELU).
  // WHISPER_HIP_P1=0 keeps the split-K path (A/B).
  static bool p1_enabled() {
    static const bool on = [] {
      const char* e = tune_env("WHISPER_HIP_P1");
      return !(e && e[0] == '0');
    }();
    return on;
  }

  int p1(GemmArgs& g, int epi, bool ln) {
    g.p1_slab = p1_slab;
    g.p1_cnt = p1_cnt;
    g.p1_slabs = P1_SLABS;
    // time_stage(7): each projection of an eager step timed by its own dispatch events
    const bool tev = proj_ev_n < (int)proj_ev.size() / 2;
    const int rc = tev ? launch_proj1<T>(g, epi, ln, st, proj_ev[2 * proj_ev_n], proj_ev[2 * proj_ev_n + 1])
                       : launch_proj1<T>(g, epi, ln, st);
    if (tev && rc == 0) ++proj_ev_n;
    return rc == 0 ? 0 : fail(-20, "k_proj1 launch failed code " + std::to_string(rc));
  }

  // the six projections of layer l as the step issues them (p1 path: k_proj1 with the
  // step's epilogues; split path: k_proj into partial slabs) — time_stage(2)
  int layer_projections(int l, int R) {
    const int n = ns;
    auto& e = dec[l];
    if (p1_active(R, cur_nwin)) {
      GemmArgs g;
      g.W = e.wqkv; g.bias = e.bqkv; g.M = R; g.N = 3 * n; g.K = n;
      g.xf32 = x_d; g.ln_g = e.ln1_g; g.ln_b = e.ln1_b; g.ln_eps = 1e-5f;
      g.out = q_d; g.ldo = n; g.hs_state = n; g.hs_heads = nh;
      g.row_win = st_row_win; g.row_slot = st_row_slot; g.row_pos = row_pos; g.kc = kc[l]; g.vc = vc[l];
      g.kv_beams = Gcap; g.kv_ctx = CTX;
      TRY(p1(g, EPI_QKV_DEC, true));
      struct Q { const T* X; int K; const T* W; const float* b; int N; int epi; const float* lg; const float* lb; T* out; };
      const Q qs[5] = {{att_d, n, e.wo, e.bo, n, EPI_RESID, nullptr, nullptr, nullptr},
                       {nullptr, n, e.wqx, e.bqx, n, EPI_STORE, e.lnx_g, e.lnx_b, q_d},
                       {att_d, n, e.wox, e.box, n, EPI_RESID, nullptr, nullptr, nullptr},
                       {nullptr, n, e.w1, e.b1, 4 * n, EPI_STORE_GELU, e.ln2_g, e.ln2_b, hm_d},
                       {hm_d, 4 * n, e.w2, e.b2, n, EPI_RESID, nullptr, nullptr, nullptr}};
      for (const Q& q : qs) {
        if (q.W == e.wqx && xq_proj1_active(R)) continue;  // the step projects the cross-q in k_xattn_seg
        g = GemmArgs();
        g.W = q.W; g.bias = q.b; g.M = R; g.N = q.N; g.K = q.K;
        if (q.lg) {
          g.xf32 = x_d; g.ln_g = q.lg; g.ln_b = q.lb; g.ln_eps = 1e-5f; g.out = q.out; g.ldo = q.N;
        } else {
          g.X = q.X; g.ldx = q.K; g.out_f32 = x_d; g.ldo = n;
        }
        TRY(p1(g, q.epi, q.lg != nullptr));
      }
      return 0;
    }
    struct P { const T* X; int K; const T* W; int N; } ps[6] = {
        {xn_d, n, e.wqkv, 3 * n}, {att_d, n, e.wo, n}, {xn_d, n, e.wqx, n},
        {att_d, n, e.wox, n},     {xn_d, n, e.w1, 4 * n}, {hm_d, 4 * n, e.w2, n}};
    for (auto& p : ps) {
      if (p.W == e.wqx && xq_proj_active(cur_G)) continue;  // the step projects the cross-q in k_xattn_seg
      int ks = 0;
      TRY(partial(p.X, p.K, p.W, R, p.N, p.K, &ks));
    }
    return 0;
  }

  // the k_proj1 layers serve exactly one window (its beams, <= P1_RMAX rows): the cut is a
  // window count, not a row count, so a window's step arithmetic is the same in every
  // batch of >= 2 windows whatever the beam count (greedy included; batch invariance,
  // DESIGN.md §2)
  bool p1_active(int R, int n_win) const { return n_win == 1 && p1_enabled() && proj1_supported(R, ns); }
  std::string step_kernels(int n_win, int group) const override {
    const bool p1 = p1_active(n_win * group, n_win), h = sizeof(T) == 2;
    return std::string("proj=") + (p1 ? "k_proj1" : "k_proj") + ",xattn=k_xattn_seg" +
           (!p1 && xq_proj_active(group) ? "<qproj>" : p1 && xq_proj1_active(group) ? (xq_proj1_mode() == 2 ? "<qproj-split+ln>" : "<qproj+ln>") : "") +
           ",self_attn=" +
           (p1 ? (h && self_attn_kco_on() ? "k_self_attn<kco>" : "k_self_attn")
               : h && group >= 2 && self_attn_grp_mode() ? "k_self_attn_grp"
                                                           : h && self_attn_pipe_on() ? (self_attn_kco_on() ? "k_self_attn_qkv<pipe+kco>" : "k_self_attn_qkv<pipe>")
                                                                                      : "k_self_attn_qkv") +
           ",tail=" + (p1 && h && ns == 1280 && vocab_select_on() ? "k_vocab_sel" : "vocab+k_logit_part");
  }

  int dec_layers_p1(int R, const int* rw, const int* rs, const int* rp, int ancG, int nwin, const int* wr0,
                    const int* wnr, const int* wsl, const int* A) {
    const int n = ns;
    // deferred residual: fc2 stores its two K-half slabs only; the next layer's QKV
    // LayerNorm prologue adds them (+ bias) to the current rows and one of its workgroups
    // publishes the sum into the other buffer, which becomes current (fc2 7.9 -> 5.9 us,
    // the QKV prologue +0.6; profiles/r03/step_w1_p1def_summary.txt)
    float* xc = x_d;
    float* xo = x2_d;
    const float* pend = nullptr;  // bias of the residual pending in p1_slab
    auto ln_in = [&](GemmArgs& g, const float* lg, const float* lb) {
      g.xf32 = xc; g.ln_g = lg; g.ln_b = lb; g.ln_eps = 1e-5f;
      if (pend) { g.res_slab = p1_slab; g.res_bias = pend; g.x_out = xo; }
    };
    auto ln_done = [&]() {
      if (pend) { std::swap(xc, xo); pend = nullptr; }
    };
    auto resid = [&](const T* X, int K, const T* W, const float* b, bool defer) -> int {
      GemmArgs g;
      g.X = X; g.ldx = K; g.W = W; g.bias = b; g.M = R; g.N = n; g.K = K; g.out_f32 = xc; g.ldo = n;
      g.p1_defer = defer;
      TRY(p1(g, EPI_RESID, false));
      if (defer) pend = b;
      return 0;
    };
    for (int l = 0; l < Ld; ++l) {
      auto& e = dec[l];
      // self-attention block: q, k, v of LN1(x) (k / v straight into the cache)
      GemmArgs g;
      g.W = e.wqkv; g.bias = e.bqkv; g.M = R; g.N = 3 * n; g.K = n;
      ln_in(g, e.ln1_g, e.ln1_b);
      g.out = q_d; g.ldo = n; g.hs_state = n; g.hs_heads = nh;
      g.row_win = rw; g.row_slot = rs; g.row_pos = rp; g.kc = kc[l]; g.vc = vc[l]; g.kv_beams = Gcap; g.kv_ctx = CTX;
      TRY(p1(g, EPI_QKV_DEC, true));
      ln_done();
      launch_self_attn<T>(q_d, n, kc[l], vc[l], rw, rs, rp, A, ancG, Gcap, nh, CTX, att_d, n, R, st);
      TRY(resid(att_d, n, e.wo, e.bo, false));  // deferring it measured +1.0 us on cross-q, -0.2 here
      // cross-attention block
      XQPart xq = step_xq(ancG);
      if (xq_proj1_active(ancG) && !pend) {
        // round 6: no cross-q k_proj1 launch; the cross-attention normalises the window's
        // fp32 rows and projects its query itself
        xq.qx = xc; xq.qw = e.wqx; xq.bias = e.bqx; xq.ln_g = e.lnx_g; xq.ln_b = e.lnx_b; xq.ln_eps = 1e-5f;
        if (xq_proj1_mode() == 2) {
          xq.q_part = xq1_part; xq.q_cnt = xq1_cnt;
        } else if (xq_frag_on()) {
          xq.qwf = e.wqx_f;
        }
      } else {
        g = GemmArgs();
        g.W = e.wqx; g.bias = e.bqx; g.M = R; g.N = n; g.K = n;
        ln_in(g, e.lnx_g, e.lnx_b);
        g.out = q_d; g.ldo = n;
        TRY(p1(g, EPI_STORE, true));
        ln_done();
      }
      const T* ck = ckv + (size_t)(2 * l) * Wcap * TKP * n;
      const T* cv = ckv + (size_t)(2 * l + 1) * Wcap * TKP * n;
      launch_cross_attn<T>(q_d, n, ck, cv, 1500, nh, NSPLIT, nwin, wr0, wnr, wsl, (int64_t)TKP * n, po, pm, pl, att_d,
                           n, R, nullptr, nullptr, 0, st, xq);
      // (not deferred: fc1's 16-wave LayerNorm prologue has no registers for two more row copies)
      TRY(resid(att_d, n, e.wox, e.box, false));
      // MLP; the last layer's fc2 reduces in-launch (the final LayerNorm reads x)
      g = GemmArgs();
      g.W = e.w1; g.bias = e.b1; g.M = R; g.N = 4 * n; g.K = n;
      ln_in(g, e.ln2_g, e.ln2_b);
      g.out = hm_d; g.ldo = 4 * n;
      TRY(p1(g, EPI_STORE_GELU, true));
      ln_done();
      TRY(resid(hm_d, 4 * n, e.w2, e.b2, l + 1 < Ld));
    }
    // the final LayerNorm runs in the vocabulary kernel's prologue (vocab(), final_x)
    final_x = xc;
    return 0;
  }

  // logits = LN(x) E^T for R rows of xn_d (optionally gathered by rows_sel)
  // (decoder.py:238-240, 316-320)
  // (after dec_layers_p1, final_x names the fp32 residual rows whose final LayerNorm
  // k_vocab_small computes itself: no separate LayerNorm launch per token)
  const float* final_x = nullptr;
  int vocab(const int* rows_sel, int R, float* out) {
    GemmArgs g;
    g.out_f32 = out; g.ldo = V; g.x_rows = rows_sel;
    // after dec_layers_p1, xn_d does not hold the final LayerNorm: only the prologue path
    // (every row, no gather) is valid there
    if (final_x && rows_sel) return fail(-20, "vocab: a row gather after the k_proj1 layers (xn_d not written)");
    if (final_x) {
      g.xf32 = final_x; g.ln_g = ln_g; g.ln_b = ln_b; g.ln_eps = 1e-5f;
    }
    return gemm(xn_d, ns, E, nullptr, R, V, ns, EPI_F32_COLS, g);
  }

  // ------------------------------------------------------------ decoding
  int set_opts(const wh_decode_opts* o) {
    if (o->group < 1 || o->group > Gcap) return fail(-11, "group exceeds context max_group");
    O = DecOpts();
    O.V = V; O.eot = o->eot; O.ts_begin = o->timestamp_begin; O.no_ts = o->no_timestamps;
    O.n_blank = std::min(o->n_blank, 3);
    for (int i = 0; i < O.n_blank; ++i) O.blank[i] = o->blank[i];
    O.blank[O.n_blank] = o->eot;  // SuppressBlank masks encode(" ") + [eot]
    O.n_blank += 1;
    O.suppress_blank = o->suppress_blank; O.timestamps = o->timestamps; O.max_initial = o->max_initial;
    O.beam = o->beam; O.sample_len = o->sample_len; O.n_ctx = CTX; O.temperature = o->temperature;
    h_seed = o->seed;
    std::vector<unsigned> mask((V + 31) / 32, 0u);
    for (int i = 0; i < o->n_suppress; ++i) {
      const int t = o->suppress[i];
      if (t >= 0 && t < V) mask[t >> 5] |= 1u << (t & 31);
    }
    HIPCHK(hipMemcpyAsync(suppress, mask.data(), mask.size() * 4, hipMemcpyHostToDevice, st));
    O.suppress = o->n_suppress > 0 ? suppress : nullptr;
    // max_candidates = round(beam_size * patience) (decoding.py:339): Python rounds half
    // to even; the host passes its own value, else nearbyint (default mode: half to even)
    maxc = !o->beam ? 0
           : o->max_candidates > 0 ? o->max_candidates
                                   : (int)std::nearbyint((double)o->group * (o->patience > 0 ? o->patience : 1.0));
    if (o->beam && (maxc < 1 || maxc > 16)) return fail(-11, "max_candidates out of range (1..16)");
    S.G = o->group;
    S.maxc = 16;
    return 0;
  }

  int prefill(int w0, int nw, const std::vector<int>& toks, const std::vector<int>& nin, const int* sot_index,
              bool first_update_rows) {
    // rows of windows w0..w0+nw-1, all in beam slot 0; cross attention per window
    std::vector<int> rt, rp, rw, rs, wr0(nw), wnr(nw), wsl(nw), sel;
    for (int i = 0; i < nw; ++i) {
      wr0[i] = (int)rt.size();
      wnr[i] = nin[i];
      wsl[i] = win_slots[w0 + i];
      for (int p = 0; p < nin[i]; ++p) {
        rt.push_back(toks[(size_t)i * HCTX + p]);
        rp.push_back(p);
        rw.push_back(w0 + i);
        rs.push_back(0);
      }
      sel.push_back(wr0[i] + sot_index[w0 + i]);
      sel.push_back(wr0[i] + nin[i] - 1);
    }
    const int R = (int)rt.size();
    HIPCHK(hipMemcpyAsync(row_tok, rt.data(), R * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(row_pos, rp.data(), R * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(row_win, rw.data(), R * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(row_slot, rs.data(), R * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(win_row0, wr0.data(), nw * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(win_nrows, wnr.data(), nw * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(win_slot, wsl.data(), nw * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(rows_in, sel.data(), sel.size() * 4, hipMemcpyHostToDevice, st));
    launch_embed<T>(E, Pdec, ns, row_tok, row_pos, nullptr, nullptr, 1, HCTX, CTX - 1, x_d, R, st);
    TRY(dec_layers(R, row_win, row_slot, row_pos, S.G, nw, win_row0, win_nrows, win_slot, nullptr, nullptr, 0));
    TRY(vocab(rows_in, 2 * nw, logits2 + (size_t)2 * w0 * V));
    (void)first_update_rows;
    // the host vectors must outlive the async copies
    HIPCHK(hipStreamSynchronize(st));
    return 0;
  }

  // prefill of the initial tokens of n_win windows (G rows each, sharing beam slot 0 of
  // the self-KV), the decode state for step len = n_init[w], and the static step-row
  // metadata.  Leaves the sot_index / last-row logits of window w in logits2 rows
  // 2w / 2w+1 (and, when no_speech >= 0, its no-speech probability in nsp).
  // Window w reads the audio features / cross-KV of slot slots[w] (identity when null):
  // a temperature fallback decodes the windows that still need work straight from the
  // slots that hold them, without re-running the encoder.
  std::vector<int> h_len;      // host mirror of S.len for the per-step ABI
  std::vector<int> win_slots;  // cross-KV slot of each decode window
  unsigned long long h_seed = 0;
  int begin_batch(int n_win, int G, const int* init, const int* n_init, int max_init, const int* sot_index,
                  int no_speech, const int* slots = nullptr) {
    if (!finalized) return fail(-9, "weights not finalized");
    // no usable batch until this one is fully set up: a failure below leaves neither the
    // device loop nor the per-step ABI (wh_step / wh_reorder_kv) a half-written batch
    cur_nwin = 0;
    step_api = false;
    if (n_win < 1 || n_win > Wcap) return fail(-11, "n_win out of range");
    if (G < 1 || G > Gcap) return fail(-11, "group exceeds context max_group");
    win_slots.resize(n_win);
    for (int w = 0; w < n_win; ++w) {
      win_slots[w] = slots ? slots[w] : w;
      if (win_slots[w] < 0 || win_slots[w] >= Wcap) return fail(-11, "window slot out of range");
    }
    // host-side initial state
    std::vector<int> hist((size_t)n_win * Gcap * HCTX, 0), anc((size_t)n_win * Gcap * CTX, 0), toks((size_t)n_win * HCTX, 0);
    std::vector<int> nin(n_win), lens(n_win), zeros(n_win, 0);
    for (int w = 0; w < n_win; ++w) {
      nin[w] = n_init[w];
      if (nin[w] < 1 || nin[w] > CTX - 1) return fail(-11, "initial token count out of range");
      if (sot_index[w] < 0 || sot_index[w] >= nin[w]) return fail(-11, "bad sot_index");
      for (int p = 0; p < nin[w]; ++p) {
        const int t = init[(size_t)w * max_init + p];
        if (t < 0 || t >= V) return fail(-11, "initial token out of vocabulary");
        toks[(size_t)w * HCTX + p] = t;
      }
    }
    S.G = G;
    // history / ancestry laid out with the runtime group G ([w][G][..])
    for (int w = 0; w < n_win; ++w)
      for (int b = 0; b < G; ++b) {
        for (int p = 0; p < nin[w]; ++p) hist[((size_t)w * G + b) * HCTX + p] = toks[(size_t)w * HCTX + p];
        for (int p = 0; p < CTX; ++p) anc[((size_t)w * G + b) * CTX + p] = p < nin[w] ? 0 : b;
      }
    // prefill (anc must be in place first: prefill rows read slot 0 through it)
    HIPCHK(hipMemcpyAsync(S.anc, anc.data(), (size_t)n_win * G * CTX * 4, hipMemcpyHostToDevice, st));
    // prefill runs with kv_beams = Gcap layout; rows use slot 0
    for (int w0 = 0; w0 < n_win;) {
      int rows = 0, nw = 0;
      while (w0 + nw < n_win && (nw == 0 || rows + nin[w0 + nw] <= PRE)) rows += nin[w0 + nw++];
      if (rows > PRE) return fail(-11, "prefill rows exceed buffer");
      std::vector<int> sub_toks(toks.begin() + (size_t)w0 * HCTX, toks.begin() + (size_t)(w0 + nw) * HCTX);
      std::vector<int> sub_n(nin.begin() + w0, nin.begin() + w0 + nw);
      TRY(prefill(w0, nw, sub_toks, sub_n, sot_index, true));
      w0 += nw;
    }
    // no_speech prob from the sot row of each window (decoding.py:716-720)
    if (no_speech >= 0) launch_no_speech(logits2, 2 * V, n_win, V, no_speech, nsp, st);
    // last-row logits replicated to the G rows of each window
    std::vector<int> src(n_win);
    for (int w = 0; w < n_win; ++w) src[w] = 2 * w + 1;
    HIPCHK(hipMemcpyAsync(src_rows, src.data(), n_win * 4, hipMemcpyHostToDevice, st));
    launch_broadcast_rows(logits2, V, src_rows, logits, V, G, n_win, V, st);
    // decode state
    HIPCHK(hipMemcpyAsync(S.hist, hist.data(), (size_t)n_win * G * HCTX * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(S.len, nin.data(), n_win * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(S.sample_begin, nin.data(), n_win * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemsetAsync(S.step, 0, n_win * 4, st));
    HIPCHK(hipMemsetAsync(S.done, 0, n_win * 4, st));
    HIPCHK(hipMemsetAsync(S.fin_n, 0, n_win * 4, st));
    HIPCHK(hipMemsetAsync(S.sum_lp, 0, n_win * G * 4, st));
    HIPCHK(hipMemcpyAsync(S.seed, &h_seed, 8, hipMemcpyHostToDevice, st));
    // static step-row metadata: row r = w*G + b
    std::vector<int> srw(n_win * G), srs(n_win * G), swr0(n_win), swnr(n_win, G), swsl(n_win);
    for (int w = 0; w < n_win; ++w) {
      swr0[w] = w * G;
      swsl[w] = win_slots[w];
      for (int b = 0; b < G; ++b) { srw[w * G + b] = w; srs[w * G + b] = b; }
    }
    HIPCHK(hipMemcpyAsync(st_row_win, srw.data(), srw.size() * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(st_row_slot, srs.data(), srs.size() * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(st_win_row0, swr0.data(), n_win * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(st_win_nrows, swnr.data(), n_win * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(st_win_slot, swsl.data(), n_win * 4, hipMemcpyHostToDevice, st));
    // the self-KV cache uses [w][Gcap][..] slots; the anc table uses [w][G][..]
    cur_nwin = n_win;
    cur_G = G;
    h_len = nin;
    // the host vectors above must outlive the async copies
    HIPCHK(hipStreamSynchronize(st));
    return 0;
  }

  int decode_begin(int n_win, const wh_decode_opts* o, const int* init, const int* n_init, int max_init,
                   const int* sot_index, const int* slots) override {
    if (!finalized) return fail(-9, "weights not finalized");
    if (n_win < 1 || n_win > Wcap) return fail(-11, "n_win out of range");
    TRY(set_opts(o));
    HIPCHK(hipEventRecord(tm.a, st));
    TRY(begin_batch(n_win, o->group, init, n_init, max_init, sot_index, o->no_speech, slots));
    S.maxc = std::max(maxc, 1);
    maxc_stride = S.maxc;
    step_api = false;
    // first update on the prefill logits (decoding.py:713-733, i == 0); the merge also
    // embeds each row's new token: the first step's input rows
    launch_select_merge(logits, V, S, O, n_win, st, merge_embed());
    rows_dirty = false;
    HIPCHK(hipEventRecord(tm.b, st));
    HIPCHK(hipStreamSynchronize(st));
    TRY(launch_status(__func__));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, tm.a, tm.b));
    stats[2] += ms;
    return 0;
  }

  // The device loop's step input rows (x_d, row_pos) are written by the previous update's
  // merge (no k_embed per token).  Any other use of those buffers between two
  // decode_steps calls (a first pass for alignment or prefill logits, a timing stage)
  // sets rows_dirty, and the next decode_steps re-embeds every row once from the decode
  // state (S.hist, S.len) before its first step.
  bool rows_dirty = false;
  void restore_rows() {
    if (!rows_dirty || cur_nwin < 1 || step_api) return;
    launch_embed<T>(E, Pdec, ns, nullptr, row_pos, S.hist, S.len, cur_G, HCTX, CTX - 1, x_d, cur_nwin * cur_G, st);
    rows_dirty = false;
  }
  // k_merge writes the next step's input rows (x_d, row_pos): no k_embed launch per token
  MergeEmbed merge_embed() const {
    MergeEmbed em;
    em.E = E; em.P = Pdec; em.x = x_d; em.row_pos = row_pos; em.n = ns; em.pmax = CTX - 1; em.half = sizeof(T) == 2;
    return em;
  }
  // one decoder step for the current batch (graph body); its input rows were embedded by
  // the previous update's k_merge (decode_begin's first update for the first step)
  int step_body() {
    const int R = cur_nwin * cur_G;
    TRY(dec_layers(R, st_row_win, st_row_slot, row_pos, cur_G, cur_nwin, st_win_row0, st_win_nrows, st_win_slot,
                   nullptr, nullptr, 0, true));
    if (final_x && cur_nwin == 1 && sizeof(T) == 2) {
      // one window (k_proj1 layers): vocabulary, selection and merge in one launch
      GemmArgs g;
      g.X = xn_d; g.ldx = ns; g.W = E; g.M = R; g.N = V; g.K = ns; g.out_f32 = logits; g.ldo = V;
      g.xf32 = final_x; g.ln_g = ln_g; g.ln_b = ln_b; g.ln_eps = 1e-5f;
      const int rc = launch_vocab_select(g, S, O, merge_embed(), vs_rec, vs_cnt, st);
      if (rc == 0) return 0;
      if (rc != -1) return fail(-20, "k_vocab_sel launch failed code " + std::to_string(rc));
    }
    TRY(vocab(nullptr, R, logits));
    launch_select_merge(logits, V, S, O, cur_nwin, st, merge_embed());
    return 0;
  }

  // ------------------------------------------------------------ per-step ABI
  // The reference's native boundary hands every step's logits to the host and reorders
  // the self-KV cache when the host asks (decoder256Predict coreml.mm:279-327,
  // decoder1Predict :404-444, rearrange_mkv :251-277), so its Python DecodingTask keeps
  // filters and beam search (decoding.py:707-737).  These entry points serve that
  // caller: the same decoder step as the graph body, without the device token selection.
  bool step_api = false;
  int step_prefill(int n_win, int G, const int* init, const int* n_init, int max_init, const int* sot_index,
                   float* lg) override {
    HIPCHK(hipEventRecord(tm.a, st));
    TRY(begin_batch(n_win, G, init, n_init, max_init, sot_index, -1));
    step_api = true;
    if (lg) HIPCHK(hipMemcpyAsync(lg, logits2, (size_t)2 * n_win * V * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipEventRecord(tm.b, st));
    HIPCHK(hipStreamSynchronize(st));
    TRY(launch_status(__func__));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, tm.a, tm.b));
    stats[2] += ms;
    return 0;
  }

  int step_tokens(const int* tok, const int* offsets, float* lg) override {
    if (!step_api || cur_nwin < 1) return fail(-13, "no per-step batch (call wh_prefill first)");
    const int R = cur_nwin * cur_G;
    for (int r = 0; r < R; ++r)
      if (tok[r] < 0 || tok[r] >= V) return fail(-13, "step token out of vocabulary");
    for (int w = 0; w < cur_nwin; ++w) {
      if (h_len[w] >= CTX) return fail(-13, "text context full (448 positions)");
      if (offsets && offsets[w] != h_len[w])
        return fail(-13, "text_offset " + std::to_string(offsets[w]) + " of window " + std::to_string(w) +
                             " != cached length " + std::to_string(h_len[w]));
    }
    HIPCHK(hipEventRecord(tm.a, st));
    HIPCHK(hipMemcpyAsync(rows_in, tok, R * 4, hipMemcpyHostToDevice, st));
    launch_append_tokens(S, rows_in, cur_nwin, st);
    launch_embed<T>(E, Pdec, ns, nullptr, row_pos, S.hist, S.len, cur_G, HCTX, CTX - 1, x_d, R, st);
    TRY(dec_layers(R, st_row_win, st_row_slot, row_pos, cur_G, cur_nwin, st_win_row0, st_win_nrows, st_win_slot,
                   nullptr, nullptr, 0, true));
    TRY(vocab(nullptr, R, logits));
    if (lg) HIPCHK(hipMemcpyAsync(lg, logits, (size_t)R * V * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipEventRecord(tm.b, st));
    HIPCHK(hipStreamSynchronize(st));  // the host token buffer must outlive its copy
    TRY(launch_status(__func__));
    for (auto& l : h_len) ++l;
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, tm.a, tm.b));
    stats[3] += ms;
    stats[4] += 1;
    return 0;
  }

  int reorder_kv(const int* src) override {
    if (!step_api || cur_nwin < 1) return fail(-13, "no per-step batch (call wh_prefill first)");
    const int R = cur_nwin * cur_G;
    for (int r = 0; r < R; ++r)
      if (src[r] / cur_G != r / cur_G || src[r] < 0)
        return fail(-13, "source row " + std::to_string(src[r]) + " of row " + std::to_string(r) +
                             " is not a row of the same window");
    HIPCHK(hipMemcpyAsync(src_rows, src, R * 4, hipMemcpyHostToDevice, st));
    launch_reorder_rows(S, src_rows, cur_nwin, st);
    HIPCHK(hipStreamSynchronize(st));
    TRY(launch_status(__func__));
    return 0;
  }

  int ensure_graph() {
    std::vector<char> key(sizeof(DecOpts) + sizeof(DecState) + 8);
    memcpy(key.data(), &O, sizeof(DecOpts));
    memcpy(key.data() + sizeof(DecOpts), &S, sizeof(DecState));
    memcpy(key.data() + sizeof(DecOpts) + sizeof(DecState), &cur_nwin, 4);
    memcpy(key.data() + sizeof(DecOpts) + sizeof(DecState) + 4, &cur_G, 4);
    if (gexec && key == graph_key) return 0;
    if (gexec) { hipGraphExecDestroy(gexec); gexec = nullptr; }
    if (graph) { hipGraphDestroy(graph); graph = nullptr; }
    if (xkv_pf_wg() > 0) TRY(kv_pull_setup());  // (no stream / event creation or hipMalloc under capture)
    HIPCHK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    const int rc = step_body();
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(st, &g);
    if (rc) { if (g) hipGraphDestroy(g); return rc; }
    if (e != hipSuccess) return fail(-12, std::string("graph capture: ") + hipGetErrorString(e));
    graph = g;
    HIPCHK(hipGraphInstantiate(&gexec, graph, nullptr, nullptr, 0));
    graph_key = key;
    return 0;
  }

  // WHISPER_HIP_XQ=0 keeps the separate cross-query reduce (A/B switch)
  const bool xq_fused = [] {
    const char* e = tune_env("WHISPER_HIP_XQ");
    return !(e && e[0] == '0');
  }();
  // round 6: the step's cross-attention query projected inside k_xattn_seg (no cross-q
  // k_proj launch) wherever xattn_fused_q serves the shape; WHISPER_HIP_XQP=0 keeps the
  // split-K projection + slabs (A/B switch)
  static bool xq_proj_on() {
    static const bool on = [] {
      const char* e = tune_env("WHISPER_HIP_XQP");
      return !(e && e[0] == '0');
    }();
    return on;
  }
  // the fragment-ordered W_q copy for it (WHISPER_HIP_XQ_FRAG=0: the [n][n] rows, A/B)
  static bool xq_frag_on() {
    static const bool on = [] {
      const char* e = tune_env("WHISPER_HIP_XQ_FRAG");
      return !(e && e[0] == '0');
    }();
    return on;
  }
  bool xq_proj_active(int rows_per_window) const {
    return xq_proj_on() && xattn_fused_q(ns, rows_per_window, (int)sizeof(T));
  }
  // and in the single-window step (k_proj1 layers: the LayerNorm too): tuning build only,
  // WHISPER_HIP_XQP1=1.  Measured slower (profiles/r06/ab_xqp1_single_window.txt): at one
  // window 240 workgroups each ingest the 164 KB W_q slice of their head before any tile can
  // run, and the cross-attention launch grows 6.1 -> 17.4 us against the 5-7 us the cross-q
  // k_proj1 launch and its boundary cost (turbo step graph 0.274 -> 0.300 ms)
  // WHISPER_HIP_XQP1=2: the projection split over each pair's 8 workgroups (k_xattn_seg QV 6)
  static int xq_proj1_mode() {
    static const int v = [] {
      const char* e = tune_env("WHISPER_HIP_XQP1");
      return e ? atoi(e) : 0;
    }();
    return v;
  }
  static bool xq_proj1_on() { return xq_proj1_mode() > 0; }
  bool xq_proj1_active(int rows_per_window) const { return xq_proj1_on() && xq_proj_active(rows_per_window); }

  // WHISPER_HIP_EAGER=1 launches the step kernels directly instead of replaying the
  // captured graph (same kernels; used under profilers that do not follow graphs)
  bool eager() const {
    const char* e = tune_env("WHISPER_HIP_EAGER");
    return e && e[0] == '1';
  }

  int launch_step() {
    if (eager()) return step_body();
    HIPCHK(hipGraphLaunch(gexec, st));
    return 0;
  }

  int decode_steps(int max_steps, int* n_done) override {
    if (cur_nwin < 1) return fail(-13, "no decode in progress");
    if (step_api) return fail(-13, "the batch was begun with wh_prefill (per-step mode): use wh_step");
    if (!eager()) TRY(ensure_graph());
    HIPCHK(hipEventRecord(tm.a, st));
    restore_rows();
    int steps = 0, done = 0;
    static const int chunk = [] {  // WHISPER_HIP_POLL_CHUNK: steps per done-flag poll (A/B)
      const char* e = tune_env("WHISPER_HIP_POLL_CHUNK");
      const int v = e ? atoi(e) : 8;
      return v < 1 ? 1 : v;
    }();
    // chunks of `chunk` steps, each followed by an async copy of the done flags; the
    // next chunk is queued before the host waits for the previous chunk's flags, so
    // the GPU never idles on the poll (at most one chunk of no-op steps after the last
    // window finishes: finished windows' rows are clamped and skipped by the selection)
    auto queue_chunk = [&](int b) -> int {
      const int k = std::min(chunk, max_steps - steps);
      for (int i = 0; i < k; ++i) TRY(launch_step());
      steps += k;
      HIPCHK(hipMemcpyAsync(h_done + b * Wcap, S.done, cur_nwin * 4, hipMemcpyDeviceToHost, st));
      HIPCHK(hipEventRecord(poll_ev[b], st));
      return k;
    };
    auto tc = std::chrono::steady_clock::now();
    int b = 0, kq[2] = {0, 0};
    kq[0] = queue_chunk(0);
    if (kq[0] < 0) return kq[0];
    while (true) {
      const int nb = b ^ 1;
      kq[nb] = steps < max_steps ? queue_chunk(nb) : 0;
      if (kq[nb] < 0) return kq[nb];
      HIPCHK(hipEventSynchronize(poll_ev[b]));
      // per-token wall time (graph launches + done poll, pipelined), for the p50
      const auto now = std::chrono::steady_clock::now();
      token_ms.push_back((float)(std::chrono::duration<double, std::milli>(now - tc).count() / kq[b]));
      tc = now;
      done = 0;
      for (int w = 0; w < cur_nwin; ++w) done += h_done[b * Wcap + w] != 0;
      if (done == cur_nwin || kq[nb] == 0) break;
      b = nb;
    }
    HIPCHK(hipEventRecord(tm.b, st));
    HIPCHK(hipStreamSynchronize(st));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, tm.a, tm.b));
    stats[3] += ms;
    stats[4] += steps;
    *n_done = done;
    return 0;
  }

  int decode_read(int slot, int* tokens, float* slp, int* len, int* fin_n, int* fin_tok, int* fin_len,
                  float* fin_score, float* nspo) override {
    if (slot < 0 || slot >= cur_nwin) return fail(-14, "slot");
    const int G = cur_G;
    HIPCHK(hipStreamSynchronize(st));
    if (tokens) HIPCHK(hipMemcpy(tokens, S.hist + (size_t)slot * G * HCTX, (size_t)G * HCTX * 4, hipMemcpyDeviceToHost));
    if (slp) HIPCHK(hipMemcpy(slp, S.sum_lp + slot * G, G * 4, hipMemcpyDeviceToHost));
    if (len) HIPCHK(hipMemcpy(len, S.len + slot, 4, hipMemcpyDeviceToHost));
    if (fin_n) HIPCHK(hipMemcpy(fin_n, S.fin_n + slot, 4, hipMemcpyDeviceToHost));
    const int mc = S.maxc;
    if (fin_tok) HIPCHK(hipMemcpy(fin_tok, S.fin_tok + (size_t)slot * mc * HCTX, (size_t)mc * HCTX * 4, hipMemcpyDeviceToHost));
    if (fin_len) HIPCHK(hipMemcpy(fin_len, S.fin_len + slot * mc, mc * 4, hipMemcpyDeviceToHost));
    if (fin_score) HIPCHK(hipMemcpy(fin_score, S.fin_score + slot * mc, mc * 4, hipMemcpyDeviceToHost));
    if (nspo) HIPCHK(hipMemcpy(nspo, nsp + slot, 4, hipMemcpyDeviceToHost));
    return 0;
  }

  // Whisper.forward (model.py:110-119): all-row logits of a first pass for one window,
  // optional raw cross-QK of alignment heads.  Uses beam slot 0 of `slot` and the anc
  // table with a 1-beam layout; call it when no decode of that slot is in flight.
  // first pass of `n` tokens at offset 0 for one window slot (beam slot 0, a 1-beam
  // anc layout), optional raw cross-QK of the alignment heads into d_aqk [na][n][1500];
  // on return xn_d holds the final LayerNorm of every row.  The host vectors are kept
  // alive in `keep` until the caller synchronises.
  // A first pass writes beam slot 0's self-KV rows of its slot: refused on a slot that the
  // live device-loop batch is still decoding (its done flag unset), which it would corrupt.
  // Slots outside the batch, finished windows and the per-step ABI's batch are allowed.
  int check_slot_idle(int slot) {
    if (cur_nwin < 1 || step_api) return 0;
    for (int w = 0; w < cur_nwin; ++w)
      if (win_slots[w] == slot) {
        int d = 0;
        HIPCHK(hipMemcpyAsync(&d, S.done + w, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (!d)
          return fail(-15, "slot " + std::to_string(slot) + " is still decoding (window " + std::to_string(w) +
                               " of the current batch): a first pass would overwrite its self-KV rows");
      }
    return 0;
  }

  int first_pass(int slot, const int* tokens, int n, const int* ah, int na, float* d_aqk,
                 std::vector<std::vector<int>>& keep) {
    if (!finalized) return fail(-9, "weights not finalized");
    if (slot < 0 || slot >= Wcap || n < 1 || n > CTX) return fail(-15, "bad slot or token count");
    TRY(check_slot_idle(slot));
    rows_dirty = true;  // the first pass runs its rows through x_d / row_pos
    for (int i = 0; i < n; ++i)
      if (tokens[i] < 0 || tokens[i] >= V) return fail(-15, "token out of vocabulary");
    keep.assign(9, {});
    auto& rt = keep[0]; auto& rp = keep[1]; auto& rw = keep[2]; auto& rs = keep[3];
    rt.assign(tokens, tokens + n); rp.resize(n); rw.assign(n, slot); rs.assign(n, 0);
    keep[4] = {0}; keep[5] = {n}; keep[6] = {slot};
    for (int i = 0; i < n; ++i) rp[i] = i;
    auto& map = keep[8];
    map.assign((size_t)Ld * nh, -1);
    for (int i = 0; i < na; ++i)
      if (ah[i] >= 0 && ah[i] < Ld * nh) map[ah[i]] = i;
    HIPCHK(hipMemcpyAsync(row_tok, rt.data(), n * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(row_pos, rp.data(), n * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(row_win, rw.data(), n * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(row_slot, rs.data(), n * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(win_row0, keep[4].data(), 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(win_nrows, keep[5].data(), 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(win_slot, keep[6].data(), 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(qk_map, map.data(), map.size() * 4, hipMemcpyHostToDevice, st));
    launch_embed<T>(E, Pdec, ns, row_tok, row_pos, nullptr, nullptr, 1, HCTX, CTX - 1, x_d, n, st);
    // its own all-zero ancestry table: the decode's S.anc ([w][G][CTX]) stays untouched,
    // so a device-loop decode of other slots can continue afterwards
    return dec_layers(n, row_win, row_slot, row_pos, 1, 1, win_row0, win_nrows, win_slot, d_aqk,
                      d_aqk ? qk_map : nullptr, n, false, fp_anc);
  }

  // grow-only device scratch for the alignment / prefill readbacks
  char* scratch = nullptr;
  size_t scratch_cap = 0;
  int ensure_scratch(size_t bytes) {
    if (bytes <= scratch_cap) return 0;
    HIPCHK(hipStreamSynchronize(st));
    if (scratch) HIPCHK(hipFree(scratch));
    scratch = nullptr;
    scratch_cap = 0;
    HIPCHK(hipMalloc((void**)&scratch, bytes));
    scratch_cap = bytes;
    return 0;
  }

  // find_alignment's device half (timing.py:163-231) for a batch of windows: window w
  // is sot_sequence + [no_timestamps] + text + [eot] (n_tokens[w] ids at tokens[sum of
  // the previous n_tokens]) over the audio features of slots[w].  The windows' first
  // passes run together (up to PRE rows per pass, cross-QK of the alignment
  // heads captured), then the text tokens' probabilities, the filtered head-mean
  // matrices and one DTW workgroup per window (all DTWs of a pass in one launch).
  // Outputs are concatenated in window order: probs [T_w], paths [2][T_w+1+F_w],
  // plens [n_win].
  int align_batch(int n_win, const int* slots, const int* tokens, const int* n_tokens, int n_sot,
                  const int* num_frames, const int* ah, int na, int medfilt, float* probs, int* paths,
                  int* plens) override {
    if (!finalized) return fail(-9, "weights not finalized");
    if (n_win < 1) return fail(-15, "align: no windows");
    if (na < 1 || na > Ld * nh) return fail(-15, "align: alignment head count");
    if (medfilt < 1 || medfilt > 15 || medfilt % 2 == 0) return fail(-15, "align: medfilt_width must be odd <= 15");
    std::vector<int64_t> tok_off(n_win + 1, 0), prob_off(n_win + 1, 0), path_off(n_win + 1, 0), mat_off(n_win + 1, 0),
        tr_off(n_win + 1, 0);
    int rows_max = 0;
    for (int w = 0; w < n_win; ++w) {
      const int n = n_tokens[w], Tt = n - n_sot - 2, F = num_frames[w] / 2;
      if (n_sot < 1 || Tt < 1) return fail(-15, "align: need sot_sequence + no_timestamps + >= 1 text token + eot");
      if (n > CTX) return fail(-15, "align: more than 448 tokens");
      if (F < 1 || F > 1500) return fail(-15, "align: num_frames out of range");
      if (slots[w] < 0 || slots[w] >= Wcap) return fail(-15, "align: bad slot");
      TRY(check_slot_idle(slots[w]));
      const int N = Tt + 1;
      tok_off[w + 1] = tok_off[w] + n;
      prob_off[w + 1] = prob_off[w] + Tt;
      path_off[w + 1] = path_off[w] + 2 * (N + F);
      mat_off[w + 1] = mat_off[w] + ((int64_t)N * F + 63) / 64 * 64;
      tr_off[w + 1] = tr_off[w] + (dtw_trace_bytes(N, F) + 255) / 256 * 256;
      rows_max = std::max(rows_max, n);
    }
    // pass grouping: consecutive windows while the rows fit PRE and the cross-QK budget
    const int64_t qk_row = (int64_t)na * 1500 * 4;
    const int cap = (int)std::max<int64_t>(rows_max, std::min<int64_t>(PRE, ((int64_t)1 << 30) / qk_row));
    auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
    const size_t b_qk = al((size_t)qk_row * cap), b_lg = al((size_t)128 * V * 4), b_mat = al(mat_off[n_win] * 4),
                 b_tr = al(tr_off[n_win]), b_path = al(path_off[n_win] * 4), b_pr = al(prob_off[n_win] * 4 + 16),
                 b_pl = al((size_t)n_win * 4), b_jobs = al((size_t)n_win * sizeof(DtwJob));
    TRY(ensure_scratch(b_qk + b_lg + b_mat + b_tr + b_path + 2 * b_pr + b_pl + b_jobs));
    char* p = scratch;
    float* d_qk = (float*)p; p += b_qk;
    float* d_lg = (float*)p; p += b_lg;
    float* d_mat = (float*)p; p += b_mat;
    char* d_tr = p; p += b_tr;
    int* d_path = (int*)p; p += b_path;
    float* d_probs = (float*)p; p += b_pr;
    int* d_ptok = (int*)p; p += b_pr;
    int* d_plen = (int*)p; p += b_pl;
    DtwJob* d_jobs = (DtwJob*)p;

    // token of every probability row (timing.py:191: text_tokens[k])
    std::vector<int> ptok(prob_off[n_win]);
    for (int w = 0; w < n_win; ++w)
      for (int k = 0; k < prob_off[w + 1] - prob_off[w]; ++k) ptok[prob_off[w] + k] = tokens[tok_off[w] + n_sot + 1 + k];
    HIPCHK(hipMemcpyAsync(d_ptok, ptok.data(), ptok.size() * 4, hipMemcpyHostToDevice, st));
    std::vector<int> map((size_t)Ld * nh, -1);
    for (int i = 0; i < na; ++i)
      if (ah[i] >= 0 && ah[i] < Ld * nh) map[ah[i]] = i;
    HIPCHK(hipMemcpyAsync(qk_map, map.data(), map.size() * 4, hipMemcpyHostToDevice, st));
    std::vector<DtwJob> jobs(n_win);
    const int eot = tokens[tok_off[1] - 1];
    for (int w0 = 0; w0 < n_win;) {
      int nw = 0, R = 0;
      while (w0 + nw < n_win && (nw == 0 || R + n_tokens[w0 + nw] <= cap)) R += n_tokens[w0 + nw++];
      // rows of this pass: window slot, beam slot 0, position
      std::vector<int> rt(R), rp(R), rw(R), rs(R, 0), wr0(nw), wnr(nw), wsl(nw), sel;
      int r = 0;
      for (int i = 0; i < nw; ++i) {
        const int w = w0 + i, n = n_tokens[w];
        wr0[i] = r; wnr[i] = n; wsl[i] = slots[w];
        for (int q = 0; q < n; ++q, ++r) { rt[r] = tokens[tok_off[w] + q]; rp[r] = q; rw[r] = slots[w]; }
        for (int k = 0; k < n - n_sot - 2; ++k) sel.push_back(wr0[i] + n_sot + k);
        if (tokens[tok_off[w] + n - 1] != eot) return fail(-15, "align: windows must end with the same eot");
      }
      for (int q = 0; q < R; ++q)
        if (rt[q] < 0 || rt[q] >= V) return fail(-15, "align: token out of vocabulary");
      // set before the first upload into row_pos / x_d (as first_pass does): a failing copy
      // below must still make the next decode_steps re-embed its rows
      rows_dirty = true;  // this first pass runs its rows through x_d / row_pos
      HIPCHK(hipMemcpyAsync(row_tok, rt.data(), R * 4, hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync(row_pos, rp.data(), R * 4, hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync(row_win, rw.data(), R * 4, hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync(row_slot, rs.data(), R * 4, hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync(win_row0, wr0.data(), nw * 4, hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync(win_nrows, wnr.data(), nw * 4, hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync(win_slot, wsl.data(), nw * 4, hipMemcpyHostToDevice, st));
      launch_embed<T>(E, Pdec, ns, row_tok, row_pos, nullptr, nullptr, 1, HCTX, CTX - 1, x_d, R, st);
      TRY(dec_layers(R, row_win, row_slot, row_pos, 1, nw, win_row0, win_nrows, win_slot, d_qk, qk_map, R, false,
                     fp_anc));
      // probabilities of the text tokens, 128 logit rows at a time
      const int64_t pb = prob_off[w0];
      for (int c0 = 0; c0 < (int)sel.size(); c0 += 128) {
        const int rr = std::min<int>(128, (int)sel.size() - c0);
        HIPCHK(hipMemcpyAsync(rows_in, sel.data() + c0, rr * 4, hipMemcpyHostToDevice, st));
        TRY(vocab(rows_in, rr, d_lg));
        launch_token_probs(d_lg, V, rr, eot, d_ptok + pb + c0, d_probs + pb + c0, st);
      }
      for (int i = 0; i < nw; ++i) {
        const int w = w0 + i, N = n_tokens[w] - n_sot - 1, F = num_frames[w] / 2;
        float* mat = d_mat + mat_off[w];
        launch_align_matrix(d_qk + (int64_t)wr0[i] * 1500, (int64_t)R * 1500, n_tokens[w], 1500, F, na, n_sot, N,
                            medfilt, mat, st);
        jobs[w] = DtwJob{mat, (unsigned*)(d_tr + tr_off[w]), d_path + path_off[w], d_plen + w, N, F, 0};
      }
      size_t lds = 0;
      if (dtw_prepare(jobs.data() + w0, nw, &lds)) return fail(-15, "align: DTW shape");
      HIPCHK(hipMemcpyAsync(d_jobs + w0, jobs.data() + w0, nw * sizeof(DtwJob), hipMemcpyHostToDevice, st));
      int max_n = 0;
      for (int i = 0; i < nw; ++i) max_n = std::max(max_n, jobs[w0 + i].N);
      if (launch_dtw_jobs(d_jobs + w0, nw, max_n, jobs[w0].in_lds, lds, -1.f, st))
        return fail(-15, "align: DTW launch");
      HIPCHK(hipStreamSynchronize(st));  // host row vectors of this pass go out of scope
      w0 += nw;
    }
    HIPCHK(hipMemcpyAsync(probs, d_probs, prob_off[n_win] * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(plens, d_plen, n_win * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(paths, d_path, path_off[n_win] * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    TRY(launch_status(__func__));
    return 0;
  }

  int align(int slot, const int* tokens, int n, int n_sot, int num_frames, const int* ah, int na, int medfilt,
            float* probs, int* path, int* plen) override {
    return align_batch(1, &slot, tokens, &n, n_sot, &num_frames, ah, na, medfilt, probs, path, plen);
  }

  // timing.dtw (timing.py:82-105, 139-151) of a host cost matrix x [N][M] on the GPU
  int dtw(const float* x, int N, int M, int* path, int* plen) override {
    if (N < 1 || M < 1 || N > 1023 || (int64_t)N * M > (int64_t)1 << 26) return fail(-15, "dtw: shape out of range");
    auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
    const size_t b_x = al((size_t)N * M * 4), b_tr = al(dtw_trace_bytes(N, M)), b_path = al((size_t)2 * (N + M) * 4);
    TRY(ensure_scratch(b_x + b_tr + b_path + 256 + al(sizeof(DtwJob))));
    char* p = scratch;
    float* d_x = (float*)p; p += b_x;
    unsigned* d_tr = (unsigned*)p; p += b_tr;
    int* d_path = (int*)p; p += b_path;
    int* d_plen = (int*)p; p += 256;
    DtwJob* d_job = (DtwJob*)p;
    DtwJob job{d_x, d_tr, d_path, d_plen, N, M, 0};
    size_t lds = 0;
    if (dtw_prepare(&job, 1, &lds)) return fail(-15, "dtw: shape");
    HIPCHK(hipMemcpyAsync(d_x, x, (size_t)N * M * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_job, &job, sizeof(job), hipMemcpyHostToDevice, st));
    if (launch_dtw_jobs(d_job, 1, N, job.in_lds, lds, 1.f, st)) return fail(-15, "dtw launch");
    HIPCHK(hipMemcpyAsync(plen, d_plen, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(path, d_path, (size_t)2 * (N + M) * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    TRY(launch_status(__func__));
    return 0;
  }

  int prefill_logits(int slot, const int* tokens, int n, float* lg, const int* ah, int na, float* aqk) override {
    float* d_aqk = nullptr;
    float* out = nullptr;
    if (na > 0 && aqk) HIPCHK(hipMalloc((void**)&d_aqk, (size_t)na * n * 1500 * 4));
    HIPCHK(hipMalloc((void**)&out, (size_t)n * V * 4));
    std::vector<std::vector<int>> keep;
    int rc = first_pass(slot, tokens, n, ah, na, d_aqk, keep);
    std::vector<int> s2(n);
    for (int i = 0; i < n; ++i) s2[i] = i;
    for (int r0 = 0; r0 < n && rc == 0; r0 += 128) {
      const int rr = std::min(128, n - r0);
      if (hipMemcpyAsync(rows_in, s2.data() + r0, rr * 4, hipMemcpyHostToDevice, st) != hipSuccess) rc = -100;
      if (!rc) rc = vocab(rows_in, rr, out + (size_t)r0 * V);
      if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = -100;
    }
    if (!rc && hipMemcpyAsync(lg, out, (size_t)n * V * 4, hipMemcpyDeviceToHost, st) != hipSuccess) rc = -100;
    if (!rc && d_aqk && hipMemcpyAsync(aqk, d_aqk, (size_t)na * n * 1500 * 4, hipMemcpyDeviceToHost, st) != hipSuccess)
      rc = -100;
    if (hipStreamSynchronize(st) != hipSuccess && !rc) rc = -100;
    if (hipFree(out) != hipSuccess && !rc) rc = -100;
    if (d_aqk && hipFree(d_aqk) != hipSuccess && !rc) rc = -100;
    if (rc == -100) return fail(-100, "prefill_logits: HIP copy / sync / free failed");
    if (rc) return rc;
    TRY(launch_status(__func__));
    return 0;
  }

  int time_stage(int what, int iters, double* ms) override {
    // the stages run on the live batch's step rows: restore them first (a first pass may
    // have left its own positions in row_pos, where the projections' QKV epilogue would
    // write the decode's self-KV); stages other than whole steps leave x_d dirty
    restore_rows();
    if (what != 0 && what != 7) rows_dirty = true;
    if (what == 0) {
      if (cur_nwin < 1) return fail(-16, "no decode batch");
      if (!eager()) TRY(ensure_graph());
      HIPCHK(hipEventRecord(tm.a, st));
      for (int i = 0; i < iters; ++i) TRY(launch_step());
      HIPCHK(hipEventRecord(tm.b, st));
    } else if (what == 1) {
      HIPCHK(hipEventRecord(tm.a, st));
      for (int i = 0; i < iters; ++i) TRY(encode_chunk(0, 1, true));
      HIPCHK(hipEventRecord(tm.b, st));
    } else if (what == 2 || what == 3 || what == 5 || what == 6) {
      // per-launch time of one decoder-step kernel at the current batch, over all
      // layers (so weights / cross-KV stream from HBM as in the step, not from cache):
      // 2 = the six split-K projection GEMVs of each layer (k_gemv_x, EPI_PARTIAL),
      // 3 = the step's cross-attention (k_xattn_seg)
      // 5 / 6 = 2 / 3 on layer 0 only, repeated (operands Infinity-Cache warm)
      if (cur_nwin < 1) return fail(-16, "no decode batch");
      const bool warm = what >= 5;
      if (warm) what -= 3;
      const int nl = warm ? 1 : Ld;
      const int R = cur_nwin * cur_G, n = ns;
      int launches = 0;
      HIPCHK(hipEventRecord(tm.a, st));
      for (int i = 0; i < iters * (warm ? Ld : 1); ++i)
        for (int l = 0; l < nl; ++l) {
          auto& e = dec[l];
          if (what == 2) {
            TRY(layer_projections(l, R));
            launches += 6;
          } else {
            const T* ck = ckv + (size_t)(2 * l) * Wcap * TKP * n;
            const T* cv = ckv + (size_t)(2 * l + 1) * Wcap * TKP * n;
            XQPart xq = step_xq(cur_G);  // the step's kernel (k_xattn_seg), query from q_d
            if (p1_active(R, cur_nwin) ? xq_proj1_active(cur_G) : xq_proj_active(cur_G)) {
              // or projected in the kernel (as the step does): from xn_d, or (single window)
              // from the fp32 rows with the LayerNorm in the kernel
              xq.qw = e.wqx; xq.bias = e.bqx;
              if (xq_frag_on()) xq.qwf = e.wqx_f;
              if (p1_active(R, cur_nwin)) {
                xq.qx = x_d; xq.ln_g = e.lnx_g; xq.ln_b = e.lnx_b;
                if (xq_proj1_mode() == 2) {  // the split projection, as the step runs it
                  xq.q_part = xq1_part; xq.q_cnt = xq1_cnt; xq.qwf = nullptr;
                }
              } else {
                xq.qx = xn_d;
              }
            }
            launch_cross_attn<T>(q_d, n, ck, cv, 1500, nh, NSPLIT, cur_nwin, st_win_row0, st_win_nrows, st_win_slot,
                                 (int64_t)TKP * n, po, pm, pl, att_d, n, R, nullptr, nullptr, 0, st, xq);
            ++launches;
          }
        }
      HIPCHK(hipEventRecord(tm.b, st));
      HIPCHK(hipStreamSynchronize(st));
      float t = 0;
      HIPCHK(hipEventElapsedTime(&t, tm.a, tm.b));
      *ms = t / launches;
      return 0;
    } else if (what == 7) {
      // per-launch time of the step's k_proj projections inside eager steps: every
      // launch carries its own start/stop events (hipExtLaunchKernelGGL: timestamps of
      // the dispatch itself, no marker packets), in the step's kernel order, so each
      // one runs behind its real producer as in the graph (not back to back)
      if (cur_nwin < 1) return fail(-16, "no decode batch");
      const int per_step = 6 * Ld;
      proj_ev.resize(2 * per_step * iters);
      // timing-only events: no system-scope fence (its L2 writeback / invalidate would be
      // charged to the timed kernel; rocprofv3's kernel trace has none)
      for (auto& ev : proj_ev) HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableSystemFence));
      double tot = 0;
      int launches = 0, rc = 0;
      // steps queued back to back as in decode_steps (no host sync between them)
      proj_ev_n = 0;
      for (int i = 0; i < iters && rc == 0; ++i) rc = step_body();
      if (rc == 0 && hipStreamSynchronize(st) != hipSuccess) rc = fail(-100, "time_stage(7): sync failed");
      for (int j = 0; rc == 0 && j < proj_ev_n; ++j) {
        float t = 0;
        if (hipEventElapsedTime(&t, proj_ev[2 * j], proj_ev[2 * j + 1]) != hipSuccess)
          rc = fail(-100, "time_stage(7): hipEventElapsedTime failed");
        tot += t;
        ++launches;
      }
      for (auto& ev : proj_ev)
        if (hipEventDestroy(ev) != hipSuccess && rc == 0) rc = fail(-100, "time_stage(7): hipEventDestroy failed");
      proj_ev.clear();
      proj_ev_n = 0;
      if (rc) return rc;
      *ms = launches ? tot / launches : 0.0;
      return 0;
    } else if (what == 8 || what == 9) {
      // the step's self-attention alone (k_self_attn_qkv, every layer, the live batch at its
      // current context; it rewrites each row's K/V at its next position from the slabs as
      // they stand, which the next real step overwrites): 8 = the decode's ancestry, 9 = every
      // row reading beam slot 0's rows (all beams share one history: the bytes an L2 that
      // deduplicated shared rows perfectly would fetch).  Per-launch ms.
      if (cur_nwin < 1 || cur_G < 1) return fail(-16, "no decode batch");
      if (p1_active(cur_nwin * cur_G, cur_nwin)) return fail(-2, "time_stage(8/9): the single-window step has no k_self_attn_qkv");
      const int R = cur_nwin * cur_G, n = ns;
      const size_t ab = (size_t)Wcap * Gcap * CTX * sizeof(int);
      int* saved = nullptr;
      if (what == 9) {
        HIPCHK(hipMalloc((void**)&saved, ab));
        HIPCHK(hipMemcpyAsync(saved, S.anc, ab, hipMemcpyDeviceToDevice, st));
        HIPCHK(hipMemsetAsync(S.anc, 0, ab, st));
      }
      int rc = 0;
      if (hipEventRecord(tm.a, st) != hipSuccess) rc = fail(-100, "time_stage(8/9): hipEventRecord failed");
      for (int i = 0; rc == 0 && i < iters; ++i)
        for (int l = 0; rc == 0 && l < Ld; ++l)
          if (launch_self_attn_qkv<T>(part, sa_probe_ks, (int64_t)R * 3 * n, dec[l].bqkv, n, kc[l], vc[l], st_row_win,
                                      st_row_slot, row_pos, S.anc, cur_G, Gcap, nh, CTX, att_d, n, R, st, sa_probe_half))
            rc = fail(-20, "time_stage(8/9): self-attention launch refused");
      if (rc == 0 && hipEventRecord(tm.b, st) != hipSuccess) rc = fail(-100, "time_stage(8/9): hipEventRecord failed");
      if (saved) {
        if (hipMemcpyAsync(S.anc, saved, ab, hipMemcpyDeviceToDevice, st) != hipSuccess && rc == 0)
          rc = fail(-100, "time_stage(9): ancestry restore failed");
        if (hipStreamSynchronize(st) != hipSuccess && rc == 0) rc = fail(-100, "time_stage(9): sync failed");
        if (hipFree(saved) != hipSuccess && rc == 0) rc = fail(-100, "time_stage(9): hipFree failed");
      }
      if (rc) return rc;
      HIPCHK(hipStreamSynchronize(st));
      float t = 0;
      HIPCHK(hipEventElapsedTime(&t, tm.a, tm.b));
      *ms = t / (iters * Ld);
      return 0;
    } else if (what == 4) {
      // the token-selection kernel alone on the current logits (state unchanged)
      if (cur_nwin < 1) return fail(-16, "no decode batch");
      HIPCHK(hipEventRecord(tm.a, st));
      for (int i = 0; i < iters; ++i) launch_logit_rows(logits, V, S, O, cur_nwin, st);
      HIPCHK(hipEventRecord(tm.b, st));
    } else {
      return fail(-2, "time_stage: unknown stage");
    }
    HIPCHK(hipStreamSynchronize(st));
    float t = 0;
    HIPCHK(hipEventElapsedTime(&t, tm.a, tm.b));
    *ms = t / iters;
    return 0;
  }
};

}  // namespace

// ============================================================ C ABI
extern "C" {

const char* wh_last_error(void) { return g_err.c_str(); }
int wh_version(void) { return 1; }

int wh_create(int device, const wh_dims* dims, int compute_dtype, int max_windows, int max_group, wh_ctx** out) {
  if (!dims || !out) return fail(-1, "null argument");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(-1, "no HIP device");
  if (device < 0 || device >= ndev) return fail(-1, "device out of range");
  int rc;
  if (compute_dtype == WH_F16) {
    auto c = new Ctx<half_t>();
    rc = c->init(device, *dims, max_windows, max_group);
    if (rc) { delete c; return rc; }
    *out = c;
  } else if (compute_dtype == WH_F32) {
    auto c = new Ctx<float>();
    rc = c->init(device, *dims, max_windows, max_group);
    if (rc) { delete c; return rc; }
    *out = c;
  } else {
    return fail(-1, "compute_dtype must be WH_F32 or WH_F16");
  }
  return 0;
}

int wh_destroy(wh_ctx* ctx) {
  if (!ctx) return 0;
  if (ctx->sharers > 0)
    return fail(-1, "wh_destroy: " + std::to_string(ctx->sharers) +
                        " context(s) still read this context's weights (wh_tune_share_weights): destroy them first");
  if (ctx->shares_from) --ctx->shares_from->sharers;
  hipSetDevice(ctx->device);
  g_release_error.clear();
  delete ctx;
  if (!g_release_error.empty()) return fail(-100, "wh_destroy: " + g_release_error);
  return 0;
}

int wh_set_mel_filters(wh_ctx* ctx, int n_mels, const float* filters) {
  if (!ctx || !filters) return fail(-1, "null argument");
  if (const int rc = enter(ctx, __func__)) return rc;
  std::vector<float> f(filters, filters + (size_t)n_mels * 201);
  // both element-type contexts share the filter map through the base pointer cast
  auto* c16 = dynamic_cast<Ctx<half_t>*>(ctx);
  auto* c32 = dynamic_cast<Ctx<float>*>(ctx);
  std::map<int, float*>& dm = c16 ? c16->d_filters : c32->d_filters;
  std::map<int, std::vector<float>>& hm = c16 ? c16->h_filters : c32->h_filters;
  float* d = nullptr;
  if (dm.count(n_mels)) d = dm[n_mels];
  else {
    HIPCHK(hipMalloc(&d, f.size() * 4));
    dm[n_mels] = d;
  }
  HIPCHK(hipMemcpy(d, f.data(), f.size() * 4, hipMemcpyHostToDevice));
  hm[n_mels] = f;
  return 0;
}

// every context call: on the context's device, and no HIP error pending from before it
// (a pending one belongs to an earlier call: reported as such, not as this call's failure)
static int enter(wh_ctx* ctx, const char* entry) {
  if (!ctx) return fail(-1, "null context");
  const hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return fail(-100, std::string(entry) + ": hipSetDevice: " + hipGetErrorString(e));
  const int rc = launch_status("HIP error pending before this call");
  if (rc) g_err = std::string(entry) + ": " + g_err;
  return rc;
}
#define CTXCALL(expr)                            \
  do {                                           \
    const int rc_e = enter(ctx, __func__);       \
    if (rc_e) return rc_e;                       \
    return (expr);                               \
  } while (0)

int wh_load_tensor(wh_ctx* ctx, const char* name, const float* data, const int64_t* shape, int ndim) {
  if (!name || !data || !shape) return fail(-1, "null argument");
  CTXCALL(ctx->load(name, data, shape, ndim));
}
int wh_finalize(wh_ctx* ctx) { CTXCALL(ctx->finalize()); }
int wh_token_ms(wh_ctx* ctx, float* out, int cap, int* n, int reset) {
  if (!ctx) return -1;
  const int cnt = (int)ctx->token_ms.size();
  if (n) *n = cnt;
  if (out)
    for (int i = 0; i < cnt && i < cap; ++i) out[i] = ctx->token_ms[i];
  if (reset) ctx->token_ms.clear();
  return 0;
}
int wh_log_mel(wh_ctx* ctx, const float* audio, int64_t n, int64_t pad, int n_mels, int normalize, int64_t* nf) {
  CTXCALL(ctx->log_mel(audio, n, pad, n_mels, normalize, nf));
}
int wh_log_mel_frames(wh_ctx* ctx, const float* audio, int64_t n, int64_t pad, int n_mels, int64_t frame0,
                      int64_t count, int normalize, int64_t* total_frames) {
  CTXCALL(ctx->log_mel_frames(audio, n, pad, n_mels, frame0, count, normalize, total_frames));
}
int wh_audio_upload(wh_ctx* ctx, const float* audio, int64_t n) {
  if (!audio || n <= 0) return fail(-1, "bad audio");
  CTXCALL(ctx->audio_upload(audio, n));
}
int wh_mel_max(wh_ctx* ctx, float* g) { CTXCALL(ctx->mel_max(g)); }
int wh_mel_normalize(wh_ctx* ctx, float g) { CTXCALL(ctx->mel_normalize(g)); }
int wh_mel_read(wh_ctx* ctx, float* out, int64_t f0, int64_t nf) { CTXCALL(ctx->mel_read(out, f0, nf)); }
int wh_mel_write(wh_ctx* ctx, const float* mel, int64_t nf) { CTXCALL(ctx->mel_write(mel, nf)); }
int wh_encode(wh_ctx* ctx, int n_win, const int64_t* seeks, const int* segs) { CTXCALL(ctx->encode(n_win, seeks, segs)); }
int wh_read_audio_features(wh_ctx* ctx, int slot, float* out) { CTXCALL(ctx->read_xa(slot, out)); }
int wh_read_cross_kv(wh_ctx* ctx, int slot, int layer, float* k, float* v) { CTXCALL(ctx->read_ckv(slot, layer, k, v)); }
int wh_decode_begin(wh_ctx* ctx, int n_win, const wh_decode_opts* o, const int* init, const int* n_init, int max_init,
                    const int* sot_index) {
  if (!o || !init || !n_init || !sot_index) return fail(-1, "null argument");
  CTXCALL(ctx->decode_begin(n_win, o, init, n_init, max_init, sot_index, nullptr));
}
int wh_decode_begin_slots(wh_ctx* ctx, int n_win, const int* slots, const wh_decode_opts* o, const int* init,
                          const int* n_init, int max_init, const int* sot_index) {
  if (!slots || !o || !init || !n_init || !sot_index) return fail(-1, "null argument");
  CTXCALL(ctx->decode_begin(n_win, o, init, n_init, max_init, sot_index, slots));
}
int wh_decode_steps(wh_ctx* ctx, int max_steps, int* n_done) { CTXCALL(ctx->decode_steps(max_steps, n_done)); }
int wh_decode_read(wh_ctx* ctx, int slot, int* tokens, float* slp, int* len, int* fin_n, int* fin_tok, int* fin_len,
                   float* fin_score, float* nsp) {
  CTXCALL(ctx->decode_read(slot, tokens, slp, len, fin_n, fin_tok, fin_len, fin_score, nsp));
}
int wh_decode_maxc(wh_ctx* ctx) { return ctx ? ctx->maxc_stride : -1; }
int wh_prefill(wh_ctx* ctx, int n_win, int group, const int* tokens, const int* n_tokens, int max_tokens,
               const int* sot_index, float* logits) {
  if (!tokens || !n_tokens || !sot_index) return fail(-1, "null argument");
  CTXCALL(ctx->step_prefill(n_win, group, tokens, n_tokens, max_tokens, sot_index, logits));
}
int wh_step(wh_ctx* ctx, const int* tokens, const int* text_offsets, float* logits) {
  if (!tokens) return fail(-1, "null argument");
  CTXCALL(ctx->step_tokens(tokens, text_offsets, logits));
}
int wh_reorder_kv(wh_ctx* ctx, const int* source_rows) {
  if (!source_rows) return fail(-1, "null argument");
  CTXCALL(ctx->reorder_kv(source_rows));
}
int wh_prefill_logits(wh_ctx* ctx, int slot, const int* tokens, int n, float* logits, const int* ah, int na, float* aqk) {
  CTXCALL(ctx->prefill_logits(slot, tokens, n, logits, ah, na, aqk));
}
int wh_align(wh_ctx* ctx, int slot, const int* tokens, int n_tokens, int n_sot, int num_frames, const int* align_heads,
             int n_align, int medfilt_width, float* token_probs, int* path, int* path_len) {
  CTXCALL(ctx->align(slot, tokens, n_tokens, n_sot, num_frames, align_heads, n_align, medfilt_width, token_probs, path,
                     path_len));
}
int wh_align_batch(wh_ctx* ctx, int n_win, const int* slots, const int* tokens, const int* n_tokens, int n_sot,
                   const int* num_frames, const int* align_heads, int n_align, int medfilt_width, float* token_probs,
                   int* paths, int* path_lens) {
  CTXCALL(ctx->align_batch(n_win, slots, tokens, n_tokens, n_sot, num_frames, align_heads, n_align, medfilt_width,
                           token_probs, paths, path_lens));
}
int wh_dtw(wh_ctx* ctx, const float* x, int n_rows, int n_cols, int* path, int* path_len) {
  CTXCALL(ctx->dtw(x, n_rows, n_cols, path, path_len));
}
int wh_stats(wh_ctx* ctx, double* out, int n) {
  if (!ctx || !out) return fail(-1, "null argument");
  for (int i = 0; i < n && i < 8; ++i) out[i] = ctx->stats[i];
  return 0;
}
int wh_step_kernels(wh_ctx* ctx, int n_win, int group, char* buf, int cap) {
  if (!ctx || !buf || cap < 1) return fail(-1, "bad arguments");
  const std::string d = ctx->step_kernels(n_win, group);
  const int n = std::min<int>((int)d.size(), cap - 1);
  memcpy(buf, d.data(), n);
  buf[n] = 0;
  return n;
}
int wh_sync(wh_ctx* ctx) {
  const int rc = enter(ctx, __func__);
  if (rc) return rc;
  HIPCHK(hipDeviceSynchronize());
  return launch_status(__func__);
}
int wh_time_stage(wh_ctx* ctx, int what, int iters, double* ms) { CTXCALL(ctx->time_stage(what, iters, ms)); }
#if WH_TUNING
int wh_tune_share_weights(wh_ctx* ctx, wh_ctx* src) {
  if (!src) return fail(-1, "null source context");
  CTXCALL(ctx->share_weights_from(src));
}
#endif

}  // extern "C"
