/*
 * libwhisper_hip — C ABI of the MI355X (gfx950) Whisper backend.
 *
 * This is the drop-in replacement for the reference's native backend boundary,
 * coreml/coreml.h:5-31 of wangchou/whisper.coreml, which Python binds through
 * ctypes in whisper/coreml.py:19-244.  The roles map one to one (citations are
 * /root/reference paths):
 *
 *   loadEncoder/loadCrossKV/loadDecoder256/loadDecoder1 (coreml.h:5,9,13,23)
 *        -> wh_create + wh_load_tensor + wh_finalize (weights come from the
 *           reference's own state_dict names, whisper/__init__.py:152-160)
 *   encoderPredict (coreml.h:7) + crossKVPredict (coreml.h:11)
 *        -> wh_encode  (AudioEncoder.forward encoder.py:103-136 and
 *           TextDecoder.crossKVCaches decoder.py:172-187, all windows batched)
 *   decoder256Predict (coreml.h:15-21) -> wh_decode_begin (first pass) /
 *           wh_prefill_logits (full-row logits + alignment cross-QK)
 *   decoder1Predict (coreml.h:26-31) + rearrange_mkv (coreml.h:25) + the host
 *           beam/filter loop (whisper/decoding.py:707-737)
 *        -> wh_decode_steps (one hipGraph per token: decoder step, logit filters,
 *           greedy/beam update, KV reorder by index indirection)
 *   the same roles one call per token, for a caller that keeps the reference's
 *   host loop (PyTorchInference.logits / rearrange_kv_cache, decoding.py:151-204):
 *        decoder256Predict (coreml.h:15-21) -> wh_prefill
 *        decoder1Predict   (coreml.h:26-31) -> wh_step
 *        rearrange_mkv     (coreml.h:25)    -> wh_reorder_kv
 *   log_mel_spectrogram (whisper/audio.py:110-157) -> wh_log_mel
 *   showCoremlPredictTime (whisper/coreml.py:247-263) -> wh_stats
 *
 * Conventions: every call returns 0 on success, a negative code on failure
 * (message via wh_last_error, thread-local).  All pointers are host pointers
 * (plain C arrays, row-major); device memory is owned by the context.  A
 * context is bound to one HIP device; use one context per GPU process.
 */
#ifndef WHISPER_HIP_H
#define WHISPER_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct wh_ctx wh_ctx;

/* ModelDimensions (whisper/model.py:18-29) */
typedef struct wh_dims {
  int n_mels, n_audio_ctx, n_audio_state, n_audio_head, n_audio_layer;
  int n_vocab, n_text_ctx, n_text_state, n_text_head, n_text_layer;
} wh_dims;

enum { WH_F32 = 0, WH_F16 = 1 };

/* DecodingOptions (whisper/decoding.py:81-115) resolved against the tokenizer */
typedef struct wh_decode_opts {
  int group;             /* rows per window: beam_size, best_of or 1 (<= 8) */
  int beam;              /* 1 = BeamSearchDecoder, 0 = GreedyDecoder */
  float patience;        /* beam: max_candidates = round(group * patience) */
  float temperature;     /* greedy: 0 = argmax, > 0 = sampling */
  int sample_len;        /* max updates (n_text_ctx / 2 by default) */
  int suppress_blank;    /* SuppressBlank */
  int timestamps;        /* ApplyTimestampRules (0 = without_timestamps) */
  int max_initial;       /* max_initial_timestamp index, -1 = none */
  int eot, no_speech, no_timestamps, timestamp_begin; /* no_speech < 0: none */
  int blank[4];          /* tokenizer.encode(" ") ids suppressed with eot at the first step */
  int n_blank;
  const int* suppress;   /* SuppressTokens ids (already resolved, -1 expanded) */
  int n_suppress;
  unsigned long long seed; /* sampling RNG seed */
  int max_candidates;    /* beam: round(beam_size * patience) as the host computes it
                            (Python round, decoding.py:339); <= 0: derived from patience */
} wh_decode_opts;

const char* wh_last_error(void);
int wh_version(void);

int wh_create(int device, const wh_dims* dims, int compute_dtype, int max_windows, int max_group, wh_ctx** out);
int wh_destroy(wh_ctx* ctx);

/* checkpoint-format float32 tensor by reference state_dict name; the decoder query
   pre-scale (decoder.py:16-20) and the encoder key scale (encoder.py:38) are
   folded here. */
int wh_load_tensor(wh_ctx* ctx, const char* name, const float* data, const int64_t* shape, int ndim);
int wh_finalize(wh_ctx* ctx);

/* mel filterbank [n_mels][201] (whisper/audio.py:91-107; the host derives it with the
   Slaney formula librosa uses and checks it against the reference asset in tests) */
int wh_set_mel_filters(wh_ctx* ctx, int n_mels, const float* filters);

/* log-mel of a whole file into the context's mel buffer: n_frames = (n + padding) / 160.
   normalize = 1 applies the global-max floor and scaling immediately. */
int wh_log_mel(wh_ctx* ctx, const float* audio, int64_t n_samples, int64_t padding, int n_mels, int normalize,
               int64_t* n_frames);
/* frames [frame0, frame0 + count) of the same log-mel (count < 0: to the end); the
   context stores them with their absolute offset, so wh_encode seeks and wh_mel_read
   frames stay absolute.  One rank of a file sharded over GPUs computes only the frames
   of its clips; the global max (wh_mel_max) is then all-reduced and applied with
   wh_mel_normalize.  *total_frames = (n + padding) / 160. */
int wh_log_mel_frames(wh_ctx* ctx, const float* audio, int64_t n_samples, int64_t padding, int n_mels,
                      int64_t frame0, int64_t count, int normalize, int64_t* total_frames);
/* keep audio resident in HBM; wh_log_mel(ctx, NULL, n, ...) then computes from it */
int wh_audio_upload(wh_ctx* ctx, const float* audio, int64_t n_samples);
int wh_mel_max(wh_ctx* ctx, float* gmax);              /* raw log10 max of the last wh_log_mel */
int wh_mel_normalize(wh_ctx* ctx, float gmax);         /* floor at gmax-8, (x+4)/4 */
int wh_mel_read(wh_ctx* ctx, float* out, int64_t frame0, int64_t n_frames); /* [n_mels][n_frames], absolute frames */
int wh_mel_write(wh_ctx* ctx, const float* mel, int64_t n_frames);          /* host mel -> context */

/* encoder + cross-KV for n_win windows of the context mel: window i = frames
   [seek[i], seek[i] + seg[i]) zero-padded to 3000 (audio.py:65-88), into slot i */
int wh_encode(wh_ctx* ctx, int n_win, const int64_t* seek_frames, const int* seg_frames);
int wh_read_audio_features(wh_ctx* ctx, int slot, float* out);                   /* [n_audio_ctx][n_state] */
int wh_read_cross_kv(wh_ctx* ctx, int slot, int layer, float* k_out, float* v_out); /* [H][n_audio_ctx][64] */

/* decode n_win windows (slots 0..n_win-1): prefill of the initial tokens
   (init_tokens[w*max_init + i], i < n_init[w]) and the first token update */
int wh_decode_begin(wh_ctx* ctx, int n_win, const wh_decode_opts* opts, const int* init_tokens, const int* n_init,
                    int max_init, const int* sot_index);
/* wh_decode_begin where decode window w attends to the audio features of encoder slot
   slots[w] (the temperature fallback, transcribe.py:188-228, re-decodes only the
   windows that failed, from the slots that already hold them).  wh_decode_read's
   `slot` is the decode window index w. */
int wh_decode_begin_slots(wh_ctx* ctx, int n_win, const int* slots, const wh_decode_opts* opts,
                          const int* init_tokens, const int* n_init, int max_init, const int* sot_index);
/* run up to max_steps token updates (hipGraph); *n_done = windows finished */
int wh_decode_steps(wh_ctx* ctx, int max_steps, int* n_done);
/* read back a window: tokens [group][n_text_ctx+1], sum_logprobs [group], len,
   finished (beam) fin_tokens [maxc][n_text_ctx+1], fin_len/fin_score [maxc] */
int wh_decode_read(wh_ctx* ctx, int slot, int* tokens, float* sum_logprobs, int* len, int* fin_n, int* fin_tokens,
                   int* fin_len, float* fin_score, float* no_speech_prob);
int wh_decode_maxc(wh_ctx* ctx);

/* ---- per-step boundary (the reference's decoder256Predict / decoder1Predict /
   rearrange_mkv, coreml.h:15-31, driven by its host DecodingTask loop,
   decoding.py:707-737).  Rows are r = w * group + b for windows w < n_win (slots
   0..n_win-1, encoded by wh_encode) and beams b < group.

   wh_prefill: first pass of each window's initial tokens (tokens[w * max_tokens + i],
   i < n_tokens[w]; all rows of a window share them, coreml.mm:279-327 runs the same
   pass once per beam).  logits (nullable) [n_win][2][n_vocab]: the rows at position
   sot_index[w] (no-speech probability, decoding.py:716-720) and n_tokens[w] - 1. */
int wh_prefill(wh_ctx* ctx, int n_win, int group, const int* tokens, const int* n_tokens, int max_tokens,
               const int* sot_index, float* logits);
/* wh_step: one decoder step.  Row r appends tokens[r] (the token the host chose for it)
   at position text_offsets[w] (nullable; when given it must equal the window's cached
   length, the text_offset of decoder1Predict) and returns logits [n_win*group][n_vocab]
   (nullable: kept on the device only). */
int wh_step(wh_ctx* ctx, const int* tokens, const int* text_offsets, float* logits);
/* wh_reorder_kv: after a beam update, row r continues the sequence of row
   source_rows[r] (a row of the same window; PyTorchInference.rearrange_kv_cache).
   No cache bytes move: the rows' ancestry tables are permuted.  Once per step. */
int wh_reorder_kv(wh_ctx* ctx, const int* source_rows);

/* decoder forward over tokens at offset 0 for one window slot (Whisper.forward,
   model.py:110-119 / the decoder256 first pass); logits [n_tokens][n_vocab];
   align_qk (nullable) [n_align][n_tokens][n_audio_ctx] raw cross q.k of the heads
   in align_heads (layer*n_head + head).  Like the reference's first pass, it writes the
   slot's self-KV rows: call it (and wh_align / wh_align_batch) on a slot whose decode has
   finished or that is not in the current batch; a device-loop decode of OTHER slots may
   continue with wh_decode_steps afterwards (its step rows are re-embedded first). */
int wh_prefill_logits(wh_ctx* ctx, int slot, const int* tokens, int n_tokens, float* logits, const int* align_heads,
                      int n_align, float* align_qk);

/* find_alignment's numeric half (reference whisper/timing.py:163-231), replacing the
   model(tokens) first pass with cross-QK capture (model.py:110-119, decoder.py:306-313,
   the decoder256 CoreML call of coreml.h:17-18 with out_cross_head_weights), the
   softmax / z-norm / median filter / head mean (timing.py:197-205) and dtw
   (timing.py:139-151, dtw_cpu :82-105 + backtrace :57-79) — all on the GPU.
   tokens = sot_sequence (n_sot ids) + [no_timestamps] + text (T ids) + [eot]
   (timing.py:175-182); the window's audio features must be in `slot`.
   token_probs [T] = softmax(logits[n_sot + k][:eot])[text[k]] (timing.py:187-191);
   path [2][T + 1 + num_frames/2]: text indices then time indices, *path_len valid
   entries of each (the rows of dtw(-matrix), timing.py:206). */
int wh_align(wh_ctx* ctx, int slot, const int* tokens, int n_tokens, int n_sot, int num_frames, const int* align_heads,
             int n_align, int medfilt_width, float* token_probs, int* path, int* path_len);
/* wh_align for n_win windows at once (slots[w], n_tokens[w] ids each, concatenated in
   tokens; num_frames[w]): their first passes run batched (up to 1024 rows per pass) and
   their DTWs run one workgroup per window in one launch.  Outputs concatenated in window
   order: token_probs [T_w], paths [2][T_w + 1 + num_frames[w]/2], path_lens [n_win]. */
int wh_align_batch(wh_ctx* ctx, int n_win, const int* slots, const int* tokens, const int* n_tokens, int n_sot,
                   const int* num_frames, const int* align_heads, int n_align, int medfilt_width, float* token_probs,
                   int* paths, int* path_lens);
/* timing.dtw(x) of a host matrix x [n_rows][n_cols] (n_rows <= 1023) on the GPU:
   path [2][n_rows + n_cols], *path_len valid entries of each */
int wh_dtw(wh_ctx* ctx, const float* x, int n_rows, int n_cols, int* path, int* path_len);

/* the kernels the decoder step runs for a batch of n_win windows x group rows, as
   "proj=<name>,xattn=<name>" (the dominant projection family and the cross-attention;
   what bench.py labels its roofline lines with).  Returns the length written. */
int wh_step_kernels(wh_ctx* ctx, int n_win, int group, char* buf, int cap);

/* cumulative stage wall times in ms: [0] mel [1] encode [2] prefill [3] steps
   [4] step count [5] encode windows */
int wh_stats(wh_ctx* ctx, double* out, int n);
int wh_sync(wh_ctx* ctx);

/* per-token wall milliseconds of every decode_steps chunk since the last reset
   (chunk wall time / steps in the chunk, host poll included): *n = count, up to
   cap values copied to out (nullable); reset != 0 clears the record.  Feeds the
   p50 per-token decode ms of BASELINE.json's metric. */
int wh_token_ms(wh_ctx* ctx, float* out, int cap, int* n, int reset);

/* timing of the dominant kernels for roofline reporting: runs `iters` launches of
   the given stage on the context's own stream between HIP events.
   what: 0 = one decoder step graph (current batch), 1 = encoder of 1 window,
         2 = one split-K projection launch (k_proj; the six per layer, all layers, back to back),
         3 = one cross-attention launch (the step kernel k_cross_attn1, all layers).
         4 = the token-selection kernel (k_logit_rows) on the current logits,
         5 / 6 = 2 / 3 on layer 0 only, repeated (operands Infinity-Cache warm),
         7 = the step's k_proj launches inside `iters` eager decoder steps, each timed by
             its own dispatch events (advances the decode state like a step),
         8 / 9 = the batched step's self-attention (k_self_attn_qkv) of every layer at the
             current context, with the decode's ancestry (8) or every row reading beam slot
             0's history (9: all beams share one history); the ancestry is restored.
   For 2, 3, 5, 6, 7, 8 and 9 *ms_per_iter is the average duration of a single kernel launch. */
int wh_time_stage(wh_ctx* ctx, int what, int iters, double* ms_per_iter);

/* ---- audio file decoding (host only, no context / GPU needed) ----
   Replaces the reference's `ffmpeg` subprocess in load_audio (whisper/audio.py:42-62)
   for FLAC input (tests/jfk.flac is 44.1 kHz stereo 24-bit).  Samples are decoded
   bit-exactly (STREAMINFO MD5); down-mixing and resampling are done by the caller.
   wh_flac_info: stream parameters from STREAMINFO.
   wh_flac_decode: interleaved int32 samples [frames][channels] into out (capacity
   cap_frames frames); *n_frames = frames decoded.  Errors: < 0, wh_flac_last_error(). */
int wh_flac_info(const uint8_t* data, int64_t n, int* sample_rate, int* channels, int* bits_per_sample,
                 int64_t* total_samples);
int wh_flac_decode(const uint8_t* data, int64_t n, int32_t* out, int64_t cap_frames, int64_t* n_frames);
const char* wh_flac_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
