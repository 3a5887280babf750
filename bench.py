#!/usr/bin/env python
"""xRT benchmark: large-v3, beam 5, fp16, synthetic audio, 1..8 MI355X (one process per GPU).

A "step" is one ``transcribe()`` of the rank's audio shard (config 3 of
BASELINE.json: 10 minutes of 16 kHz audio per GPU, weak scaling), in the
sharded schedule of SURVEY.md §8(e): 30 s clip grid, condition_on_previous_text
= False, temperature 0 — every clip's windows are batched through the encoder
and the hipGraph decoder together.  The audio is resident in HBM before the
timed region (``HipContext.audio_upload``); the only cross-rank exchanges are
an all-reduce MAX of the log-mel global maximum (audio.py:155 is a whole-file
max) and the final gather of the segment records, both over RCCL.

value = (audio seconds of all ranks x steps) / (max over ranks of the timed wall
time) = whole-job xRT.  rank 0 prints one JSON line.
"""

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "whisper.coreml_amd"))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
MFMA_F16_PEAK_TFS = 2500.0  # dense fp16/bf16 MFMA, spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--model", default="large-v3")
    p.add_argument("--seconds", type=float, default=600.0, help="audio seconds per GPU")
    p.add_argument("--beam", type=int, default=5)
    p.add_argument("--dtype", default="fp16")
    p.add_argument("--max-windows", type=int, default=20)
    p.add_argument("--cpu-baseline", type=int, default=1)
    p.add_argument("--cpu-steps", type=int, default=6, help="decoder steps in the CPU baseline sample")
    p.add_argument("--dump", default="", help="write the last step's segments (tokens, avg_logprob) as JSON")
    p.add_argument("--word-timestamps", type=int, default=0,
                   help="config 5: transcribe(word_timestamps=True) (alignment + DTW on the GPU per window)")
    return p.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pg = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
        pg = dist
    return world, rank, local, pg


def allreduce_max(pg, x: float) -> float:
    if pg is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float32, device="cuda")
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def barrier(pg):
    if pg is not None:
        pg.barrier()


def decoder_step_bytes(dims, n_windows, beams, mean_ctx, elem=2):
    """Algorithmic HBM bytes of one decoder step: decoder weights
    (L*14 n^2 + V n params, read once per step for the whole batch), the cross-KV of
    every window (2 * 1500 * n * L), the self-KV of every beam row (2 * t * n * L)."""
    n, L, V = dims["n_text_state"], dims["n_text_layer"], dims["n_vocab"]
    weights = (L * 14 * n * n + V * n) * elem
    cross = n_windows * 2 * 1500 * n * L * elem
    selfkv = n_windows * beams * 2 * mean_ctx * n * L * elem
    return weights + cross + selfkv


def projection_bytes_per_launch(dims, rows, elem=2):
    """Algorithmic bytes of one split-K projection GEMV, averaged over the six per
    decoder layer (qkv n->3n, out n->n, cross-q n->n, cross-out n->n, fc1 n->4n,
    fc2 4n->n): weights N*K + activations rows*K (fp16) + fp32 result rows*N."""
    n = dims["n_text_state"]
    shapes = [(3 * n, n), (n, n), (n, n), (n, n), (4 * n, n), (n, 4 * n)]
    tot = sum(N * K * elem + rows * K * elem + rows * N * 4 for N, K in shapes)
    return tot // len(shapes)


def cross_attn_bytes_per_launch(dims, n_windows, rows, elem=2):
    """One layer's cross-attention: K and V of every window (2*1500*n) + q in / out."""
    n = dims["n_text_state"]
    return n_windows * 2 * 1500 * n * elem + 2 * rows * n * elem


def load_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed PMC pass
    (profiles/<round>/traffic.json, written by profiles/pmc_traffic.py: FETCH_SIZE x2
    + WRITE_SIZE per the gfx950 correction of MI355X_MICROARCH.md), or None."""
    path = os.path.join(REPO, "profiles", "r01", "traffic.json")
    try:
        with open(path) as f:
            return json.load(f)[kernel]["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def encoder_flops(dims):
    n, L, T = dims["n_audio_state"], dims["n_audio_layer"], 1500
    conv = 2 * 3000 * dims["n_mels"] * 3 * n + 2 * 1500 * n * 3 * n
    block = 2 * T * n * (3 * n) + 2 * 2 * T * T * n + 2 * T * n * n + 2 * 2 * T * n * 4 * n
    return conv + L * block


def cpu_baseline(model_name, sd, audio, beams, n_steps):
    """The oracle (CPU fp32 restatement, oracle/ref_whisper.py) on a bounded sample of
    one 30 s window: encoder + first pass + n_steps beam decoder steps, extrapolated
    to the 224-step fixed work of a window."""
    import torch
    from oracle import ref_whisper as R
    from whisper import synthetic as S
    threads = torch.get_num_threads()
    dims = S.MODEL_DIMS[model_name]
    m = R.OracleWhisper(dims, sd)
    st = R.SpecialTokens.for_model(dims)
    mel = R.pad_or_trim(R.log_mel_spectrogram(audio[:480000], dims["n_mels"], padding=R.N_SAMPLES)[:, :3000])
    t0 = time.time()
    xa = m.encode(mel)
    t_enc = time.time() - t0
    m.set_audio(xa)
    toks = torch.tensor([list(st.sot_sequence)] * beams)
    t0 = time.time()
    logits, cache, _ = m.decoder_forward(toks, 0, None)
    t_pre = time.time() - t0
    offset = toks.shape[1]
    nxt = logits[:, -1].argmax(-1, keepdim=True)
    t0 = time.time()
    for _ in range(n_steps):
        logits, cache, _ = m.decoder_forward(nxt, offset, cache)
        offset += 1
        nxt = logits[:, -1].argmax(-1, keepdim=True)
    t_step = (time.time() - t0) / n_steps
    per_window = t_enc + t_pre + 224 * t_step
    return dict(value=round(30.0 / per_window, 4), unit="xRT (audio-s/s)", cores=threads, kind="port",
                sample=f"1 window of {model_name}: encoder {t_enc:.2f}s + first pass {t_pre:.2f}s + "
                       f"{n_steps} beam-{beams} steps at {t_step*1e3:.0f} ms/step, extrapolated to 224 steps "
                       f"(oracle/ref_whisper.py, torch CPU fp32, {threads} threads)")


def main():
    args = parse()
    world, rank, local, pg = dist_setup(args)
    import whisper
    from whisper import synthetic as S

    dims = S.MODEL_DIMS[args.model]
    sd = S.synthetic_state_dict(dims, 0)
    model = whisper.Whisper(whisper.ModelDimensions(**dims), args.model, device=local, dtype=args.dtype,
                            max_windows=args.max_windows, max_group=args.beam)
    model.load_state_dict(sd)
    if args.model in whisper._ALIGNMENT_HEADS:  # as load_model does (reference __init__.py:176-177)
        model.set_alignment_heads(whisper._ALIGNMENT_HEADS[args.model])
    if not (rank == 0 and world == 1 and args.cpu_baseline):
        del sd
        sd = None
    n_clips = int(round(args.seconds / 30.0))
    # start,end pairs of a 30 s grid covering the whole shard (transcribe.py:172-181)
    clip_ts = ",".join(f"{30 * i},{30 * (i + 1)}" for i in range(n_clips))
    # the rank's shard of one long synthetic file (seeded per rank)
    audio = S.synthetic_audio(args.seconds, seed=1000 + rank)
    dev_audio = model.ctx.audio_upload(audio)

    def reduce_max(x):
        return allreduce_max(pg, x)

    if args.word_timestamps:
        # word splitting needs token bytes; the box has no BPE rank file, so every text
        # id decodes to its own word " w<id>" (host-side grouping only: the GPU work,
        # first pass + alignment + DTW per window, is the same for any byte table)
        from whisper import tokenizer as T
        T.set_token_bytes("multilingual" if model.is_multilingual else "gpt2",
                          {i: b" w%d" % i for i in range(dims["n_vocab"])})

    def one_step():
        # per-rank log-mel, global max over ranks (all-reduce MAX), normalize, transcribe
        return whisper.transcribe(model, dev_audio, temperature=0.0, beam_size=args.beam, language="en",
                                  condition_on_previous_text=False, clip_timestamps=clip_ts,
                                  mel_max_reduce=reduce_max if pg is not None else None, schedule="batched",
                                  word_timestamps=bool(args.word_timestamps))

    for _ in range(args.warmup):
        one_step()
    barrier(pg)
    model.ctx.sync()
    st0 = model.ctx.stats()
    model.ctx.token_ms(reset=True)
    t0 = time.perf_counter()
    results = []
    for _ in range(args.steps):
        results.append(one_step())
    model.ctx.sync()
    barrier(pg)
    elapsed = time.perf_counter() - t0
    st1 = model.ctx.stats()
    elapsed_max = allreduce_max(pg, elapsed)

    if args.dump and rank == 0:
        with open(args.dump, "w") as f:
            json.dump([{k: s[k] for k in ("seek", "tokens", "avg_logprob", "no_speech_prob")}
                       for s in results[-1]["segments"]], f)

    # segment gather to rank 0 (the only data-path exchange besides the mel max)
    seg_tokens = sum(len(s["tokens"]) for s in results[-1]["segments"])
    n_segments = len(results[-1]["segments"])
    if pg is not None:
        gathered = [None] * world
        pg.all_gather_object(gathered, (n_segments, seg_tokens))
    else:
        gathered = [(n_segments, seg_tokens)]

    steps_done = st1["steps"] - st0["steps"]
    steps_ms = st1["steps_ms"] - st0["steps_ms"]
    enc_ms = st1["encode_ms"] - st0["encode_ms"]
    enc_windows = st1["encode_windows"] - st0["encode_windows"]
    ms_per_token = steps_ms / max(steps_done, 1)

    # p50 per-token decode ms: median over the timed region's decode_steps chunks
    tok = model.ctx.token_ms()
    p50_token_ms = float(np.median(tok)) if len(tok) else ms_per_token

    # roofline of the dominant kernel (k_proj: the split-K projections of the decoder
    # step, ~31% of step time over its three tile variants), timed live with HIP events on the context's
    # stream over launches at the bench batch (all layers, so weights stream from HBM)
    n_win = min(args.max_windows, n_clips)
    model.ctx.encode([3000 * i for i in range(n_win)], [3000] * n_win)
    from whisper.decoding import DecodingTask
    task = DecodingTask(model, whisper.DecodingOptions(language="en", beam_size=args.beam))
    model.ctx.decode_begin(task.wh_opts(), [task.initial_tokens] * n_win, [task.sot_index] * n_win)
    rows = n_win * args.beam
    # in-step: every k_proj of 3 eager steps bracketed by HIP events on the context
    # stream, each behind its real producer kernel (what rocprof sees in the step);
    # back-to-back: the same launches queued without their producers (time_stage 2)
    gemv_ms = model.ctx.time_stage(7, 3)
    gemv_b2b_ms = model.ctx.time_stage(2, 3)
    gemv_bytes = projection_bytes_per_launch(dims, rows)
    xattn_ms = model.ctx.time_stage(3, 3)
    xattn_bytes = cross_attn_bytes_per_launch(dims, n_win, rows)
    step_ms = model.ctx.time_stage(0, 20)
    mean_ctx = 3 + 112  # mid-window self-KV length for the byte count
    step_bytes = decoder_step_bytes(dims, n_win, args.beam, mean_ctx)

    def gbs(b, ms):
        return b / (ms * 1e-3) / 1e9

    traffic = load_traffic("k_proj")
    out = {
        "metric": "xRT (audio-s/s) large-v3 beam=5 @1/2/4/8 GPU; p50 per-token decode ms",
        "value": round(world * args.seconds * args.steps / elapsed_max, 3),
        "unit": "audio-s/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed_max * 1e3 / args.steps, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp16" if args.dtype == "fp16" else "f32",
        "data": "synthetic: seeded N(0,0.1^2)+440 Hz audio, seeded random-init weights at real dims",
        "config": {"workload": f"{args.model} beam={args.beam} transcribe(), {args.seconds:.0f} s audio per GPU, "
                               f"30 s clip grid, condition_on_previous_text=False, temperature=0"
                               + (", word_timestamps=True" if args.word_timestamps else ""),
                   "model": args.model, "global_batch": n_clips * world, "seq_len": 448,
                   "parallelism": f"windows sharded over {world} GPU(s), RCCL all-reduce(max)+gather"},
        "p50_token_ms": round(p50_token_ms, 4),
        "mean_token_ms": round(ms_per_token, 4),
        "tokens_per_window": round(gathered[0][1] / max(1, n_clips), 1),
        "encoder_ms_per_window": round(enc_ms / max(enc_windows, 1), 3),
        "encoder_tflops": round(encoder_flops(dims) * enc_windows / (enc_ms * 1e-3) / 1e12, 1) if enc_ms else None,
        "roofline": {"bound": "hbm", "kernel": f"k_proj split-K projection ({rows} rows, avg of the six "
                                                f"per decoder layer)",
                     "achieved": round(gbs(gemv_bytes, gemv_ms), 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(gbs(gemv_bytes, gemv_ms) / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "bytes_per_launch": gemv_bytes, "ms_per_launch": round(gemv_ms, 5),
                     "timing": "HIP events around each launch inside eager decoder steps",
                     "ms_per_launch_back_to_back": round(gemv_b2b_ms, 5)},
        "roofline_cross_attn": {"bound": "hbm", "kernel": f"k_cross_attn1 ({n_win} windows x {args.beam} beams)",
                                "achieved": round(gbs(xattn_bytes, xattn_ms), 1), "peak": HBM_PEAK_GBS,
                                "frac": round(gbs(xattn_bytes, xattn_ms) / HBM_PEAK_GBS, 4),
                                "bytes_per_launch": xattn_bytes, "ms_per_launch": round(xattn_ms, 5)},
        "roofline_step": {"bound": "hbm", "kernel": f"decoder step hipGraph ({n_win} windows x {args.beam} beams)",
                          "achieved": round(gbs(step_bytes, step_ms), 1), "peak": HBM_PEAK_GBS,
                          "frac": round(gbs(step_bytes, step_ms) / HBM_PEAK_GBS, 4),
                          "bytes_per_launch": step_bytes, "ms_per_launch": round(step_ms, 4)},
    }
    if rank == 0 and world == 1 and args.cpu_baseline and sd is not None:
        try:
            out["cpu_baseline"] = cpu_baseline(args.model, sd, audio, args.beam, args.cpu_steps)
        except Exception as e:  # reported, never fatal for the GPU number
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
