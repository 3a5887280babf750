"""Golden-vector generator: runs the REFERENCE (/root/reference) on seeded inputs.

TEST INFRASTRUCTURE ONLY.  This script is run by hand in the survey/build
container, where /root/reference exists.  It imports the reference fork's own
``whisper`` package (CPU PyTorch path, ``use_coreml=False``) with two
stand-in modules for the absent third-party packages (oracle/standins/:
``tiktoken`` = plain BPE, ``numba`` = identity ``jit``) and
writes small fixtures to tests/golden/.  Nothing from the reference travels:
only inputs (as seeds) and outputs (as arrays).

Weights come from whisper.coreml_amd/whisper/synthetic.py (our own seeded
generator, loaded by file path so it does not clash with the reference's
``whisper`` package); the GPU box regenerates the identical weights.

Usage:  python oracle/gen_golden.py [micro tiny.en turbo large-v3 mel tokens dtw]
"""

import importlib.util
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden")
REF = "/root/reference"

sys.path.insert(0, REF)
sys.path.insert(0, os.path.join(HERE, "standins"))

import torch  # noqa: E402

torch.set_num_threads(os.cpu_count() or 8)

import whisper as refw  # noqa: E402  (the REFERENCE package)
from whisper import audio as ref_audio  # noqa: E402
from whisper import decoding as ref_decoding  # noqa: E402
from whisper import timing as ref_timing  # noqa: E402
from whisper import tokenizer as ref_tok  # noqa: E402
from whisper.model import ModelDimensions, Whisper  # noqa: E402

assert os.path.realpath(os.path.dirname(refw.__file__)).startswith(REF), refw.__file__

_spec = importlib.util.spec_from_file_location(
    "wh_synthetic", os.path.join(REPO, "whisper.coreml_amd", "whisper", "synthetic.py"))
syn = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(syn)

N_SAMPLES = ref_audio.N_SAMPLES


def build_ref_model(name: str, seed: int = 0, eot_scale=None):
    dims = syn.MODEL_DIMS[name]
    sd = syn.synthetic_state_dict(dims, seed)
    if eot_scale is not None:
        syn.scale_eot_embedding(sd, dims, eot_scale)
    model = Whisper(ModelDimensions(**dims), False, name)
    ref_keys = set(model.state_dict().keys())
    assert ref_keys == set(sd.keys()), (ref_keys ^ set(sd.keys()))
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    if name in refw._ALIGNMENT_HEADS:
        model.set_alignment_heads(refw._ALIGNMENT_HEADS[name])
    model.eval()
    return model, sd


class MarginRecorder:
    """Wraps GreedyDecoder.update to record the post-filter top-2 margin per step."""

    def __init__(self):
        self.margins = []
        self._orig = ref_decoding.GreedyDecoder.update
        rec = self

        def update(this, tokens, logits, sum_logprobs):
            top2 = torch.topk(logits.float(), 2, dim=-1).values
            rec.margins.append((top2[:, 0] - top2[:, 1]).tolist())
            return rec._orig(this, tokens, logits, sum_logprobs)

        ref_decoding.GreedyDecoder.update = update

    def close(self):
        ref_decoding.GreedyDecoder.update = self._orig


class StepRecorder:
    """Wraps PyTorchInference.logits / rearrange_kv_cache (decoding.py:151-204) to record,
    for every decoder call of the reference's _main_loop (decoding.py:707-737): the last
    input token of each row, the top-K of the raw last-position logits (before the logit
    filters modify them in place, decoding.py:726-727) with the row's logsumexp, and the
    beam reorder indices.  This is the trajectory a teacher-forced step replays."""

    def __init__(self, k: int = 32):
        self.tok, self.topv, self.topi, self.lse, self.src = [], [], [], [], []
        self._orig = (ref_decoding.PyTorchInference.logits, ref_decoding.PyTorchInference.rearrange_kv_cache)
        rec, orig_logits, orig_rearr = self, self._orig[0], self._orig[1]

        def logits(this, tokens, audio_features):
            out, qk = orig_logits(this, tokens, audio_features)
            last = out[:, -1].detach().float().clone()
            v, i = torch.topk(last, k, dim=-1)
            rec.tok.append(tokens[:, -1].tolist())
            rec.topv.append(v.numpy())
            rec.topi.append(i.numpy())
            rec.lse.append(torch.logsumexp(last.double(), dim=-1).numpy())
            return out, qk

        def rearrange(this, source_indices):
            rec.src.append(list(source_indices))
            return orig_rearr(this, source_indices)

        ref_decoding.PyTorchInference.logits = logits
        ref_decoding.PyTorchInference.rearrange_kv_cache = rearrange

    def close(self):
        ref_decoding.PyTorchInference.logits, ref_decoding.PyTorchInference.rearrange_kv_cache = self._orig

    def pack(self, prefix: str, out: dict):
        out[f"{prefix}_tok"] = np.asarray(self.tok, dtype=np.int32)          # [steps][rows]
        out[f"{prefix}_topv"] = np.stack(self.topv).astype(np.float32)       # [steps][rows][K]
        out[f"{prefix}_topi"] = np.stack(self.topi).astype(np.int32)
        out[f"{prefix}_lse"] = np.stack(self.lse).astype(np.float64)         # [steps][rows]
        if self.src:
            out[f"{prefix}_src"] = np.asarray(self.src, dtype=np.int32)      # [steps][rows]


def step_goldens(name: str, seed: int = 0, audio_seed: int = 1, mixed_seeds=(2, 3, 4)):
    """Per-step reference trajectories for the fp16/beam tolerance test (teacher-forced
    steps through wh_step / wh_reorder_kv) and fixed-work tokens of further windows for
    the co-batched (bench-configuration) parity test."""
    t0 = time.time()
    model, _ = build_ref_model(name, seed)
    dims = syn.MODEL_DIMS[name]
    eot = 50257 if dims["n_vocab"] >= 51865 else 50256
    out = {"seed": np.int32(seed), "audio_seed": np.int32(audio_seed), "mixed_seeds": np.asarray(mixed_seeds, np.int32)}

    def window(aseed):
        audio = syn.synthetic_audio(30.0, seed=aseed)
        mel = ref_audio.log_mel_spectrogram(audio, dims["n_mels"], padding=N_SAMPLES)
        return ref_audio.pad_or_trim(mel[:, :3000], 3000)

    seg = window(audio_seed)
    for kind, extra in [("greedy_fixed", {}), ("beam_fixed", dict(beam_size=5))]:
        rec = StepRecorder()
        r = refw.decode(model, seg, ref_decoding.DecodingOptions(
            temperature=0.0, suppress_tokens=f"-1,{eot}", language="en", fp16=False, **extra))
        rec.close()
        rec.pack(f"tf_{kind}", out)
        out[f"tf_{kind}_tokens"] = np.asarray(r.tokens, dtype=np.int32)
        print(f"[{name}] steps {kind}: {len(rec.tok)} calls {time.time()-t0:.1f}s", flush=True)
    for s in mixed_seeds:
        seg = window(s)
        r = refw.decode(model, seg, ref_decoding.DecodingOptions(
            temperature=0.0, beam_size=5, suppress_tokens=f"-1,{eot}", language="en", fp16=False))
        pack_result(f"mixed{s}_beam_fixed", r, out)
        print(f"[{name}] mixed window seed {s}: {len(r.tokens)} tok {time.time()-t0:.1f}s", flush=True)
    np.savez_compressed(os.path.join(OUT, f"{name}_steps.npz"), **out)


def step_goldens_mixed(name: str, seed: int = 0, audio_seeds=(2, 3, 4)):
    """Teacher-forced beam trajectories of further audio windows, so that a co-batched
    teacher-forced test holds every window of a mixed batch to its own reference
    trajectory (the kernel-selection branches by window count: wh_kernels.hip
    launch_cross_attn, wh_proj.hip launch_proj_partial)."""
    t0 = time.time()
    model, _ = build_ref_model(name, seed)
    dims = syn.MODEL_DIMS[name]
    eot = 50257 if dims["n_vocab"] >= 51865 else 50256
    out = {"seed": np.int32(seed), "audio_seeds": np.asarray(audio_seeds, np.int32)}
    for s in audio_seeds:
        audio = syn.synthetic_audio(30.0, seed=s)
        mel = ref_audio.log_mel_spectrogram(audio, dims["n_mels"], padding=N_SAMPLES)
        seg = ref_audio.pad_or_trim(mel[:, :3000], 3000)
        rec = StepRecorder()
        r = refw.decode(model, seg, ref_decoding.DecodingOptions(
            temperature=0.0, beam_size=5, suppress_tokens=f"-1,{eot}", language="en", fp16=False))
        rec.close()
        rec.pack(f"s{s}_tf_beam_fixed", out)
        out[f"s{s}_tf_beam_fixed_tokens"] = np.asarray(r.tokens, dtype=np.int32)
        print(f"[{name}] mixed steps seed {s}: {len(rec.tok)} calls {time.time()-t0:.1f}s", flush=True)
    np.savez_compressed(os.path.join(OUT, f"{name}_steps_mixed.npz"), **out)


def prefix_goldens(names=("micro", "tiny.en")):
    """DecodingOptions(prefix=...) at the default sample_len (max_prefix_len = 0: Python's
    [-0:] keeps the WHOLE prefix, decoding.py:620-626), at sample_len = 200 (keeps the
    last 24 tokens) and 300 (max_prefix_len = -76: drops the FIRST 76), plus a string
    prefix; greedy and beam 5, natural decoding."""
    res = {}
    for name in names:
        model, _ = build_ref_model(name)
        dims = syn.MODEL_DIMS[name]
        audio = syn.synthetic_audio(30.0, seed=1)
        mel = ref_audio.log_mel_spectrogram(audio, dims["n_mels"], padding=N_SAMPLES)
        seg = ref_audio.pad_or_trim(mel[:, :3000], 3000)
        pre = [int(t) for t in np.random.default_rng(9).integers(300, 20000, 100)]
        cases = {
            "list_default": dict(prefix=pre),
            "list_len200": dict(prefix=pre, sample_len=200),
            "list_len300": dict(prefix=pre, sample_len=300),
            "str_default": dict(prefix="And so my fellow Americans"),
            "list_default_beam": dict(prefix=pre[:30], beam_size=5),
            "prompt_prefix": dict(prefix=pre[:12], prompt=list(range(1000, 1040))),
        }
        out = {}
        for key, kw in cases.items():
            t0 = time.time()
            r = refw.decode(model, seg, ref_decoding.DecodingOptions(temperature=0.0, language="en", fp16=False, **kw))
            out[key] = dict(options={k: v for k, v in kw.items()}, tokens=[int(t) for t in r.tokens],
                            avg_logprob=float(r.avg_logprob), no_speech_prob=float(r.no_speech_prob))
            print(f"[{name}] prefix {key}: {len(r.tokens)} tok {time.time()-t0:.1f}s", flush=True)
        res[name] = dict(seed=0, audio_seed=1, cases=out)
        del model
    with open(os.path.join(OUT, "prefix.json"), "w") as f:
        json.dump(res, f, indent=0)


class FinalizeRecorder:
    """Wraps BeamSearchDecoder.finalize (decoding.py:411-431) to record the candidates the
    ranker sees: their lengths after trimming at EOT and their summed log-probabilities
    (so a test can tell whether length_penalty had a choice to make)."""

    def __init__(self):
        self.cands = []
        self._orig = ref_decoding.BeamSearchDecoder.finalize
        rec = self

        def finalize(this, preceding_tokens, sum_logprobs):
            toks, lps = rec._orig(this, preceding_tokens, sum_logprobs)
            # [untrimmed length (sot sequence .. EOT), summed log-probability], in the
            # finished set's insertion order
            rec.cands.append([[len(t.tolist()), float(lp)] for t, lp in zip(toks[0], lps[0])])
            return toks, lps

        ref_decoding.BeamSearchDecoder.finalize = finalize

    def close(self):
        ref_decoding.BeamSearchDecoder.finalize = self._orig


BEAM_OPTION_CASES = {
    # decoding.py:339-345: max_candidates = round(beam_size * patience) (Python rounds half to even)
    "patience2": dict(beam_size=5, patience=2.0),
    "patience0.5": dict(beam_size=5, patience=0.5),      # round(2.5) = 2
    "beam3_patience1.5": dict(beam_size=3, patience=1.5),  # round(4.5) = 4
    # decoding.py:223-240: score = sum_logprob / ((5 + len) / 6) ** length_penalty
    "lp0.0": dict(beam_size=5, length_penalty=0.0),
    "lp0.6": dict(beam_size=5, length_penalty=0.6),
    "lp1.0": dict(beam_size=5, length_penalty=1.0),
    "patience2_lp0.6": dict(beam_size=5, patience=2.0, length_penalty=0.6),
    "default": dict(beam_size=5),
}


# With the seeded random weights EOT never wins a natural decode (every candidate runs to
# sample_len, so patience and length_penalty have nothing to choose between).  Scaling the
# EOT row of the token embedding (= its logit, decoder.py:319-320) makes EOT compete:
# these factors give finished candidates of many lengths (micro 8-22 tokens, tiny.en 5-117)
# and a length_penalty that changes the chosen candidate (micro).
BEAM_OPTION_EOT_SCALE = {"micro": -3.0, "tiny.en": 3.3}


def beam_option_goldens(names=("micro", "tiny.en"), audio_seeds=(1, 2, 3)):
    """Non-default beam options: natural-mode decodes (EOT allowed)
    of seeded 30 s windows with patience and length_penalty, tokens / avg_logprob /
    no_speech_prob plus the finished candidates the ranker chose from, on the seeded
    weights with the EOT embedding row scaled (BEAM_OPTION_EOT_SCALE)."""
    res = {}
    for name in names:
        model, _ = build_ref_model(name, eot_scale=BEAM_OPTION_EOT_SCALE[name])
        dims = syn.MODEL_DIMS[name]
        per_seed = {}
        for aseed in audio_seeds:
            audio = syn.synthetic_audio(30.0, seed=aseed)
            mel = ref_audio.log_mel_spectrogram(audio, dims["n_mels"], padding=N_SAMPLES)
            seg = ref_audio.pad_or_trim(mel[:, :3000], 3000)
            out = {}
            for key, kw in BEAM_OPTION_CASES.items():
                t0 = time.time()
                rec = FinalizeRecorder()
                r = refw.decode(model, seg, ref_decoding.DecodingOptions(temperature=0.0, language="en", fp16=False,
                                                                         **kw))
                rec.close()
                out[key] = dict(options=kw, tokens=[int(t) for t in r.tokens], avg_logprob=float(r.avg_logprob),
                                no_speech_prob=float(r.no_speech_prob), candidates=rec.cands[0])
                print(f"[{name}] seed {aseed} {key}: {len(r.tokens)} tok, {len(rec.cands[0])} candidates "
                      f"{sorted(c[0] for c in rec.cands[0])} {time.time()-t0:.1f}s", flush=True)
            per_seed[str(aseed)] = out
        res[name] = dict(seed=0, eot_scale=BEAM_OPTION_EOT_SCALE[name], audio_seeds=list(audio_seeds), cases=per_seed)
        del model
    with open(os.path.join(OUT, "beam_options.json"), "w") as f:
        json.dump(res, f, indent=0)


def words_beam_goldens(name: str = "large-v3"):
    """Config 5 as specified (beam 5 + word timestamps) at real dims: the reference's
    transcribe(..., beam_size=5, word_timestamps=True) on the 65 s clip grid, merged
    into <name>_words.json next to the greedy run."""
    import base64
    model, _ = build_ref_model(name)
    path = os.path.join(OUT, f"{name}_words.json")
    with open(path) as f:
        res = json.load(f)
    dims = syn.MODEL_DIMS[name]
    tok = ref_tok.get_tokenizer(dims["n_vocab"] >= 51865, num_languages=dims["n_vocab"] - 51765 -
                                int(dims["n_vocab"] >= 51865), language="en", task="transcribe")
    audio = syn.synthetic_audio(res["audio_seconds"], seed=res["audio_seed"])
    kw = dict(beam_size=5, condition_on_previous_text=False, clip_timestamps="0,30,30,60,60", word_timestamps=True)
    t0 = time.time()
    out = refw.transcribe(model, audio, temperature=0.0, language="en", fp16=False, verbose=None, **kw)
    segs, ids = [], set()
    for s_ in out["segments"]:
        ids.update(int(t) for t in s_["tokens"])
        segs.append(dict(seek=s_["seek"], start=s_["start"], end=s_["end"], tokens=[int(t) for t in s_["tokens"]],
                         words=[dict(word=w["word"], start=w["start"], end=w["end"],
                                     probability=float(w["probability"])) for w in s_.get("words", [])]))
    res["runs"]["clip_beam_words"] = kw
    res["segments"]["clip_beam_words"] = segs
    dec = tok.encoding._decoder
    for i in sorted(ids):
        if i < tok.eot:
            res["token_bytes"][str(i)] = base64.b64encode(dec[i]).decode()
    print(f"[{name}] transcribe clip_beam_words: {len(segs)} segs {time.time()-t0:.1f}s", flush=True)
    with open(path, "w") as f:
        json.dump(res, f, indent=0)


def pack_result(prefix: str, r, out: dict):
    out[f"{prefix}_tokens"] = np.asarray(r.tokens, dtype=np.int32)
    out[f"{prefix}_avg_logprob"] = np.float64(r.avg_logprob)
    out[f"{prefix}_no_speech_prob"] = np.float64(r.no_speech_prob)


def topk_pack(prefix: str, row: torch.Tensor, out: dict, k: int = 64):
    v, i = torch.topk(row.float(), k)
    out[f"{prefix}_topv"] = v.numpy().astype(np.float32)
    out[f"{prefix}_topi"] = i.numpy().astype(np.int32)
    out[f"{prefix}_lse"] = np.float64(torch.logsumexp(row.double(), 0).item())
    out[f"{prefix}_mean"] = np.float64(row.double().mean().item())
    out[f"{prefix}_std"] = np.float64(row.double().std().item())


def model_goldens(name: str, seed: int = 0, audio_seed: int = 1, full: bool = False,
                  beam_natural: bool = True):
    t0 = time.time()
    model, sd = build_ref_model(name, seed)
    dims = syn.MODEL_DIMS[name]
    out = {"seed": np.int32(seed), "audio_seed": np.int32(audio_seed),
           "weights_checksum": np.float64(syn.state_dict_checksum(sd))}
    del sd
    lang_opts = dict(language="en", fp16=False)
    audio = syn.synthetic_audio(30.0, seed=audio_seed)
    mel = ref_audio.log_mel_spectrogram(audio, dims["n_mels"], padding=N_SAMPLES)
    mel_seg = ref_audio.pad_or_trim(mel[:, :3000], 3000)
    out["mel_window_sum"] = np.float64(mel_seg.double().sum().item())
    with torch.no_grad():
        xa = model.encoder(mel_seg.unsqueeze(0))[0]
        out["xa_rownorm"] = xa.double().norm(dim=1).numpy()
        out["xa_head"] = xa[:64].numpy().astype(np.float32)
        out["xa_tail"] = xa[-64:].numpy().astype(np.float32)
        if full:
            out["xa_full"] = xa.numpy().astype(np.float32)
        ck, cv = model.decoder.crossKVCaches(xa.unsqueeze(0))
        # ck: (L, H, 64, 1500); cv: (L, H, 1500, 64)
        out["ck_norm"] = ck.double().norm(dim=(2, 3)).numpy()
        out["cv_norm"] = cv.double().norm(dim=(2, 3)).numpy()
        out["ck_slice"] = (ck[:, :, :, :32] if full else ck[[0, -1]][:, :, :, :8]).numpy().astype(np.float32)
        tok = refw.tokenizer.get_tokenizer(model.is_multilingual, num_languages=model.num_languages,
                                           language="en", task="transcribe")
        sot = list(tok.sot_sequence)
        out["sot_sequence"] = np.asarray(sot, dtype=np.int32)
        logits, cross_qks, _ = model.decoder(torch.tensor([sot]), xa.unsqueeze(0), 0, None)
        topk_pack("first_last", logits[0, -1], out)
        topk_pack("first_sot", logits[0, 0], out)
        if full:
            out["first_last_full"] = logits[0, -1].numpy().astype(np.float32)
        # a prompt-conditioned first pass (sequential transcribe mode, decoding.py:628-638)
        prompt = [tok.sot_prev] + list(range(1000, 1040)) + sot
        out["prompt_tokens"] = np.asarray(prompt, dtype=np.int32)
        model.decoder.cross_k_caches = None
        logits_p, _, _ = model.decoder(torch.tensor([prompt]), xa.unsqueeze(0), 0, None)
        topk_pack("prompt_last", logits_p[0, -1], out)
    print(f"[{name}] encoder+first pass {time.time()-t0:.1f}s", flush=True)

    # greedy, natural
    rec = MarginRecorder()
    r = refw.decode(model, mel_seg, ref_decoding.DecodingOptions(temperature=0.0, **lang_opts))
    rec.close()
    pack_result("greedy", r, out)
    out["greedy_margins"] = np.asarray([m[0] for m in rec.margins], dtype=np.float32)
    print(f"[{name}] greedy natural {len(r.tokens)} tok {time.time()-t0:.1f}s", flush=True)
    # greedy, fixed work (EOT suppressed -> 224 steps)
    eot = tok.eot
    rec = MarginRecorder()
    r = refw.decode(model, mel_seg, ref_decoding.DecodingOptions(
        temperature=0.0, suppress_tokens=f"-1,{eot}", **lang_opts))
    rec.close()
    pack_result("greedy_fixed", r, out)
    out["greedy_fixed_margins"] = np.asarray([m[0] for m in rec.margins], dtype=np.float32)
    print(f"[{name}] greedy fixed {len(r.tokens)} tok {time.time()-t0:.1f}s", flush=True)
    # greedy with a prompt
    r = refw.decode(model, mel_seg, ref_decoding.DecodingOptions(
        temperature=0.0, prompt=list(range(1000, 1040)), **lang_opts))
    pack_result("greedy_prompt", r, out)
    # beam search
    if beam_natural:
        r = refw.decode(model, mel_seg, ref_decoding.DecodingOptions(temperature=0.0, beam_size=5, **lang_opts))
        pack_result("beam", r, out)
        print(f"[{name}] beam natural {len(r.tokens)} tok {time.time()-t0:.1f}s", flush=True)
    r = refw.decode(model, mel_seg, ref_decoding.DecodingOptions(
        temperature=0.0, beam_size=5, suppress_tokens=f"-1,{eot}", **lang_opts))
    pack_result("beam_fixed", r, out)
    print(f"[{name}] beam fixed {len(r.tokens)} tok {time.time()-t0:.1f}s", flush=True)
    # without timestamps (sot_sequence_including_notimestamps)
    r = refw.decode(model, mel_seg, ref_decoding.DecodingOptions(
        temperature=0.0, without_timestamps=True, **lang_opts))
    pack_result("greedy_notime", r, out)
    return model, out


def transcribe_goldens(model, name: str, out: dict):
    """transcribe() on 35 s + 65 s audio: sharded mode and sequential mode."""
    segs_all = {}
    audio = syn.synthetic_audio(65.0, seed=7)
    runs = {
        "clip_beam": dict(beam_size=5, condition_on_previous_text=False, clip_timestamps="0,30,30,60,60"),
        "clip_greedy": dict(condition_on_previous_text=False, clip_timestamps="0,30,30,60,60"),
        "seq_greedy": dict(condition_on_previous_text=True),
        "seq_beam": dict(beam_size=5, condition_on_previous_text=True),
    }
    for key, kw in runs.items():
        t0 = time.time()
        res = refw.transcribe(model, audio, temperature=0.0, language="en", fp16=False, verbose=None, **kw)
        segs_all[key] = [
            dict(seek=s["seek"], start=s["start"], end=s["end"], tokens=s["tokens"],
                 avg_logprob=s["avg_logprob"], no_speech_prob=s["no_speech_prob"],
                 temperature=s["temperature"])
            for s in res["segments"]]
        print(f"[{name}] transcribe {key}: {len(res['segments'])} segs {time.time()-t0:.1f}s", flush=True)
    with open(os.path.join(OUT, f"{name}_transcribe.json"), "w") as f:
        json.dump(dict(audio_seconds=65.0, audio_seed=7, runs=runs, segments=segs_all), f, indent=0)


def words_goldens(model, name: str, run_keys=None):
    """Word-level timestamps (config 5 / SURVEY §8 a19): the reference's own
    find_alignment on one window, and transcribe(word_timestamps=True) on 65 s of
    audio; plus the decoded bytes of every token id involved (the product ships no
    BPE rank file, so tests install these few ids with tokenizer.set_token_bytes)."""
    import base64
    dims = syn.MODEL_DIMS[name]
    tok = ref_tok.get_tokenizer(dims["n_vocab"] >= 51865, num_languages=dims["n_vocab"] - 51765 -
                                int(dims["n_vocab"] >= 51865), language="en", task="transcribe")
    audio = syn.synthetic_audio(65.0, seed=7)
    ids = set()
    res = {"audio_seconds": 65.0, "audio_seed": 7, "runs": {}, "segments": {}, "find_alignment": {}}
    # direct find_alignment on window 0 with a fixed text
    mel = ref_audio.log_mel_spectrogram(audio, dims["n_mels"], padding=N_SAMPLES)
    seg = ref_audio.pad_or_trim(mel[:, :3000], 3000)
    with torch.no_grad():
        model.decoder.cross_k_caches, model.decoder.cross_v_caches = model.decoder.crossKVCaches(
            model.encoder(seg.unsqueeze(0)))
        model.text_offset = 0
    rng = np.random.default_rng(5)
    for key, ntok, nf in [("a", 17, 3000), ("b", 40, 2200), ("c", 3, 800)]:
        text = [int(t) for t in rng.integers(0, tok.eot, ntok)]
        ids.update(text)
        al = ref_timing.find_alignment(model, tok, text, nf)
        res["find_alignment"][key] = dict(
            text_tokens=text, num_frames=nf,
            words=[dict(word=w.word, tokens=[int(t) for t in w.tokens], start=float(w.start), end=float(w.end),
                        probability=float(w.probability)) for w in al])
    runs = {
        "seq_greedy_words": dict(condition_on_previous_text=True, word_timestamps=True),
        "clip_beam_words": dict(beam_size=5, condition_on_previous_text=False, clip_timestamps="0,30,30,60,60",
                                word_timestamps=True),
        "clip_greedy_words": dict(condition_on_previous_text=False, clip_timestamps="0,30,30,60,60",
                                  word_timestamps=True),
        "seq_greedy_halluc": dict(condition_on_previous_text=True, word_timestamps=True,
                                  hallucination_silence_threshold=2.0),
    }
    if run_keys is not None:
        runs = {k: v for k, v in runs.items() if k in run_keys}
    for key, kw in runs.items():
        t0 = time.time()
        out = refw.transcribe(model, audio, temperature=0.0, language="en", fp16=False, verbose=None, **kw)
        segs = []
        for s_ in out["segments"]:
            ids.update(int(t) for t in s_["tokens"])
            segs.append(dict(seek=s_["seek"], start=s_["start"], end=s_["end"], tokens=[int(t) for t in s_["tokens"]],
                             words=[dict(word=w["word"], start=w["start"], end=w["end"],
                                         probability=float(w["probability"])) for w in s_.get("words", [])]))
        res["runs"][key] = kw
        res["segments"][key] = segs
        print(f"[{name}] transcribe {key}: {len(segs)} segs {time.time()-t0:.1f}s", flush=True)
    dec = tok.encoding._decoder
    res["token_bytes"] = {str(i): base64.b64encode(dec[i]).decode() for i in sorted(ids) if i < tok.eot}
    res["encoding"] = tok.encoding.name
    with open(os.path.join(OUT, f"{name}_words.json"), "w") as f:
        json.dump(res, f, indent=0)


def mel_goldens():
    out = {}
    out["filters_80"] = ref_audio.mel_filters("cpu", 80).numpy()
    out["filters_128"] = ref_audio.mel_filters("cpu", 128).numpy()
    cases = [("a", 1.0, 11, 80, 0), ("b", 2.0, 12, 128, 0), ("c", 31.5, 13, 128, N_SAMPLES),
             ("d", 30.0, 14, 80, N_SAMPLES), ("e", 0.5, 15, 80, 0), ("f", 600.0, 16, 128, N_SAMPLES)]
    meta = []
    for tag, sec, seed, nm, pad in cases:
        audio = syn.synthetic_audio(sec, seed=seed)
        m = ref_audio.log_mel_spectrogram(audio, nm, padding=pad).numpy()
        meta.append(dict(tag=tag, seconds=sec, seed=seed, n_mels=nm, padding=pad, frames=int(m.shape[1])))
        if m.shape[1] <= 256:
            out[f"{tag}_full"] = m
        else:
            for lo, hi in [(0, 48), (m.shape[1] // 2 - 8, m.shape[1] // 2 + 8), (m.shape[1] - 3016, m.shape[1] - 2984),
                           (m.shape[1] - 16, m.shape[1])]:
                out[f"{tag}_{lo}"] = m[:, lo:hi]
        out[f"{tag}_max"] = np.float64(m.max())
        out[f"{tag}_sum"] = np.float64(m.astype(np.float64).sum())
        out[f"{tag}_colsum"] = m.astype(np.float64).sum(axis=0)
    out["meta"] = np.asarray(json.dumps(meta))
    np.savez_compressed(os.path.join(OUT, "mel.npz"), **out)
    print("mel goldens:", [m["frames"] for m in meta])


def _is_ws(b: bytes) -> bool:
    try:
        return b.decode("utf-8").strip() == ""
    except UnicodeDecodeError:
        return False


def token_goldens():
    res = {}
    for multilingual, nl in [(True, 100), (True, 99), (False, 99)]:
        tok = ref_tok.get_tokenizer(multilingual, num_languages=nl, language="en", task="transcribe")
        key = f"{'multilingual' if multilingual else 'gpt2'}_{nl}"
        res[key] = dict(
            eot=tok.eot, sot=tok.sot, translate=tok.translate, transcribe=tok.transcribe,
            sot_lm=tok.sot_lm, sot_prev=tok.sot_prev, no_speech=tok.no_speech,
            no_timestamps=tok.no_timestamps, timestamp_begin=tok.timestamp_begin,
            sot_sequence=list(tok.sot_sequence), non_speech_tokens=list(tok.non_speech_tokens),
            blank=tok.encode(" "), n_vocab=tok.encoding.n_vocab,
            all_language_tokens=list(tok.all_language_tokens),
            fellow=tok.encode(" And so my fellow Americans"),
            # ids whose decoded text is whitespace only: transcribe.py:494-499 clears
            # segments whose text .strip() == "" (needs no BPE decoder with this list)
            whitespace_tokens=sorted(i for b, i in tok.encoding._ranks.items()
                                     if _is_ws(b)),
        )
    with open(os.path.join(OUT, "tokens.json"), "w") as f:
        json.dump(res, f, indent=0)
    print("token goldens:", {k: len(v["non_speech_tokens"]) for k, v in res.items()})


def planted_dtw(N, M, rng):
    """Same construction as reference tests/test_timing.py:22-49 (own seeded rng)."""
    steps = np.concatenate([np.zeros(N - 1), np.ones(M - 1)])
    rng.shuffle(steps)
    x = rng.random((N, M)).astype(np.float32)
    i, j, k = 0, 0, 0
    trace = []
    while True:
        x[i, j] -= 1
        trace.append((i, j))
        if k == len(steps):
            break
        if k + 1 < len(steps) and steps[k] != steps[k + 1]:
            i += 1
            j += 1
            k += 2
            continue
        if steps[k] == 0:
            i += 1
        if steps[k] == 1:
            j += 1
        k += 1
    return x, np.array(trace).T


def dtw_goldens():
    out = {}
    rng = np.random.default_rng(42)
    for N, M in [(10, 20), (32, 16), (123, 1500), (234, 189)]:
        x, trace = planted_dtw(N, M, rng)
        out[f"planted_{N}x{M}_x"] = x
        out[f"planted_{N}x{M}_trace"] = trace.astype(np.int32)
        got = ref_timing.dtw_cpu(x.astype(np.float64))
        assert np.array_equal(got, trace), (N, M)
    for N, M in [(8, 40), (57, 300), (120, 750)]:
        x = rng.standard_normal((N, M)).astype(np.float32)
        out[f"rand_{N}x{M}_x"] = x
        out[f"rand_{N}x{M}_path"] = np.asarray(ref_timing.dtw_cpu(x.astype(np.float64)), dtype=np.int32)
    for shape in [(10,), (1, 15), (4, 5, 345), (2, 3, 20, 100)]:
        x = rng.standard_normal(shape).astype(np.float32)
        for w in (3, 5, 7, 13):
            key = "x".join(map(str, shape))
            out[f"med_{key}_x"] = x
            out[f"med_{key}_w{w}"] = ref_timing.median_filter(torch.from_numpy(x), w).numpy()
    np.savez_compressed(os.path.join(OUT, "dtw.npz"), **out)
    print("dtw goldens:", len(out))


def checkpoint_goldens(name: str = "micro", seed: int = 0, audio_seed: int = 1):
    """A checkpoint in the released format: {"dims", "model_state_dict"}
    from the reference's own Whisper.state_dict() on the seeded weights, every tensor fp16
    as OpenAI's released .pt files store them, written with torch.save to
    tests/golden/<name>_ckpt.pt; then the REFERENCE's load_model(path) (__init__.py:151-166)
    loads it back and decodes a seeded 30 s window (fp32 CPU path): greedy and beam 5 with
    EOT suppressed (224 steps of fixed work) and natural greedy.  Tokens / avg_logprob go
    to tests/golden/<name>_ckpt.json with the checkpoint's sha256."""
    import hashlib
    model, _ = build_ref_model(name, seed)
    dims = syn.MODEL_DIMS[name]
    state = {k: v.detach().half().contiguous() for k, v in model.state_dict().items()}
    path = os.path.join(OUT, f"{name}_ckpt.pt")
    torch.save({"dims": dict(dims), "model_state_dict": state}, path)
    del model
    ref = refw.load_model(path, device="cpu")
    ref.eval()
    tok = ref_tok.get_tokenizer(ref.is_multilingual, num_languages=ref.num_languages, language="en",
                                task="transcribe")
    audio = syn.synthetic_audio(30.0, seed=audio_seed)
    mel = ref_audio.log_mel_spectrogram(audio, dims["n_mels"], padding=N_SAMPLES)
    seg = ref_audio.pad_or_trim(mel[:, :3000], 3000)
    cases = {"greedy_fixed": dict(suppress_tokens=f"-1,{tok.eot}"),
             "beam_fixed": dict(beam_size=5, suppress_tokens=f"-1,{tok.eot}"),
             "greedy_natural": {}}
    out = {}
    for key, kw in cases.items():
        r = refw.decode(ref, seg, ref_decoding.DecodingOptions(temperature=0.0, language="en", fp16=False, **kw))
        out[key] = dict(options=kw, tokens=[int(t) for t in r.tokens], avg_logprob=float(r.avg_logprob),
                        no_speech_prob=float(r.no_speech_prob))
        print(f"[{name} checkpoint] {key}: {len(r.tokens)} tokens, avg_logprob {r.avg_logprob:.5f}", flush=True)
    with open(path, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()
    with open(os.path.join(OUT, f"{name}_ckpt.json"), "w") as f:
        json.dump(dict(checkpoint=os.path.basename(path), sha256=sha, dims=dims, seed=seed, audio_seed=audio_seed,
                       state_dtype="float16", keys=sorted(state), cases=out), f, indent=0)


def asset_export():
    """Product asset (data only): language codes in token order and, per
    vocabulary, the special ids / SuppressTokens(-1) list / whitespace-only ids
    that tokenizer.py:132-327 computes with tiktoken.  Written to
    whisper.coreml_amd/whisper/assets/specials.json."""
    langs = list(ref_tok.LANGUAGES.items())
    res = {"languages": [[c, n] for c, n in langs], "to_language_code": dict(ref_tok.TO_LANGUAGE_CODE),
           "vocab": {}}
    for multilingual in (True, False):
        for nl in range(99, 101):
            tok = ref_tok.get_tokenizer(multilingual, num_languages=nl)
            key = f"{'multilingual' if multilingual else 'gpt2'}_{nl}"
            res["vocab"][key] = dict(
                n_base=len(tok.encoding._ranks), n_vocab=tok.encoding.n_vocab,
                non_speech_tokens=list(tok.non_speech_tokens), blank=tok.encode(" "),
                whitespace_tokens=sorted(i for b, i in tok.encoding._ranks.items() if _is_ws(b)))
    out = os.path.join(REPO, "whisper.coreml_amd", "whisper", "assets")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "specials.json"), "w") as f:
        json.dump(res, f)
    print("assets exported")


def main(argv):
    os.makedirs(OUT, exist_ok=True)
    what = argv or ["tokens", "mel", "dtw", "micro", "tiny.en", "turbo", "large-v3"]
    for w in what:
        if w == "tokens":
            token_goldens()
        elif w == "mel":
            mel_goldens()
        elif w == "dtw":
            dtw_goldens()
        elif w == "assets":
            asset_export()
        elif w == "prefix":
            prefix_goldens()
        elif w == "beam_options":
            beam_option_goldens()
        elif w.endswith("_ckpt"):
            checkpoint_goldens(w[:-len("_ckpt")])
        elif w.endswith("_steps_mixed"):
            step_goldens_mixed(w[:-len("_steps_mixed")])
        elif w.endswith("_words_beam"):
            words_beam_goldens(w[:-len("_words_beam")])
        elif w.endswith("_words"):
            base = w[:-len("_words")]
            model, _ = build_ref_model(base)
            # full-size models: find_alignment with the real alignment heads plus one
            # clip-grid transcribe run (the sequential and beam runs cost minutes each on CPU)
            big = base in ("turbo", "large-v3")
            words_goldens(model, base, run_keys=("clip_greedy_words",) if big else None)
        elif w.endswith("_steps"):
            step_goldens(w[:-len("_steps")])
        else:
            small = w.startswith("micro")
            big = w in ("turbo", "large-v3", "large-v3-turbo")
            model, out = model_goldens(w, full=small, beam_natural=not big)
            np.savez_compressed(os.path.join(OUT, f"{w}.npz"), **out)
            if small:
                transcribe_goldens(model, w, out)
            del model


if __name__ == "__main__":
    main(sys.argv[1:])
