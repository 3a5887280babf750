"""CPU fp32 restatement of the reference fork's hot path — TEST INFRASTRUCTURE ONLY.

This module is the *oracle*: a plain PyTorch-CPU / numpy restatement of the
algorithm of wangchou/whisper.coreml's CPU path (``--use_coreml=False``),
written from reading the reference, not copied from it.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use
it, and only as the checker / the timed CPU baseline.  The product path
(``whisper.coreml_amd/whisper``) never imports it.

Pinning: every stage is checked against golden vectors produced by the
reference itself in the build container (oracle/gen_golden.py ->
tests/golden/*.npz, *.json) by tests/test_oracle.py.

Citations are ``path:line`` in /root/reference.

Fork numerics restated:
  * encoder LayerNorm eps 1e-7 (whisper/encoder.py:66,72,95); decoder eps 1e-5
    (whisper/decoder.py:99,104,110,147)
  * encoder scales K by d^-1/2 after projection (encoder.py:38); the decoder
    folds 0.125 into every *query* weight and bias at load (decoder.py:16-20,42)
  * key projections have no bias (encoder.py:32, decoder.py:39)
  * exact-erf GELU (nn.GELU())
"""

import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

SAMPLE_RATE = 16000
N_FFT = 400
HOP_LENGTH = 160
N_SAMPLES = 480000
N_FRAMES = 3000

_GOLDEN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


# ----------------------------------------------------------------------------- mel
def golden_mel_filters(n_mels: int) -> np.ndarray:
    """The reference's own filterbank values (whisper/assets/mel_filters.npz via
    audio.py:91-107), as captured into tests/golden/mel.npz."""
    with np.load(os.path.join(_GOLDEN, "mel.npz")) as g:
        return g[f"filters_{n_mels}"].astype(np.float32)


def log_mel_spectrogram(audio: np.ndarray, n_mels: int, padding: int = 0) -> torch.Tensor:
    """audio.py:110-157: right-pad, centred reflect-padded STFT (hann 400 / hop 160),
    drop last frame, |X|^2, mel projection, log10(clamp 1e-10), floor at max-8,
    (x+4)/4.  Returns float32 (n_mels, frames)."""
    x = torch.from_numpy(np.ascontiguousarray(audio, dtype=np.float32))
    if padding > 0:
        x = F.pad(x, (0, padding))
    window = torch.hann_window(N_FFT)
    stft = torch.stft(x, N_FFT, HOP_LENGTH, window=window, return_complex=True)
    mag = stft[..., :-1].abs() ** 2
    filters = torch.from_numpy(golden_mel_filters(n_mels))
    mel = filters @ mag
    log_spec = torch.clamp(mel, min=1e-10).log10()
    log_spec = torch.maximum(log_spec, log_spec.max() - 8.0)
    return (log_spec + 4.0) / 4.0


def pad_or_trim(mel: torch.Tensor, length: int = N_FRAMES) -> torch.Tensor:
    """audio.py:65-88 for the last axis."""
    if mel.shape[-1] > length:
        mel = mel[..., :length]
    if mel.shape[-1] < length:
        mel = F.pad(mel, (0, length - mel.shape[-1]))
    return mel


# ----------------------------------------------------------------------------- model
def _ln(x, w, b, eps):
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


class OracleWhisper:
    """The fork's model math over a checkpoint-format state dict (float32)."""

    def __init__(self, dims: Dict[str, int], state_dict: Dict[str, np.ndarray],
                 alignment_heads: Optional[np.ndarray] = None):
        self.dims = dims
        sd = {}
        for k, v in state_dict.items():
            t = torch.from_numpy(np.asarray(v, dtype=np.float32))
            # decoder.py:16-20,42: pre-hook multiplies decoder query weight+bias by 0.125
            if k.startswith("decoder.") and "query" in k:
                t = t * 0.125
            sd[k] = t
        self.sd = sd
        self.n_vocab = dims["n_vocab"]
        L, H = dims["n_text_layer"], dims["n_text_head"]
        if alignment_heads is None:
            # model.py:51-56 default: last half of the decoder layers
            alignment_heads = np.zeros((L, H), dtype=bool)
            alignment_heads[L // 2:] = True
        self.alignment_heads = np.asarray(alignment_heads, dtype=bool).reshape(L, H)
        self.cross_k = None
        self.cross_v = None

    @property
    def is_multilingual(self):
        return self.dims["n_vocab"] >= 51865

    @property
    def num_languages(self):
        return self.dims["n_vocab"] - 51765 - int(self.is_multilingual)

    # -- encoder: encoder.py:103-136
    def encode(self, mel: torch.Tensor) -> torch.Tensor:
        s = self.sd
        x = mel.unsqueeze(0) if mel.dim() == 2 else mel
        x = F.gelu(F.conv1d(x, s["encoder.conv1.weight"], s["encoder.conv1.bias"], padding=1))
        x = F.gelu(F.conv1d(x, s["encoder.conv2.weight"], s["encoder.conv2.bias"], stride=2, padding=1))
        x = x.permute(0, 2, 1) + s["encoder.positional_embedding"]
        H = self.dims["n_audio_head"]
        for i in range(self.dims["n_audio_layer"]):
            p = f"encoder.blocks.{i}."
            h = _ln(x, s[p + "attn_ln.weight"], s[p + "attn_ln.bias"], 1e-7)
            q = F.linear(h, s[p + "attn.query.weight"], s[p + "attn.query.bias"])
            k = F.linear(h, s[p + "attn.key.weight"]) * (64 ** -0.5)
            v = F.linear(h, s[p + "attn.value.weight"], s[p + "attn.value.bias"])
            o = self._mha(q, k, v, H, None)
            x = x + F.linear(o, s[p + "attn.out.weight"], s[p + "attn.out.bias"])
            h = _ln(x, s[p + "mlp_ln.weight"], s[p + "mlp_ln.bias"], 1e-7)
            h = F.gelu(F.linear(h, s[p + "mlp.0.weight"], s[p + "mlp.0.bias"]))
            x = x + F.linear(h, s[p + "mlp.2.weight"], s[p + "mlp.2.bias"])
        x = _ln(x, s["encoder.ln_post.weight"], s["encoder.ln_post.bias"], 1e-7)
        return x[0] if mel.dim() == 2 else x

    @staticmethod
    def _mha(q, k, v, H, mask, return_qk=False):
        B, Tq, n = q.shape
        Tk = k.shape[1]
        d = n // H
        qh = q.view(B, Tq, H, d).permute(0, 2, 1, 3)
        kh = k.view(B, Tk, H, d).permute(0, 2, 3, 1)
        vh = v.view(B, Tk, H, d).permute(0, 2, 1, 3)
        qk = qh @ kh
        if mask is not None:
            qk = qk + mask
        w = qk.softmax(dim=-1)
        o = (w @ vh).permute(0, 2, 1, 3).reshape(B, Tq, n)
        return (o, qk) if return_qk else o

    # -- decoder.py:172-187: per-layer cross K (no bias) and V from xa
    def set_audio(self, xa: torch.Tensor):
        s = self.sd
        xa = xa.unsqueeze(0) if xa.dim() == 2 else xa
        self.cross_k, self.cross_v = [], []
        for i in range(self.dims["n_text_layer"]):
            p = f"decoder.blocks.{i}.cross_attn."
            self.cross_k.append(F.linear(xa, s[p + "key.weight"]))
            self.cross_v.append(F.linear(xa, s[p + "value.weight"], s[p + "value.bias"]))

    def decoder_forward(self, tokens: torch.Tensor, offset: int, cache: Optional[List]) -> Tuple:
        """One decoder pass over ``tokens`` [B, n] at positions offset..offset+n-1
        (decoder.py:189-329 without the static padding, which is a numerical no-op).
        ``cache``: per layer [k, v] of shape [B, offset, n] or None.
        Returns logits [B, n, V], new cache, cross-QK of alignment heads (batch 0)."""
        s = self.sd
        H = self.dims["n_text_head"]
        B, n_ctx = tokens.shape
        x = s["decoder.token_embedding.weight"][tokens] + s["decoder.positional_embedding"][offset:offset + n_ctx]
        tot = offset + n_ctx
        mask = torch.full((n_ctx, tot), float("-inf")).triu_(offset + 1)
        new_cache, align = [], []
        for i in range(self.dims["n_text_layer"]):
            p = f"decoder.blocks.{i}."
            h = _ln(x, s[p + "attn_ln.weight"], s[p + "attn_ln.bias"], 1e-5)
            q = F.linear(h, s[p + "attn.query.weight"], s[p + "attn.query.bias"])
            k = F.linear(h, s[p + "attn.key.weight"])
            v = F.linear(h, s[p + "attn.value.weight"], s[p + "attn.value.bias"])
            if cache is not None:
                k = torch.cat([cache[i][0], k], dim=1)
                v = torch.cat([cache[i][1], v], dim=1)
            new_cache.append([k, v])
            x = x + F.linear(self._mha(q, k, v, H, mask), s[p + "attn.out.weight"], s[p + "attn.out.bias"])
            h = _ln(x, s[p + "cross_attn_ln.weight"], s[p + "cross_attn_ln.bias"], 1e-5)
            q = F.linear(h, s[p + "cross_attn.query.weight"], s[p + "cross_attn.query.bias"])
            ck = self.cross_k[i].expand(B, -1, -1)
            cv = self.cross_v[i].expand(B, -1, -1)
            o, qk = self._mha(q, ck, cv, H, None, return_qk=True)
            for hh in range(H):
                if self.alignment_heads[i, hh]:
                    align.append(qk[0, hh])
            x = x + F.linear(o, s[p + "cross_attn.out.weight"], s[p + "cross_attn.out.bias"])
            h = _ln(x, s[p + "mlp_ln.weight"], s[p + "mlp_ln.bias"], 1e-5)
            h = F.gelu(F.linear(h, s[p + "mlp.0.weight"], s[p + "mlp.0.bias"]))
            x = x + F.linear(h, s[p + "mlp.2.weight"], s[p + "mlp.2.bias"])
        x = _ln(x, s["decoder.ln.weight"], s["decoder.ln.bias"], 1e-5)
        logits = x @ s["decoder.token_embedding.weight"].t()
        return logits, new_cache, (torch.stack(align) if align else None)


# ----------------------------------------------------------------------------- tokens
@dataclass
class SpecialTokens:
    """Special ids of tokenizer.py:132-253 for a vocabulary (base vocab size + languages)."""
    eot: int
    sot: int
    translate: int
    transcribe: int
    sot_lm: int
    sot_prev: int
    no_speech: int
    no_timestamps: int
    timestamp_begin: int
    sot_sequence: Tuple[int, ...]
    non_speech_tokens: Tuple[int, ...]
    blank: Tuple[int, ...]
    whitespace: Tuple[int, ...] = ()

    @staticmethod
    def for_model(dims, language="en", task="transcribe"):
        import json
        with open(os.path.join(_GOLDEN, "tokens.json")) as f:
            g = json.load(f)
        multilingual = dims["n_vocab"] >= 51865
        nl = dims["n_vocab"] - 51765 - int(multilingual)
        key = f"{'multilingual' if multilingual else 'gpt2'}_{nl}"
        t = g[key]
        return SpecialTokens(t["eot"], t["sot"], t["translate"], t["transcribe"], t["sot_lm"], t["sot_prev"],
                             t["no_speech"], t["no_timestamps"], t["timestamp_begin"], tuple(t["sot_sequence"]),
                             tuple(t["non_speech_tokens"]), tuple(t["blank"]),
                             tuple(t["whitespace_tokens"]))


# ----------------------------------------------------------------------------- decoding
@dataclass
class Options:
    """Subset of DecodingOptions (decoding.py:81-115) the oracle restates (T=0 only)."""
    beam_size: Optional[int] = None
    patience: Optional[float] = None
    length_penalty: Optional[float] = None
    prompt: Optional[List[int]] = None
    prefix: Optional[List[int]] = None
    suppress_tokens: Optional[str] = "-1"
    suppress_blank: bool = True
    without_timestamps: bool = False
    max_initial_timestamp: Optional[float] = 1.0
    sample_len: Optional[int] = None


@dataclass
class Result:
    tokens: List[int]
    sum_logprob: float
    avg_logprob: float
    no_speech_prob: float
    all_logits_first: Optional[torch.Tensor] = None
    # beam: the candidates the ranker chose from, [untrimmed length, sum_logprob] in the
    # finished set's order (BeamSearchDecoder.finalize, decoding.py:411-431)
    candidates: Optional[List[List[float]]] = None


def _suppress_list(opts: Options, st: SpecialTokens) -> List[int]:
    """decoding.py:642-669."""
    s = opts.suppress_tokens
    toks = [int(t) for t in s.split(",")] if isinstance(s, str) and s else list(s or [])
    if -1 in toks:
        toks = [t for t in toks if t >= 0] + list(st.non_speech_tokens)
    toks += [st.transcribe, st.translate, st.sot, st.sot_prev, st.sot_lm, st.no_speech]
    return sorted(set(toks))


def apply_filters(logits: torch.Tensor, tokens: torch.Tensor, sample_begin: int, st: SpecialTokens,
                  opts: Options, suppress: List[int], max_initial_index: Optional[int]):
    """SuppressBlank / SuppressTokens / ApplyTimestampRules (decoding.py:450-532), in place."""
    if opts.suppress_blank and tokens.shape[1] == sample_begin:
        logits[:, list(st.blank) + [st.eot]] = -np.inf
    if suppress:
        logits[:, suppress] = -np.inf
    if opts.without_timestamps:
        return
    tb = st.timestamp_begin
    logits[:, st.no_timestamps] = -np.inf
    for k in range(tokens.shape[0]):
        seq = tokens[k, sample_begin:].tolist()
        last_ts = len(seq) >= 1 and seq[-1] >= tb
        penult_ts = len(seq) < 2 or seq[-2] >= tb
        if last_ts:
            if penult_ts:
                logits[k, tb:] = -np.inf
            else:
                logits[k, :st.eot] = -np.inf
        ts = [t for t in seq if t >= tb]
        if ts:
            upto = ts[-1] if (last_ts and not penult_ts) else ts[-1] + 1
            logits[k, tb:upto] = -np.inf
    if tokens.shape[1] == sample_begin:
        logits[:, :tb] = -np.inf
        if max_initial_index is not None:
            logits[:, tb + max_initial_index + 1:] = -np.inf
    lp = F.log_softmax(logits.float(), dim=-1)
    for k in range(tokens.shape[0]):
        if lp[k, tb:].logsumexp(dim=-1) > lp[k, :tb].max():
            logits[k, :tb] = -np.inf


def decode(model: OracleWhisper, mel: torch.Tensor, opts: Options, st: Optional[SpecialTokens] = None,
           xa: Optional[torch.Tensor] = None, inference=None) -> Result:
    """DecodingTask.run (decoding.py:740-816) for one window, temperature 0.

    ``inference`` (tests only): an object with the reference's Inference interface
    (``logits(tokens, audio_features)``, ``rearrange_kv_cache(source_indices)``,
    decoding.py:127-204) that replaces the oracle's own decoder calls, so this host
    loop drives another implementation's per-step boundary (libwhisper_hip's
    wh_prefill / wh_step / wh_reorder_kv through whisper.inference.HipInference)."""
    st = st or SpecialTokens.for_model(model.dims)
    n_text_ctx = model.dims["n_text_ctx"]
    sample_len = opts.sample_len or n_text_ctx // 2
    sot_seq = list(st.sot_sequence) + ([st.no_timestamps] if opts.without_timestamps else [])
    init = list(sot_seq)
    if opts.prefix:
        init = init + list(opts.prefix)[-(n_text_ctx // 2 - sample_len):]
    if opts.prompt:
        init = [st.sot_prev] + list(opts.prompt)[-(n_text_ctx // 2 - 1):] + init
    sample_begin = len(init)
    sot_index = init.index(st.sot)
    suppress = _suppress_list(opts, st) if opts.suppress_tokens else []
    max_init = None
    if not opts.without_timestamps and opts.max_initial_timestamp:
        max_init = round(opts.max_initial_timestamp / (30.0 / model.dims["n_audio_ctx"]))
    if inference is None:
        if xa is None:
            xa = model.encode(mel)
        model.set_audio(xa)
    G = opts.beam_size or 1
    tokens = torch.tensor([init] * G)
    sum_lp = torch.zeros(G)
    cache, offset = None, 0
    finished: Dict[Tuple[int, ...], float] = {}
    beam = opts.beam_size is not None
    max_cand = round(G * (opts.patience or 1.0))
    no_speech = float("nan")
    for i in range(sample_len):
        if inference is None:
            inp = tokens if i == 0 else tokens[:, -1:]
            logits, cache, _ = model.decoder_forward(inp, offset, cache)
            offset += inp.shape[1]
        else:
            logits = torch.from_numpy(np.asarray(inference.logits(tokens, None)[0]))
        if i == 0:
            no_speech = logits[:, sot_index].float().softmax(dim=-1)[0, st.no_speech].item()
        logits = logits[:, -1].clone()
        apply_filters(logits, tokens, sample_begin, st, opts, suppress, max_init)
        lp = F.log_softmax(logits.float(), dim=-1)
        if not beam:  # GreedyDecoder.update, decoding.py:304-320 (T=0)
            nxt = logits.argmax(dim=-1)
            cur = lp[torch.arange(G), nxt]
            sum_lp += cur * (tokens[:, -1] != st.eot)
            nxt[tokens[:, -1] == st.eot] = st.eot
            tokens = torch.cat([tokens, nxt[:, None]], dim=-1)
            done = bool((tokens[:, -1] == st.eot).all())
        else:  # BeamSearchDecoder.update, decoding.py:350-409 (one audio)
            scores, sources = {}, {}
            for j in range(G):
                prefix = tokens[j].tolist()
                v, ix = lp[j].topk(G + 1)
                for logprob, tok in zip(v.tolist(), ix.tolist()):
                    seq = tuple(prefix + [tok])
                    scores[seq] = sum_lp[j].item() + logprob
                    sources[seq] = j
            alive, src, new_fin = [], [], {}
            for seq in sorted(scores, key=scores.get, reverse=True):
                if seq[-1] == st.eot:
                    new_fin[seq] = scores[seq]
                else:
                    sum_lp[len(alive)] = scores[seq]
                    alive.append(seq)
                    src.append(sources[seq])
                    if len(alive) == G:
                        break
            tokens = torch.tensor(alive)
            if inference is None:
                cache = [[c[0][src], c[1][src]] for c in cache]
            else:
                inference.rearrange_kv_cache(src)
            for seq in sorted(new_fin, key=new_fin.get, reverse=True):
                if len(finished) >= max_cand:
                    break
                finished[seq] = new_fin[seq]
            done = len(finished) >= max_cand
        if done or tokens.shape[-1] > n_text_ctx:
            break
    # finalize + rank (decoding.py:322-325, 411-431, 217-240, 775-789)
    if beam:
        if len(finished) < G:
            for j in list(np.argsort(sum_lp.numpy()))[::-1]:
                finished[tuple(tokens[j].tolist() + [st.eot])] = sum_lp[j].item()
                if len(finished) >= G:
                    break
        cands = [list(s) for s in finished.keys()]
        cand_lp = list(finished.values())
    else:
        cands = [tokens[j].tolist() + [st.eot] for j in range(G)]
        cand_lp = sum_lp.tolist()
    trimmed = [c[sample_begin:c.index(st.eot, sample_begin)] for c in cands]
    lens = [len(t) for t in trimmed]
    if opts.length_penalty is None:
        sc = [lp_ / n for lp_, n in zip(cand_lp, lens)]
    else:
        sc = [lp_ / ((5 + n) / 6) ** opts.length_penalty for lp_, n in zip(cand_lp, lens)]
    best = int(np.argmax(sc))
    toks = trimmed[best]
    return Result(toks, cand_lp[best], cand_lp[best] / (len(toks) + 1), no_speech,
                  candidates=[[len(c), lp_] for c, lp_ in zip(cands, cand_lp)] if beam else None)


# ----------------------------------------------------------------------------- transcribe
def transcribe(model: OracleWhisper, audio: np.ndarray, *, beam_size: Optional[int] = None,
               condition_on_previous_text: bool = True, clip_timestamps: str = "0",
               no_speech_threshold: Optional[float] = 0.6, logprob_threshold: Optional[float] = -1.0,
               suppress_tokens: str = "-1") -> List[dict]:
    """transcribe.py:41-524, temperature 0, no word timestamps: returns segment dicts."""
    st = SpecialTokens.for_model(model.dims)
    mel = log_mel_spectrogram(audio, model.dims["n_mels"], padding=N_SAMPLES)
    content_frames = mel.shape[-1] - N_FRAMES
    pts = [round(float(t) * 100) for t in clip_timestamps.split(",")] if clip_timestamps else []
    if not pts:
        pts = [0]
    if len(pts) % 2 == 1:
        pts.append(content_frames)
    clips = list(zip(pts[::2], pts[1::2]))
    tb = st.timestamp_begin
    input_stride = N_FRAMES // model.dims["n_audio_ctx"]
    time_precision = input_stride * HOP_LENGTH / SAMPLE_RATE
    all_tokens, segments, prompt_reset = [], [], 0
    clip_idx, seek = 0, clips[0][0]
    while clip_idx < len(clips):
        cs, ce = clips[clip_idx]
        if seek < cs:
            seek = cs
        if seek >= ce:
            clip_idx += 1
            if clip_idx < len(clips):
                seek = clips[clip_idx][0]
            continue
        time_offset = float(seek * HOP_LENGTH / SAMPLE_RATE)
        seg_size = min(N_FRAMES, content_frames - seek, ce - seek)
        seg = pad_or_trim(mel[:, seek:seek + seg_size])
        seg_dur = seg_size * HOP_LENGTH / SAMPLE_RATE
        if seg_dur < 1.0:
            clip_idx += 1
            continue
        prompt = all_tokens[prompt_reset:]
        res = decode(model, seg, Options(beam_size=beam_size, prompt=prompt or None,
                                          suppress_tokens=suppress_tokens), st)
        tokens = torch.tensor(res.tokens, dtype=torch.long)
        if no_speech_threshold is not None:
            skip = res.no_speech_prob > no_speech_threshold
            if logprob_threshold is not None and res.avg_logprob > logprob_threshold:
                skip = False
            if skip:
                seek += seg_size
                continue
        cur = []

        def mk(start, end, toks):
            return dict(seek=seek, start=start, end=end, tokens=toks.tolist(),
                        avg_logprob=res.avg_logprob, no_speech_prob=res.no_speech_prob)

        is_ts = tokens.ge(tb)
        single_end = is_ts[-2:].tolist() == [False, True]
        consec = torch.where(is_ts[:-1] & is_ts[1:])[0] + 1
        if len(consec) > 0:
            slices = consec.tolist()
            if single_end:
                slices.append(len(tokens))
            last = 0
            for cut in slices:
                part = tokens[last:cut]
                cur.append(mk(time_offset + (part[0].item() - tb) * time_precision,
                              time_offset + (part[-1].item() - tb) * time_precision, part))
                last = cut
            if single_end:
                seek += seg_size
            else:
                seek += (tokens[last - 1].item() - tb) * input_stride
        else:
            dur = seg_dur
            tss = tokens[is_ts.nonzero().flatten()]
            if len(tss) > 0 and tss[-1].item() != tb:
                dur = (tss[-1].item() - tb) * time_precision
            cur.append(mk(time_offset, time_offset + dur, tokens))
            seek += seg_size
        ws = set(st.whitespace)
        for s in cur:  # transcribe.py:494-499 (text .strip()=="" <=> only whitespace ids)
            if s["start"] == s["end"] or all(t in ws for t in s["tokens"] if t < st.eot):
                s["tokens"] = []
        segments.extend(cur)
        all_tokens.extend(t for s in cur for t in s["tokens"])
        if not condition_on_previous_text:
            prompt_reset = len(all_tokens)
    return segments
