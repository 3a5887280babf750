"""Window decoding on the device (reference whisper/decoding.py:81-853).

The reference runs its per-token loop in Python: decoder call, logit filters,
beam/greedy update, KV reorder (decoding.py:707-737).  Here ``DecodingTask``
only prepares the options and the initial tokens of each window; the whole loop
— prefill, then one hipGraph per token containing the decoder step, the filters
(SuppressBlank/SuppressTokens/ApplyTimestampRules), log-softmax, top-k, the beam
merge with finished-sequence bookkeeping and the KV reorder by index
indirection — runs in libwhisper_hip.  Several windows are decoded together
(their rows are batched in every GEMM), which is how ``transcribe`` shards the
30 s windows of a file.  The host does what the reference does once per window
after the loop: finalize, rank, build ``DecodingResult`` (decoding.py:766-816).
"""

import itertools
import zlib
from dataclasses import dataclass, field, replace
from typing import TYPE_CHECKING, Dict, Iterable, List, Optional, Sequence, Tuple, Union

import numpy as np

from .audio import CHUNK_LENGTH, N_FRAMES
from .backend_hip import WhDecodeOpts
from .tokenizer import Tokenizer, get_tokenizer

if TYPE_CHECKING:
    from .model import Whisper

_seed_counter = itertools.count(1)


def compression_ratio(text: str) -> float:
    """utils.py:45-47."""
    b = text.encode("utf-8")
    return len(b) / len(zlib.compress(b)) if b else 0.0


@dataclass(frozen=True)
class DecodingOptions:
    task: str = "transcribe"
    language: Optional[str] = None
    temperature: float = 0.0
    sample_len: Optional[int] = None
    best_of: Optional[int] = None
    beam_size: Optional[int] = None
    patience: Optional[float] = None
    length_penalty: Optional[float] = None
    prompt: Optional[Union[str, List[int]]] = None
    prefix: Optional[Union[str, List[int]]] = None
    suppress_tokens: Optional[Union[str, Iterable[int]]] = "-1"
    suppress_blank: bool = True
    without_timestamps: bool = False
    max_initial_timestamp: Optional[float] = 1.0
    fp16: bool = True


@dataclass(frozen=True)
class DecodingResult:
    audio_features: Optional[np.ndarray]
    language: str
    language_probs: Optional[Dict[str, float]] = None
    tokens: List[int] = field(default_factory=list)
    text: str = ""
    avg_logprob: float = np.nan
    no_speech_prob: float = np.nan
    temperature: float = np.nan
    compression_ratio: float = np.nan


class DecodingTask:
    """Options resolution of decoding.py:535-669; the loop itself is on the device."""

    def __init__(self, model: "Whisper", options: DecodingOptions):
        self.model = model
        language = options.language or "en"
        self.tokenizer: Tokenizer = get_tokenizer(model.is_multilingual, num_languages=model.num_languages,
                                                  language=language, task=options.task)
        self.options = self._verify_options(options)
        self.n_group = options.beam_size or options.best_of or 1
        self.n_ctx = model.dims.n_text_ctx
        self.sample_len = options.sample_len or model.dims.n_text_ctx // 2
        self.sot_sequence = self.tokenizer.sot_sequence
        if options.without_timestamps:
            self.sot_sequence = self.tokenizer.sot_sequence_including_notimestamps
        self.initial_tokens = self._initial_tokens(options.prompt)
        self.sample_begin = len(self.initial_tokens)
        self.sot_index = self.initial_tokens.index(self.tokenizer.sot)

    @staticmethod
    def _verify_options(o: DecodingOptions) -> DecodingOptions:
        if o.beam_size is not None and o.best_of is not None:
            raise ValueError("beam_size and best_of can't be given together")
        if o.temperature == 0 and o.best_of is not None:
            raise ValueError("best_of with greedy sampling (T=0) is not compatible")
        if o.patience is not None and o.beam_size is None:
            raise ValueError("patience requires beam_size to be given")
        if o.length_penalty is not None and not (0 <= o.length_penalty <= 1):
            raise ValueError("length_penalty (alpha) should be a value between 0 and 1")
        return o

    def _text_ids(self, v) -> List[int]:
        """decoding.py:617-619, 628-630: text is encoded as " " + text.strip()."""
        if isinstance(v, str):
            return self.tokenizer.encode(" " + v.strip())
        return list(v)

    def _initial_tokens(self, prompt) -> Tuple[int, ...]:
        """decoding.py:614-640, Python slice semantics included: with the default
        sample_len max_prefix_len is 0 and [-0:] keeps the whole prefix; a negative
        max_prefix_len (sample_len > n_ctx // 2) drops the FIRST -max_prefix_len tokens."""
        toks = list(self.sot_sequence)
        if self.options.prefix:
            pre = self._text_ids(self.options.prefix)
            if self.sample_len is not None:
                max_prefix_len = self.n_ctx // 2 - self.sample_len
                pre = pre[-max_prefix_len:]
            toks = toks + pre
        if prompt:
            p = self._text_ids(prompt)
            toks = [self.tokenizer.sot_prev] + p[-(self.n_ctx // 2 - 1):] + toks
        return tuple(toks)

    def suppress_list(self) -> List[int]:
        """decoding.py:642-669."""
        s = self.options.suppress_tokens
        if isinstance(s, str):
            s = [int(t) for t in s.split(",")] if s else []
        s = list(s or [])
        if -1 in s:
            s = [t for t in s if t >= 0] + list(self.tokenizer.non_speech_tokens)
        t = self.tokenizer
        s += [t.transcribe, t.translate, t.sot, t.sot_prev, t.sot_lm, t.no_speech]
        return sorted(set(s))

    def wh_opts(self) -> WhDecodeOpts:
        o, t = self.options, self.tokenizer
        w = WhDecodeOpts()
        w.group = self.n_group
        w.beam = 1 if o.beam_size is not None else 0
        w.patience = float(o.patience or 1.0)
        # max_candidates = round(beam_size * patience) with Python's rounding (decoding.py:339)
        w.max_candidates = round(self.n_group * (o.patience or 1.0)) if o.beam_size is not None else 0
        w.temperature = float(o.temperature) if o.beam_size is None else 0.0
        w.sample_len = self.sample_len
        w.suppress_blank = int(o.suppress_blank)
        w.timestamps = int(not o.without_timestamps)
        max_init = -1
        if not o.without_timestamps and o.max_initial_timestamp:
            precision = CHUNK_LENGTH / self.model.dims.n_audio_ctx
            max_init = round(o.max_initial_timestamp / precision)
        w.max_initial = max_init
        w.eot, w.no_speech, w.no_timestamps, w.timestamp_begin = t.eot, t.no_speech, t.no_timestamps, t.timestamp_begin
        blank = t.encode_blank()[:3]
        for i, b in enumerate(blank):
            w.blank[i] = b
        w.n_blank = len(blank)
        sup = self.suppress_list() if o.suppress_tokens else []
        self._sup = (np.asarray(sup, dtype=np.int32) if sup else np.zeros(1, dtype=np.int32))
        import ctypes
        w.suppress = self._sup.ctypes.data_as(ctypes.POINTER(ctypes.c_int))
        w.n_suppress = len(sup)
        # the seed is part of the captured step graph: keep it constant for T = 0
        w.seed = (next(_seed_counter) * 0x9E3779B97F4A7C15 % (1 << 64)) if w.temperature > 0 else 0
        return w

    def finalize(self, raw: dict) -> Tuple[List[int], float, float]:
        """BeamSearchDecoder/GreedyDecoder.finalize + MaximumLikelihoodRanker
        (decoding.py:217-240, 322-325, 411-431, 775-789) for one window."""
        eot, sb, G = self.tokenizer.eot, self.sample_begin, self.n_group
        L = raw["length"]
        if self.options.beam_size is not None:
            cands = [list(raw["fin_tokens"][i, :raw["fin_len"][i]]) for i in range(len(raw["fin_len"]))]
            scores = [float(x) for x in raw["fin_score"]]
            if len(cands) < G:
                slp = raw["sum_logprobs"]
                for j in list(np.argsort(slp))[::-1]:
                    cands.append(list(raw["tokens"][j, :L]) + [eot])
                    scores.append(float(slp[j]))
                    if len(cands) >= G:
                        break
        else:
            cands = [list(raw["tokens"][j, :L]) + [eot] for j in range(G)]
            scores = [float(x) for x in raw["sum_logprobs"]]
        trimmed = [c[sb:c.index(eot, sb)] for c in cands]
        lp = self.options.length_penalty
        ranked = [s / (len(t) if lp is None else ((5 + len(t)) / 6) ** lp) for s, t in zip(scores, trimmed)]
        best = int(np.argmax(ranked))
        toks = [int(x) for x in trimmed[best]]
        return toks, scores[best], scores[best] / (len(toks) + 1)


def run_windows(model: "Whisper", options: DecodingOptions, prompts: Sequence[Optional[List[int]]],
                audio_features: bool = False, slots: Optional[Sequence[int]] = None) -> List[DecodingResult]:
    """Decode windows already encoded into the model's context: window i uses encoder
    slot ``slots[i]`` (default i), all with ``options`` except the per-window prompt."""
    tasks = [DecodingTask(model, replace(options, prompt=p)) for p in prompts]
    t0 = tasks[0]
    opts = t0.wh_opts()
    ctx = model.ctx
    ctx.decode_begin(opts, [t.initial_tokens for t in tasks], [t.sot_index for t in tasks], slots=slots)
    # every window stops on the device (completion, n_ctx or sample_len updates);
    # decode_steps returns once all of them are done
    ctx.decode_steps(t0.sample_len)
    out = []
    lang = t0.tokenizer.language or "en"
    for i, t in enumerate(tasks):
        raw = ctx.decode_read(i, t.n_group)
        toks, _, avg = t.finalize(raw)
        text = t.tokenizer.decode(toks).strip()
        out.append(DecodingResult(
            audio_features=ctx.audio_features(slots[i] if slots is not None else i) if audio_features else None,
            language=lang, tokens=toks,
            text=text, avg_logprob=avg, no_speech_prob=raw["no_speech_prob"], temperature=options.temperature,
            compression_ratio=compression_ratio(text)))
    return out


def decode(model: "Whisper", mel, options: DecodingOptions = DecodingOptions(), **kwargs
           ) -> Union[DecodingResult, List[DecodingResult]]:
    """decoding.py:820-853: mel (n_mels, 3000) or (n, n_mels, 3000)."""
    mel = np.asarray(mel.detach().cpu().numpy() if hasattr(mel, "detach") else mel, dtype=np.float32)
    single = mel.ndim == 2
    if single:
        mel = mel[None]
    if kwargs:
        options = replace(options, **kwargs)
    if not options.fp16 and model.dtype != "fp32":
        # decoding.py:745-752 would compute in fp32; the context's precision is fixed at load
        raise ValueError("DecodingOptions(fp16=False) needs a context loaded with dtype='fp32'")
    n = mel.shape[0]
    if n > model.ctx.max_windows:
        res = []
        for i in range(0, n, model.ctx.max_windows):
            res += decode(model, mel[i:i + model.ctx.max_windows], options)
        return res
    if options.language is None and model.is_multilingual:
        options = replace(options, language="en")
    flat = np.concatenate(list(mel), axis=1)
    model.ctx.mel_write(flat)
    model.ctx.encode([i * N_FRAMES for i in range(n)], [N_FRAMES] * n)
    res = run_windows(model, options, [options.prompt] * n, audio_features=True)
    return res[0] if single else res


def detect_language(model: "Whisper", mel, tokenizer: Optional[Tokenizer] = None):
    """Language id as upstream whisper does it (the fork's version is broken,
    decoding.py:58 calls the removed Whisper.logits): one decoder pass over
    <|startoftranscript|>, argmax over the language tokens."""
    mel = np.asarray(mel.detach().cpu().numpy() if hasattr(mel, "detach") else mel, dtype=np.float32)
    single = mel.ndim == 2
    if single:
        mel = mel[None]
    if tokenizer is None:
        tokenizer = get_tokenizer(model.is_multilingual, num_languages=model.num_languages)
    if tokenizer.language is None or tokenizer.language_token not in tokenizer.sot_sequence:
        raise ValueError("This model doesn't have language tokens so it can't perform lang id")
    lang_tokens = np.asarray(tokenizer.all_language_tokens)
    codes = tokenizer.all_language_codes
    out_tokens, out_probs = [], []
    for m in mel:
        model.ctx.mel_write(m)
        model.ctx.encode([0], [N_FRAMES])
        logits, _ = model.ctx.prefill_logits(0, [tokenizer.sot])
        row = logits[0].astype(np.float64)
        sel = row[lang_tokens]
        p = np.exp(sel - sel.max())
        p /= p.sum()
        out_tokens.append(int(lang_tokens[int(np.argmax(sel))]))
        out_probs.append({c: float(pp) for c, pp in zip(codes, p)})
    if single:
        return out_tokens[0], out_probs[0]
    return out_tokens, out_probs
