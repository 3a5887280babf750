"""Word-level timestamps (reference whisper/timing.py).

The numeric half of ``find_alignment`` — the first decoder pass with the alignment
heads' cross-QK, the text-token probabilities, softmax / z-norm / median filter /
head mean and the DTW with its backtrace — runs in libwhisper_hip (``wh_align``,
csrc/wh_align.hip).  What stays here is the reference's host logic on the returned
path: word splitting, jump times, punctuation merging and the segment-level
refinements of ``add_word_timestamps`` (timing.py:234-376), pinned to the reference's
own outputs by tests/golden/micro_words.json.
"""

import itertools
from dataclasses import dataclass
from typing import TYPE_CHECKING, List

import numpy as np

from .audio import HOP_LENGTH, SAMPLE_RATE, TOKENS_PER_SECOND
from .tokenizer import Tokenizer

if TYPE_CHECKING:
    from .model import Whisper


@dataclass
class WordTiming:
    word: str
    tokens: List[int]
    start: float
    end: float
    probability: float


def _alignment_head_ids(model: "Whisper") -> List[int]:
    """Flat (layer * n_head + head) ids of the alignment heads in the order the
    reference stacks their cross-QK (decoder.py:306-313: layer-major)."""
    heads = np.asarray(model.alignment_heads, dtype=bool)
    return [int(i) for i in np.flatnonzero(heads.reshape(-1))]


def dtw(model: "Whisper", x: np.ndarray) -> np.ndarray:
    """timing.py:139-151: DTW path [2][L] of cost matrix x, computed on the GPU."""
    return model.ctx.dtw(np.asarray(x, dtype=np.float32))


def find_alignment(model: "Whisper", tokenizer: Tokenizer, text_tokens: List[int], num_frames: int, *,
                   medfilt_width: int = 7, qk_scale: float = 1.0, slot: int = 0) -> List[WordTiming]:
    """timing.py:163-231.  `slot` names the context slot holding the window's audio
    features (the reference uses the model's cached cross-KV of the last window)."""
    return find_alignment_batch(model, tokenizer, [text_tokens], [num_frames], [slot], medfilt_width=medfilt_width,
                                qk_scale=qk_scale)[0]


def find_alignment_batch(model: "Whisper", tokenizer: Tokenizer, text_tokens: List[List[int]],
                         num_frames: List[int], slots: List[int], *, medfilt_width: int = 7,
                         qk_scale: float = 1.0) -> List[List[WordTiming]]:
    """find_alignment of several windows (slots) with one wh_align_batch call: their
    first passes batched on the GPU, one DTW workgroup per window."""
    if qk_scale != 1.0:
        raise NotImplementedError("qk_scale != 1.0 (the reference always passes 1.0)")
    out: List[List[WordTiming]] = [[] for _ in text_tokens]
    todo = [i for i, t in enumerate(text_tokens) if len(t) > 0]
    if not todo:
        return out
    seqs = [[*tokenizer.sot_sequence, tokenizer.no_timestamps, *text_tokens[i], tokenizer.eot] for i in todo]
    res = model.ctx.align_batch([slots[i] for i in todo], seqs, len(tokenizer.sot_sequence),
                                [num_frames[i] for i in todo], _alignment_head_ids(model), medfilt_width)
    for i, (probs, text_indices, time_indices) in zip(todo, res):
        out[i] = _words_from_path(tokenizer, text_tokens[i], probs, text_indices, time_indices)
    return out


def _words_from_path(tokenizer: Tokenizer, text_tokens: List[int], probs: np.ndarray, text_indices: np.ndarray,
                     time_indices: np.ndarray) -> List[WordTiming]:
    """timing.py:208-231 on the device results."""
    text_token_probs = probs.astype(np.float64)
    words, word_tokens = tokenizer.split_to_word_tokens(text_tokens + [tokenizer.eot])
    if len(word_tokens) <= 1:
        return []
    word_boundaries = np.pad(np.cumsum([len(t) for t in word_tokens[:-1]]), (1, 0))

    jumps = np.pad(np.diff(text_indices), (1, 0), constant_values=1).astype(bool)
    jump_times = time_indices[jumps] / TOKENS_PER_SECOND
    start_times = jump_times[word_boundaries[:-1]].tolist()
    end_times = jump_times[word_boundaries[1:]].tolist()
    # per-word mean probability (np.mean over each word's tokens, timing.py:221-224),
    # as segment sums in one pass: equal to the per-word np.mean up to summation order
    lo, hi = word_boundaries[:-1], word_boundaries[1:]
    csum = np.concatenate(([0.0], np.cumsum(text_token_probs)))
    n = hi - lo
    word_probabilities = np.where(n > 0, (csum[hi] - csum[lo]) / np.maximum(n, 1), np.nan).tolist()

    return [WordTiming(word, tokens, start, end, probability)
            for word, tokens, start, end, probability in zip(words, word_tokens, start_times, end_times,
                                                              word_probabilities)]


def merge_punctuations(alignment: List[WordTiming], prepended: str, appended: str):
    """timing.py:234-265, in place: opening punctuation (a word " X" with X in
    `prepended`) moves onto the next word that is not itself such punctuation (the last
    word always takes what is pending); closing punctuation (a word in `appended`)
    moves onto the nearest kept word before it unless that word ends in a space.
    Moved words stay in the list with empty text and tokens."""
    pending: List[WordTiming] = []
    last = len(alignment) - 1
    for k, w in enumerate(alignment):
        if k < last and w.word.startswith(" ") and w.word.strip() in prepended:
            pending.append(w)
            continue
        if pending:
            w.word = "".join(p.word for p in pending) + w.word
            w.tokens = [t for p in pending for t in p.tokens] + w.tokens
            for p in pending:
                p.word, p.tokens = "", []
            pending = []
    if not alignment:
        return
    host = alignment[0]
    for w in alignment[1:]:
        if not host.word.endswith(" ") and w.word in appended:
            host.word += w.word
            host.tokens = host.tokens + w.tokens
            w.word, w.tokens = "", []
        else:
            host = w


def add_word_timestamps(*, segments: List[dict], model: "Whisper", tokenizer: Tokenizer, num_frames: int,
                        prepend_punctuations: str = "\"'“¿([{-",
                        append_punctuations: str = "\"'.。,，!！?？:：”)]}、", last_speech_timestamp: float,
                        **kwargs):
    """timing.py:268-376 (kwargs go to find_alignment, e.g. slot=)."""
    if len(segments) == 0:
        return
    text_tokens = list(itertools.chain.from_iterable(_text_tokens_per_segment(segments, tokenizer)))
    alignment = find_alignment(model, tokenizer, text_tokens, num_frames, **kwargs)
    apply_alignment(segments, alignment, tokenizer, prepend_punctuations, append_punctuations,
                    last_speech_timestamp)


def _text_tokens_per_segment(segments: List[dict], tokenizer: Tokenizer) -> List[List[int]]:
    return [[token for token in segment["tokens"] if token < tokenizer.eot] for segment in segments]


def _duration_limits(alignment: List[WordTiming]):
    """(median, max) word duration of timing.py:292-296: the median over non-zero
    durations, capped at 0.7 s; the max is twice that."""
    d = np.array([w.end - w.start for w in alignment])
    d = d[d.nonzero()]
    med = min(0.7, float(np.median(d) if len(d) > 0 else 0.0))
    return med, 2 * med, len(d) > 0


def _clip_at_sentence_marks(alignment: List[WordTiming], max_duration: float):
    """timing.py:301-312: a too-long word that is a sentence end mark keeps its start;
    a too-long word right after one keeps its end."""
    marks = ".。!！?？"
    for prev, w in zip(alignment, alignment[1:]):
        if w.end - w.start <= max_duration:
            continue
        if w.word in marks:
            w.end = w.start + max_duration
        elif prev.word in marks:
            w.start = w.end - max_duration


def _fit_segment_words(segment: dict, words: List[dict], last_speech: float, med: float, max_d: float) -> float:
    """timing.py:343-374 for one segment: shorten an overlong first word after a pause,
    then reconcile the segment's bounds with its first / last word.  Returns the new
    last-speech time."""
    first, last = words[0], words[-1]
    second = words[1] if len(words) > 1 else None
    too_long = first["end"] - first["start"] > max_d or (
        second is not None and second["end"] - first["start"] > 2 * max_d)
    if first["end"] - last_speech > 4 * med and too_long:
        if second is not None and second["end"] - second["start"] > max_d:
            cut = max(second["end"] / 2, second["end"] - max_d)
            first["end"] = second["start"] = cut
        first["start"] = max(0, first["end"] - max_d)
    if segment["start"] < first["end"] and segment["start"] - 0.5 > first["start"]:
        first["start"] = max(0, min(first["end"] - med, segment["start"]))
    else:
        segment["start"] = first["start"]
    if segment["end"] > last["start"] and segment["end"] + 0.5 < last["end"]:
        last["end"] = max(last["start"] + med, segment["end"])
    else:
        segment["end"] = last["end"]
    return segment["end"]


def apply_alignment(segments: List[dict], alignment: List[WordTiming], tokenizer: Tokenizer,
                    prepend_punctuations: str, append_punctuations: str, last_speech_timestamp: float):
    """The host half of add_word_timestamps (timing.py:292-376) on an alignment from
    find_alignment (mutated: pass a copy to keep it).  Words are dealt to segments in
    order until each segment's text-token count is covered; emptied (merged)
    punctuation entries consume their tokens without producing a word."""
    if len(segments) == 0:
        return
    med, max_d, any_duration = _duration_limits(alignment)
    if any_duration:
        _clip_at_sentence_marks(alignment, max_d)
    merge_punctuations(alignment, prepend_punctuations, append_punctuations)
    t0 = segments[0]["seek"] * HOP_LENGTH / SAMPLE_RATE
    source = iter(alignment)
    for segment, need in zip(segments, (len(t) for t in _text_tokens_per_segment(segments, tokenizer))):
        words, covered = [], 0
        while covered < need:
            timing = next(source, None)
            if timing is None:
                break
            covered += len(timing.tokens)
            if timing.word:
                words.append(dict(word=timing.word, start=round(t0 + timing.start, 2), end=round(t0 + timing.end, 2),
                                  probability=timing.probability))
        if words:
            last_speech_timestamp = _fit_segment_words(segment, words, last_speech_timestamp, med, max_d)
        segment["words"] = words
