"""Word-level timestamps (reference whisper/timing.py).

The numeric half of ``find_alignment`` — the first decoder pass with the alignment
heads' cross-QK, the text-token probabilities, softmax / z-norm / median filter /
head mean and the DTW with its backtrace — runs in libwhisper_hip (``wh_align``,
csrc/wh_align.hip).  What stays here is the reference's host logic on the returned
path: word splitting, jump times, punctuation merging and the segment-level
refinements of ``add_word_timestamps`` (timing.py:234-376), restated line by line.
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
    """timing.py:234-265."""
    i = len(alignment) - 2
    j = len(alignment) - 1
    while i >= 0:
        previous = alignment[i]
        following = alignment[j]
        if previous.word.startswith(" ") and previous.word.strip() in prepended:
            following.word = previous.word + following.word
            following.tokens = previous.tokens + following.tokens
            previous.word = ""
            previous.tokens = []
        else:
            j = i
        i -= 1

    i = 0
    j = 1
    while j < len(alignment):
        previous = alignment[i]
        following = alignment[j]
        if not previous.word.endswith(" ") and following.word in appended:
            previous.word = previous.word + following.word
            previous.tokens = previous.tokens + following.tokens
            following.word = ""
            following.tokens = []
        else:
            i = j
        j += 1


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


def apply_alignment(segments: List[dict], alignment: List[WordTiming], tokenizer: Tokenizer,
                    prepend_punctuations: str, append_punctuations: str, last_speech_timestamp: float):
    """The host half of add_word_timestamps (timing.py:292-376) on an alignment from
    find_alignment (mutated: pass a copy to keep it)."""
    if len(segments) == 0:
        return
    text_tokens_per_segment = _text_tokens_per_segment(segments, tokenizer)
    word_durations = np.array([t.end - t.start for t in alignment])
    word_durations = word_durations[word_durations.nonzero()]
    median_duration = np.median(word_durations) if len(word_durations) > 0 else 0.0
    median_duration = min(0.7, float(median_duration))
    max_duration = median_duration * 2

    # truncate long words at sentence boundaries (timing.py:301-312)
    if len(word_durations) > 0:
        sentence_end_marks = ".。!！?？"
        for i in range(1, len(alignment)):
            if alignment[i].end - alignment[i].start > max_duration:
                if alignment[i].word in sentence_end_marks:
                    alignment[i].end = alignment[i].start + max_duration
                elif alignment[i - 1].word in sentence_end_marks:
                    alignment[i].start = alignment[i].end - max_duration

    merge_punctuations(alignment, prepend_punctuations, append_punctuations)

    time_offset = segments[0]["seek"] * HOP_LENGTH / SAMPLE_RATE
    word_index = 0

    for segment, text_tokens in zip(segments, text_tokens_per_segment):
        saved_tokens = 0
        words = []

        while word_index < len(alignment) and saved_tokens < len(text_tokens):
            timing = alignment[word_index]

            if timing.word:
                words.append(dict(word=timing.word, start=round(time_offset + timing.start, 2),
                                  end=round(time_offset + timing.end, 2), probability=timing.probability))

            saved_tokens += len(timing.tokens)
            word_index += 1

        # truncate long words at segment boundaries (timing.py:343-360)
        if len(words) > 0:
            if words[0]["end"] - last_speech_timestamp > median_duration * 4 and (
                    words[0]["end"] - words[0]["start"] > max_duration
                    or (len(words) > 1 and words[1]["end"] - words[0]["start"] > max_duration * 2)):
                if len(words) > 1 and words[1]["end"] - words[1]["start"] > max_duration:
                    boundary = max(words[1]["end"] / 2, words[1]["end"] - max_duration)
                    words[0]["end"] = words[1]["start"] = boundary
                words[0]["start"] = max(0, words[0]["end"] - max_duration)

            # prefer the segment-level start timestamp if the first word is too long
            if segment["start"] < words[0]["end"] and segment["start"] - 0.5 > words[0]["start"]:
                words[0]["start"] = max(0, min(words[0]["end"] - median_duration, segment["start"]))
            else:
                segment["start"] = words[0]["start"]

            # prefer the segment-level end timestamp if the last word is too long
            if segment["end"] > words[-1]["start"] and segment["end"] + 0.5 < words[-1]["end"]:
                words[-1]["end"] = max(words[-1]["start"] + median_duration, segment["end"])
            else:
                segment["end"] = words[-1]["end"]

            last_speech_timestamp = segment["end"]

        segment["words"] = words
