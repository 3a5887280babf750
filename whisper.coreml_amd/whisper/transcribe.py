"""Long-form transcription driver (reference whisper/transcribe.py:41-524).

Same options and segment semantics as the reference loop (30 s windows, data-
dependent ``seek``, temperature fallback, prompt carry-over, no-speech skip,
empty-segment clearing).  Two schedules:

* sequential — the reference order, one window at a time; required whenever a
  window depends on the previous one (``condition_on_previous_text=True``,
  ``carry_initial_prompt``, ``hallucination_silence_threshold``);
* batched — with ``condition_on_previous_text=False`` and several clips
  (``clip_timestamps`` on a grid), windows of different clips are independent
  (each clip's seek is clip-local, the prompt resets every window:
  transcribe.py:277-287, 513-515), so every round encodes and decodes the next
  window of *all* unfinished clips together on the GPU.  Segments are assembled
  in clip order afterwards, which reproduces the reference's output exactly.
  With word timestamps the alignment of every window runs in the round (GPU);
  the words are then re-derived in clip order with the reference's running
  ``last_speech_timestamp``; if that would move any window's seek (it can only
  through a one-word last segment) the file is re-run sequentially.

The log-mel of the whole file is computed on the GPU and stays there; windows
are cut from it on the device.
"""

import os
import warnings
from dataclasses import replace
from typing import TYPE_CHECKING, List, Optional, Tuple, Union

import numpy as np

from .audio import FRAMES_PER_SECOND, HOP_LENGTH, N_FRAMES, N_SAMPLES, SAMPLE_RATE, load_audio
from .backend_hip import DeviceAudio
from .decoding import DecodingOptions, DecodingResult, detect_language, run_windows
from .timing import WordTiming, apply_alignment, find_alignment, find_alignment_batch
from .tokenizer import LANGUAGES, get_tokenizer

if TYPE_CHECKING:
    from .model import Whisper


def _decode_with_fallback(model, base_opts: DecodingOptions, temperatures, prompts: List, thresholds
                          ) -> List[DecodingResult]:
    """transcribe.py:188-228 for a batch of windows (slots 0..n-1 already encoded).
    A retry at the next temperature decodes only the windows that still need work,
    from the encoder slots that already hold their audio features (no re-encode)."""
    cr_thr, lp_thr, ns_thr = thresholds
    n = len(prompts)
    results: List[Optional[DecodingResult]] = [None] * n
    pending = list(range(n))
    for t in temperatures:
        kw = {}
        if t > 0:
            kw = dict(beam_size=None, patience=None)
        else:
            kw = dict(best_of=None)
        opts = replace(base_opts, temperature=t, **kw)
        if t > 0 and opts.best_of is None:
            opts = replace(opts, best_of=None)
        res = run_windows(model, opts, [prompts[i] for i in pending],
                          slots=None if pending == list(range(n)) else pending)
        nxt = []
        for i, r in zip(pending, res):
            results[i] = r
            fallback = False
            if cr_thr is not None and r.compression_ratio > cr_thr:
                fallback = True
            if lp_thr is not None and r.avg_logprob < lp_thr:
                fallback = True
            if ns_thr is not None and r.no_speech_prob > ns_thr and lp_thr is not None and r.avg_logprob < lp_thr:
                fallback = False
            if fallback:
                nxt.append(i)
        pending = nxt
        if not pending:
            break
    return results


def _split_segments(tokenizer, result: DecodingResult, seek: int, time_offset: float, segment_size: int,
                    segment_duration: float, input_stride: int, time_precision: float
                    ) -> Tuple[List[dict], int, bool]:
    """Segment building and seek advance of transcribe.py:350-410; returns (segments,
    seek, single_timestamp_ending)."""
    tokens = np.asarray(result.tokens, dtype=np.int64)
    tb = tokenizer.timestamp_begin

    def new_segment(start, end, toks):
        toks = [int(x) for x in toks]
        return dict(seek=seek, start=start, end=end, text=tokenizer.decode([x for x in toks if x < tokenizer.eot]),
                    tokens=toks, temperature=result.temperature, avg_logprob=result.avg_logprob,
                    compression_ratio=result.compression_ratio, no_speech_prob=result.no_speech_prob)

    segs = []
    is_ts = tokens >= tb
    single_end = is_ts[-2:].tolist() == [False, True]
    consecutive = np.where(is_ts[:-1] & is_ts[1:])[0] + 1
    if len(consecutive) > 0:
        slices = consecutive.tolist()
        if single_end:
            slices.append(len(tokens))
        last = 0
        for cut in slices:
            part = tokens[last:cut]
            segs.append(new_segment(time_offset + (int(part[0]) - tb) * time_precision,
                                    time_offset + (int(part[-1]) - tb) * time_precision, part))
            last = cut
        if single_end:
            seek += segment_size
        else:
            seek += (int(tokens[last - 1]) - tb) * input_stride
    else:
        duration = segment_duration
        ts = tokens[is_ts]
        if len(ts) > 0 and int(ts[-1]) != tb:
            duration = (int(ts[-1]) - tb) * time_precision
        segs.append(new_segment(time_offset, time_offset + duration, tokens))
        seek += segment_size
    return segs, seek, single_end


def _check_fp16(model: "Whisper", fp16: bool):
    """transcribe.py:131-140 picks the compute dtype from ``fp16``; here the precision is
    fixed when the context is created (``load_model(..., dtype=)``).  fp16=True on an
    fp32 context computes in fp32 without a warning (the reference warns only on CPU,
    and this fork has that warning commented out, reference transcribe.py:136);
    fp16=False on an fp16 context cannot be honoured and raises instead of silently
    computing in fp16."""
    if not fp16 and model.dtype != "fp32":
        raise ValueError("fp16=False needs a context loaded with dtype='fp32' "
                         "(load_model(..., dtype='fp32')); this one computes in fp16")


def _clear_empty(tokenizer, segs: List[dict]):
    """transcribe.py:494-499 (after word timestamps)."""
    for s in segs:
        if s["start"] == s["end"] or tokenizer.is_blank_text(s["tokens"]):
            s["text"] = ""
            s["tokens"] = []
            s["words"] = []


def transcribe(model: "Whisper", audio: Union[str, np.ndarray], *, verbose: Optional[bool] = None,
               temperature: Union[float, Tuple[float, ...]] = (0.0, 0.2, 0.4, 0.6, 0.8, 1.0),
               compression_ratio_threshold: Optional[float] = 2.4, logprob_threshold: Optional[float] = -1.0,
               no_speech_threshold: Optional[float] = 0.6, condition_on_previous_text: bool = True,
               initial_prompt: Optional[Union[str, List[int]]] = None, carry_initial_prompt: bool = False,
               word_timestamps: bool = False, prepend_punctuations: str = "\"'“¿([{-",
               append_punctuations: str = "\"'.。,，!！?？:：”)]}、", clip_timestamps: Union[str, List[float]] = "0",
               hallucination_silence_threshold: Optional[float] = None, schedule: str = "auto",
               mel_max_reduce=None, _mel_prepared: Optional[Tuple[int, int, int]] = None,
               **decode_options) -> dict:
    """transcribe.py:41-524.  Extra keywords: ``schedule`` ("auto", "sequential",
    "batched") and ``mel_max_reduce`` (callable local max -> global max, used when
    one file is sharded over GPUs: the log-mel floor is a whole-file max,
    audio.py:155, so ranks all-reduce it before normalizing)."""
    _check_fp16(model, decode_options.pop("fp16", True))
    ctx = model.ctx
    n_mels = model.dims.n_mels
    if _mel_prepared is not None:
        # distributed.run_shard: this rank's frames are already in the context and
        # normalised with the all-reduced max; seeks stay absolute
        if decode_options.get("language") is None:
            raise ValueError("sharded transcription needs an explicit language")

        def compute_mel():
            return _mel_prepared[0]
        mel_max_reduce = None
    elif isinstance(audio, DeviceAudio):
        if audio.ctx is not ctx:
            raise ValueError("DeviceAudio belongs to another model context")
        resident = audio.n_samples

        def compute_mel():
            return ctx.log_mel_resident(resident, n_mels, padding=N_SAMPLES, normalize=mel_max_reduce is None)
    else:
        if isinstance(audio, str):
            audio = load_audio(audio)
        audio = np.ascontiguousarray(audio.detach().cpu().numpy() if hasattr(audio, "detach") else audio,
                                     dtype=np.float32)

        def compute_mel():
            return ctx.log_mel(audio, n_mels, padding=N_SAMPLES, normalize=mel_max_reduce is None)

    def prepare_mel():
        nf = compute_mel()
        if mel_max_reduce is not None and _mel_prepared is None:
            ctx.mel_normalize(float(mel_max_reduce(ctx.mel_max())))
        return nf

    frames = prepare_mel()
    content_frames = frames - N_FRAMES
    content_duration = float(content_frames * HOP_LENGTH / SAMPLE_RATE)

    if decode_options.get("language") is None:
        if not model.is_multilingual:
            decode_options["language"] = "en"
        else:
            seg = ctx.mel_read(n_mels, 0, min(N_FRAMES, frames))
            if seg.shape[1] < N_FRAMES:
                seg = np.pad(seg, ((0, 0), (0, N_FRAMES - seg.shape[1])))
            _, probs = detect_language(model, seg)
            decode_options["language"] = max(probs, key=probs.get)
            # detect_language overwrote the context mel with the probe window
            frames = prepare_mel()
            if verbose is not None:
                print(f"Detected language: {LANGUAGES[decode_options['language']].title()}")
    language = decode_options["language"]
    task = decode_options.get("task", "transcribe")
    tokenizer = get_tokenizer(model.is_multilingual, num_languages=model.num_languages, language=language,
                              task=task)

    if isinstance(clip_timestamps, str):
        clip_timestamps = [float(ts) for ts in (clip_timestamps.split(",") if clip_timestamps else [])]
    seek_points = [round(ts * FRAMES_PER_SECOND) for ts in clip_timestamps]
    if len(seek_points) == 0:
        seek_points.append(0)
    if len(seek_points) % 2 == 1:
        seek_points.append(content_frames)
    seek_clips = list(zip(seek_points[::2], seek_points[1::2]))

    temperatures = [temperature] if isinstance(temperature, (int, float)) else list(temperature)
    thresholds = (compression_ratio_threshold, logprob_threshold, no_speech_threshold)
    base = DecodingOptions(**{k: v for k, v in decode_options.items() if k in DecodingOptions.__dataclass_fields__})
    input_stride = N_FRAMES // model.dims.n_audio_ctx
    time_precision = input_stride * HOP_LENGTH / SAMPLE_RATE

    if isinstance(initial_prompt, str):  # transcribe.py:243-244
        initial_prompt_tokens = tokenizer.encode(" " + initial_prompt.strip())
    else:
        initial_prompt_tokens = list(initial_prompt) if initial_prompt else []

    if word_timestamps and task == "translate":
        warnings.warn("Word-level timestamps on translations may not be reliable.")
    batched = schedule == "batched" or (
        schedule == "auto" and not condition_on_previous_text and not carry_initial_prompt
        and not initial_prompt_tokens and len(seek_clips) > 1)
    if hallucination_silence_threshold is not None and word_timestamps:
        batched = False  # its seek rules read the running last_speech_timestamp
    state = dict(content_frames=content_frames, content_duration=content_duration, tokenizer=tokenizer,
                 temperatures=temperatures, thresholds=thresholds, base=base, input_stride=input_stride,
                 time_precision=time_precision, word_timestamps=word_timestamps, prepend=prepend_punctuations,
                 append=append_punctuations, hallucination=hallucination_silence_threshold)
    segments = None
    if batched:
        segments = _run_batched(model, seek_clips, initial_prompt_tokens, state)
    if segments is None:
        segments = _run_sequential(model, seek_clips, initial_prompt_tokens, condition_on_previous_text,
                                   carry_initial_prompt, state)
    all_tokens = list(initial_prompt_tokens)
    all_segments = []
    for s in segments:
        all_segments.append({"id": len(all_segments), **s})
        all_tokens.extend(s["tokens"])
        if verbose:
            print(f"[{s['start']:.2f} --> {s['end']:.2f}] {s['text']}")
    return dict(text=tokenizer.decode(all_tokens[len(initial_prompt_tokens):]), segments=all_segments,
                language=language)


def _window_at(seek: int, clip: Tuple[int, int], content_frames: int):
    segment_size = min(N_FRAMES, content_frames - seek, clip[1] - seek)
    return segment_size, segment_size * HOP_LENGTH / SAMPLE_RATE


def _apply_result(model, result, seek, segment_size, st) -> Tuple[List[dict], int, bool, bool]:
    """no-speech skip (transcribe.py:308-321) then segment split; returns
    (segments, new seek, skipped, single_timestamp_ending).  Empty segments are not
    cleared yet (word timestamps see them first, transcribe.py:412-499)."""
    thr_ns, thr_lp = st["thresholds"][2], st["thresholds"][1]
    if thr_ns is not None:
        skip = result.no_speech_prob > thr_ns
        if thr_lp is not None and result.avg_logprob > thr_lp:
            skip = False
        if skip:
            return [], seek + segment_size, True, False
    time_offset = float(seek * HOP_LENGTH / SAMPLE_RATE)
    segs, new_seek, single_end = _split_segments(st["tokenizer"], result, seek, time_offset, segment_size,
                                                 segment_size * HOP_LENGTH / SAMPLE_RATE, st["input_stride"],
                                                 st["time_precision"])
    return segs, new_seek, False, single_end


def get_end(segments: List[dict]) -> Optional[float]:
    """utils.py:78-82."""
    return next((w["end"] for s in reversed(segments) for w in reversed(s.get("words", []))),
                segments[-1]["end"] if segments else None)


_PUNCTUATION = "\"'“¿([{-\"'.。,，!！?？:：”)]}、"  # transcribe.py:183


def _word_anomaly_score(word: dict) -> float:
    """transcribe.py:327-337."""
    probability = word.get("probability", 0.0)
    duration = word["end"] - word["start"]
    score = 0.0
    if probability < 0.15:
        score += 1.0
    if duration < 0.133:
        score += (0.133 - duration) * 15
    if duration > 2.0:
        score += duration - 2.0
    return score


def _is_segment_anomaly(segment: Optional[dict]) -> bool:
    """transcribe.py:339-345."""
    if segment is None or not segment["words"]:
        return False
    words = [w for w in segment["words"] if w["word"] not in _PUNCTUATION]
    words = words[:8]
    score = sum(_word_anomaly_score(w) for w in words)
    return score >= 3 or score + 0.01 >= len(words)


def _next_words_segment(segments: List[dict]) -> Optional[dict]:
    return next((s for s in segments if s["words"]), None)


def _window_alignment(model, st, segs: List[dict], segment_size: int, slot: int):
    """find_alignment of one window's segments (its audio features in `slot`)."""
    tok = st["tokenizer"]
    text_tokens = [t for s in segs for t in s["tokens"] if t < tok.eot]
    return find_alignment(model, tok, text_tokens, segment_size, slot=slot)


def _words_and_seek(st, segs, alignment, seek, previous_seek, segment_size, single_end, last_speech):
    """transcribe.py:412-426 on a precomputed alignment: words of every segment, the
    seek refinement from the last word; returns (seek, last_speech_timestamp)."""
    fresh = [WordTiming(w.word, list(w.tokens), w.start, w.end, w.probability) for w in alignment]
    apply_alignment(segs, fresh, st["tokenizer"], st["prepend"], st["append"], last_speech)
    time_offset = float(previous_seek * HOP_LENGTH / SAMPLE_RATE)
    if not single_end:
        last_word_end = get_end(segs)
        if last_word_end is not None and last_word_end > time_offset:
            seek = round(last_word_end * FRAMES_PER_SECOND)
    return seek


def _run_sequential(model, clips, initial_prompt_tokens, condition_on_previous_text, carry_initial_prompt, st):
    ctx = model.ctx
    content_frames = st["content_frames"]
    all_tokens = list(initial_prompt_tokens)
    segments = []
    prompt_reset_since = 0
    remaining_prompt_length = model.dims.n_text_ctx // 2 - 1 - len(initial_prompt_tokens)
    last_speech_timestamp = 0.0
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
        segment_size, segment_duration = _window_at(seek, clips[clip_idx], content_frames)
        if segment_duration < 1.0:  # fork: drop < 1 s tails (transcribe.py:292-297)
            clip_idx += 1
            continue
        if carry_initial_prompt:
            nignored = max(len(initial_prompt_tokens), prompt_reset_since)
            prompt = initial_prompt_tokens + all_tokens[nignored:][-remaining_prompt_length:]
        else:
            prompt = all_tokens[prompt_reset_since:]
        ctx.encode([seek], [segment_size])
        model._last_windows = ([seek], [segment_size])
        result = _decode_with_fallback(model, st["base"], st["temperatures"], [prompt or None], st["thresholds"])[0]
        previous_seek = seek
        segs, seek, skipped, single_end = _apply_result(model, result, seek, segment_size, st)
        if skipped:
            continue
        if st["word_timestamps"]:
            alignment = _window_alignment(model, st, segs, segment_size, 0) if segs else []
            seek = _words_and_seek(st, segs, alignment, seek, previous_seek, segment_size, single_end,
                                   last_speech_timestamp)
            time_offset = float(previous_seek * HOP_LENGTH / SAMPLE_RATE)
            window_end_time = float((previous_seek + N_FRAMES) * HOP_LENGTH / SAMPLE_RATE)
            segment_duration = segment_size * HOP_LENGTH / SAMPLE_RATE
            threshold = st["hallucination"]
            if threshold is not None:  # transcribe.py:428-484
                if not single_end:
                    last_word_end = get_end(segs)
                    if last_word_end is not None and last_word_end > time_offset:
                        remaining_duration = window_end_time - last_word_end
                        if remaining_duration > threshold:
                            seek = round(last_word_end * FRAMES_PER_SECOND)
                        else:
                            seek = previous_seek + segment_size
                first_segment = _next_words_segment(segs)
                if first_segment is not None and _is_segment_anomaly(first_segment):
                    gap = first_segment["start"] - time_offset
                    if gap > threshold:
                        seek = previous_seek + round(gap * FRAMES_PER_SECOND)
                        continue
                hal_last_end = last_speech_timestamp
                for si in range(len(segs)):
                    segment = segs[si]
                    if not segment["words"]:
                        continue
                    if _is_segment_anomaly(segment):
                        next_segment = _next_words_segment(segs[si + 1:])
                        if next_segment is not None:
                            hal_next_start = next_segment["words"][0]["start"]
                        else:
                            hal_next_start = time_offset + segment_duration
                        silence_before = (segment["start"] - hal_last_end > threshold
                                          or segment["start"] < threshold or segment["start"] - time_offset < 2.0)
                        silence_after = (hal_next_start - segment["end"] > threshold
                                         or _is_segment_anomaly(next_segment) or window_end_time - segment["end"] < 2.0)
                        if silence_before and silence_after:
                            seek = round(max(time_offset + 1, segment["start"]) * FRAMES_PER_SECOND)
                            if st["content_duration"] - segment["end"] < threshold:
                                seek = content_frames
                            segs[si:] = []
                            break
                    hal_last_end = segment["end"]
            last_word_end = get_end(segs)
            if last_word_end is not None:
                last_speech_timestamp = last_word_end
        _clear_empty(st["tokenizer"], segs)
        segments.extend(segs)
        all_tokens.extend(t for s in segs for t in s["tokens"])
        if not condition_on_previous_text or result.temperature > 0.5:
            prompt_reset_since = len(all_tokens)
    return segments


def _run_batched(model, clips, initial_prompt_tokens, st):
    """Rounds over clips: every unfinished clip contributes its next window."""
    ctx = model.ctx
    content_frames = st["content_frames"]
    seeks = [c[0] for c in clips]
    live = [True] * len(clips)
    per_clip: List[List[dict]] = [[] for _ in clips]
    windows: List[List[tuple]] = [[] for _ in clips]  # word timestamps: per-window records
    clip_speech = [0.0] * len(clips)
    first_window = True
    while any(live):
        batch = []  # (clip, seek, segment_size)
        for ci, (cs, ce) in enumerate(clips):
            if not live[ci]:
                continue
            if seeks[ci] < cs:
                seeks[ci] = cs
            if seeks[ci] >= ce:
                live[ci] = False
                continue
            segment_size, segment_duration = _window_at(seeks[ci], clips[ci], content_frames)
            if segment_duration < 1.0:
                live[ci] = False
                continue
            batch.append((ci, seeks[ci], segment_size))
        if not batch:
            break
        for b0 in range(0, len(batch), model.ctx.max_windows):
            chunk = batch[b0:b0 + model.ctx.max_windows]
            prompts = []
            for ci, _, _ in chunk:
                # only the very first window of the file sees the initial prompt
                prompts.append(initial_prompt_tokens if (first_window and ci == 0 and initial_prompt_tokens) else None)
            first_window = False
            ctx.encode([s for _, s, _ in chunk], [z for _, _, z in chunk])
            model._last_windows = ([s for _, s, _ in chunk], [z for _, _, z in chunk])
            results = _decode_with_fallback(model, st["base"], st["temperatures"], prompts, st["thresholds"])
            applied = [_apply_result(model, r, seek, segment_size, st) for (ci, seek, segment_size), r in
                       zip(chunk, results)]
            if st["word_timestamps"]:
                # every window's alignment of this chunk in one batched device call
                tok = st["tokenizer"]
                texts = [[t for s_ in a[0] for t in s_["tokens"] if t < tok.eot] for a in applied]
                aligns = find_alignment_batch(model, tok, texts, [z for _, _, z in chunk], list(range(len(chunk))))
            for slot, ((ci, seek, segment_size), r) in enumerate(zip(chunk, results)):
                segs, new_seek, skipped, single_end = applied[slot]
                if st["word_timestamps"] and not skipped:
                    alignment = aligns[slot]
                    # provisional: the clip-local running last-speech time (the true one,
                    # from the preceding clips, is applied in the ordered pass below)
                    new_seek = _words_and_seek(st, segs, alignment, new_seek, seek, segment_size, single_end,
                                               clip_speech[ci])
                    end = get_end(segs)
                    if end is not None:
                        clip_speech[ci] = end
                    windows[ci].append((seek, segment_size, r, alignment, new_seek))
                    segs = []
                elif st["word_timestamps"]:
                    windows[ci].append((seek, segment_size, r, None, new_seek))
                _clear_empty(st["tokenizer"], segs)
                per_clip[ci].extend(segs)
                seeks[ci] = new_seek
    if not st["word_timestamps"]:
        return [s for clip in per_clip for s in clip]
    # ordered pass: word timings with the running last_speech_timestamp of the
    # reference's sequential loop (transcribe.py:271, 412-426, 485-486); a window whose
    # seek would change under it makes the caller re-run the sequential schedule
    out, last_speech = [], 0.0
    for ci in range(len(clips)):
        for seek, segment_size, r, alignment, prov_seek in windows[ci]:
            if alignment is None:
                continue
            segs, new_seek, _, single_end = _apply_result(model, r, seek, segment_size, st)
            new_seek = _words_and_seek(st, segs, alignment, new_seek, seek, segment_size, single_end, last_speech)
            if new_seek != prov_seek:
                return None
            end = get_end(segs)
            if end is not None:
                last_speech = end
            _clear_empty(st["tokenizer"], segs)
            out.extend(segs)
    return out
