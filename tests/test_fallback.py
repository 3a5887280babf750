"""Temperature fallback of a batch of windows (reference transcribe.py:188-228).

CPU: the batched driver re-decodes exactly the windows that still fail, each from the
encoder slot that holds its own audio (original batch index), at every temperature,
and stores every result under its own window (run_windows scripted, no GPU).
GPU: decode windows straight from chosen encoder slots (wh_decode_begin_slots) gives
what decoding the same windows encoded into slots 0..k-1 gives, and a batched
transcribe whose thresholds fail only some windows runs through three temperatures."""
import numpy as np
import pytest

from whisper.decoding import DecodingOptions, DecodingResult


def _res(avg, t):
    return DecodingResult(audio_features=None, language="en", tokens=[1, 2], text="", avg_logprob=avg,
                          no_speech_prob=0.0, temperature=t, compression_ratio=1.0)


def _transcribe_module():
    import importlib
    return importlib.import_module("whisper.transcribe")  # the package re-exports the function


def test_batched_fallback_keeps_window_identity(monkeypatch):
    T = _transcribe_module()
    calls = []
    # avg_logprob per (window, temperature): window 1 recovers at 0.4, window 3 never,
    # windows 0 and 2 pass at 0.0
    table = {(0, 0.0): -0.1, (1, 0.0): -2.0, (2, 0.0): -0.2, (3, 0.0): -3.0,
             (1, 0.2): -1.5, (3, 0.2): -1.7, (1, 0.4): -0.5, (3, 0.4): -1.9}

    def fake_run_windows(model, opts, prompts, audio_features=False, slots=None):
        win = list(range(len(prompts))) if slots is None else list(slots)
        calls.append((opts.temperature, win, list(prompts)))
        return [_res(table[(w, opts.temperature)], opts.temperature) for w in win]

    monkeypatch.setattr(T, "run_windows", fake_run_windows)
    prompts = [[10], [11], [12], [13]]
    out = T._decode_with_fallback(object(), DecodingOptions(), [0.0, 0.2, 0.4], prompts, (2.4, -1.0, 0.6))
    assert [(t, w) for t, w, _ in calls] == [(0.0, [0, 1, 2, 3]), (0.2, [1, 3]), (0.4, [1, 3])]
    assert [p for _, _, p in calls][1] == [[11], [13]]
    assert [r.temperature for r in out] == [0.0, 0.4, 0.0, 0.4]
    assert [r.avg_logprob for r in out] == [-0.1, -0.5, -0.2, -1.9]


def test_batched_fallback_shrinking_subset(monkeypatch):
    """pending [1, 3] then [3] (the case that used to index a re-encoded subset)."""
    T = _transcribe_module()
    seen = []
    table = {0.0: {0: -0.1, 1: -2.0, 2: -0.1, 3: -2.0}, 0.2: {1: -0.3, 3: -2.0}, 0.4: {3: -0.2}}

    def fake_run_windows(model, opts, prompts, audio_features=False, slots=None):
        win = list(range(len(prompts))) if slots is None else list(slots)
        seen.append(win)
        return [_res(table[opts.temperature][w], opts.temperature) for w in win]

    monkeypatch.setattr(T, "run_windows", fake_run_windows)
    out = T._decode_with_fallback(object(), DecodingOptions(), [0.0, 0.2, 0.4], [None] * 4, (None, -1.0, None))
    assert seen == [[0, 1, 2, 3], [1, 3], [3]]
    assert [r.temperature for r in out] == [0.0, 0.2, 0.0, 0.4]


@pytest.mark.gpu
def test_decode_from_chosen_slots():
    import whisper
    from whisper import synthetic as S
    from whisper.decoding import run_windows
    m = whisper.load_model("micro", device=0, dtype="fp32", max_windows=4, max_group=5, synthetic=True)
    try:
        audio = S.synthetic_audio(95.0, seed=21)
        mel = whisper.log_mel_spectrogram(audio, 80, padding=whisper.audio.N_SAMPLES)
        m.ctx.mel_write(mel)
        seeks = [0, 3000, 6000]
        opts = DecodingOptions(language="en", beam_size=5)
        m.ctx.encode(seeks, [3000] * 3)
        picked = run_windows(m, opts, [None, None], slots=[2, 0])
        m.ctx.encode([seeks[2], seeks[0]], [3000, 3000])
        fresh = run_windows(m, opts, [None, None])
        for a, b in zip(picked, fresh):
            assert a.tokens == b.tokens and a.avg_logprob == b.avg_logprob
    finally:
        m.close()


@pytest.mark.gpu
def test_batched_transcribe_with_partial_fallback():
    """clip grid (batched schedule) with a logprob threshold that only some windows
    miss at T = 0: three temperatures, results stay per window; the windows that pass
    at T = 0 equal the sequential schedule's."""
    import whisper
    from whisper import synthetic as S
    m = whisper.load_model("micro", device=0, dtype="fp32", max_windows=4, max_group=5, synthetic=True)
    try:
        audio = S.synthetic_audio(120.0, seed=5)
        clips = "0,30,30,60,60,90,90,120"
        probe = whisper.transcribe(m, audio, temperature=0.0, language="en", condition_on_previous_text=False,
                                   clip_timestamps=clips, logprob_threshold=None, no_speech_threshold=None,
                                   compression_ratio_threshold=None)
        lps = sorted({s["avg_logprob"] for s in probe["segments"]})
        assert len(lps) >= 2
        thr = (lps[0] + lps[-1]) / 2
        kw = dict(language="en", condition_on_previous_text=False, clip_timestamps=clips, logprob_threshold=thr,
                  no_speech_threshold=None, compression_ratio_threshold=None, temperature=(0.0, 0.2, 0.4))
        out = whisper.transcribe(m, audio, schedule="batched", **kw)
        temps = {s["temperature"] for s in out["segments"]}
        assert 0.0 in temps and temps - {0.0}
        seq = whisper.transcribe(m, audio, schedule="sequential", **kw)
        a = [s["tokens"] for s in out["segments"] if s["temperature"] == 0.0]
        b = [s["tokens"] for s in seq["segments"] if s["temperature"] == 0.0]
        assert a == b
    finally:
        m.close()
