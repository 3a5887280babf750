"""HIP path vs the reference's golden vectors on the micro model (n_state 128,
2+2 layers) — small enough that every stage can be compared in full.

fp32 contexts must reproduce the reference CPU path token-for-token; fp16
contexts are held to the logit tolerances stated in each test."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _golden(name):
    return np.load(os.path.join(GOLDEN, f"{name}.npz"))


@pytest.fixture(scope="module", params=["fp32", "fp16"])
def micro(request):
    import whisper
    m = whisper.load_model("micro", device=0, dtype=request.param, max_windows=4, max_group=5,
                             synthetic=True)
    yield m, request.param
    m.close()


@pytest.fixture(scope="module")
def window_mel():
    import whisper
    from whisper import synthetic as S
    g = _golden("micro")
    audio = S.synthetic_audio(30.0, seed=int(g["audio_seed"]))
    mel = whisper.log_mel_spectrogram(audio, 80, padding=whisper.audio.N_SAMPLES)
    return whisper.pad_or_trim(mel[:, :3000], 3000)


def test_window_mel_sum(window_mel):
    g = _golden("micro")
    # the window sum aggregates 240k values: fp32 DFT vs pocketfft rounding
    assert float(window_mel.astype(np.float64).sum()) == pytest.approx(float(g["mel_window_sum"]), rel=2e-5)


def test_encoder_and_cross_kv(micro, window_mel):
    m, dt = micro
    g = _golden("micro")
    m.ctx.mel_write(window_mel)
    m.ctx.encode([0], [3000])
    xa = m.ctx.audio_features(0)
    tol = 2e-3 if dt == "fp32" else 6e-2
    err = np.abs(xa - g["xa_full"]).max()
    assert err < tol, f"xa max abs err {err}"
    k, v = m.ctx.cross_kv(0, 1)
    # golden ck: (L, H, 64, 1500) -> norms per (L, H)
    np.testing.assert_allclose(np.linalg.norm(k.reshape(k.shape[0], -1), axis=1), g["ck_norm"][1],
                               rtol=2e-3 if dt == "fp32" else 2e-2)
    np.testing.assert_allclose(np.linalg.norm(v.reshape(v.shape[0], -1), axis=1), g["cv_norm"][1],
                               rtol=2e-3 if dt == "fp32" else 2e-2)


def test_first_pass_logits(micro, window_mel):
    m, dt = micro
    g = _golden("micro")
    m.ctx.mel_write(window_mel)
    m.ctx.encode([0], [3000])
    logits, _ = m.ctx.prefill_logits(0, list(g["sot_sequence"]))
    ref = g["first_last_full"]
    err = np.abs(logits[-1] - ref).max()
    tol = 2e-3 if dt == "fp32" else 5e-2 * float(np.abs(ref).max())
    assert err < tol, f"last-row logits max abs err {err}"
    assert int(np.argmax(logits[-1])) == int(np.argmax(ref))
    assert int(np.argmax(logits[0])) == int(g["first_sot_topi"][0])


@pytest.mark.parametrize("key,opts", [
    ("greedy", dict()),
    ("greedy_fixed", dict(suppress_tokens="-1,50257")),
    ("greedy_prompt", dict(prompt=list(range(1000, 1040)))),
    ("greedy_notime", dict(without_timestamps=True)),
    ("beam", dict(beam_size=5)),
    ("beam_fixed", dict(beam_size=5, suppress_tokens="-1,50257")),
])
def test_decode_tokens(micro, window_mel, key, opts):
    import whisper
    m, dt = micro
    g = _golden("micro")
    res = whisper.decode(m, window_mel, whisper.DecodingOptions(language="en", **opts))
    ref = g[f"{key}_tokens"]
    got = np.asarray(res.tokens)
    if dt == "fp32":
        np.testing.assert_array_equal(got, ref)
        assert res.avg_logprob == pytest.approx(float(g[f"{key}_avg_logprob"]), abs=2e-3)
        assert res.no_speech_prob == pytest.approx(float(g[f"{key}_no_speech_prob"]), rel=2e-2, abs=1e-7)
    else:
        # fp16: equal through the decisive prefix where the reference recorded its
        # per-step top-2 margins (greedy runs): every step whose margin exceeds twice
        # the teacher-forced fp16 logit bound (test_gpu_batch.py, micro row); other
        # runs: the first token, agreement length reported
        from test_gpu_batch import TAU, _steps
        n = min(len(got), len(ref))
        agree = int(np.argmax(got[:n] != ref[:n])) if np.any(got[:n] != ref[:n]) else n
        need = 1
        if f"{key}_margins" in g.files:
            topv = _steps("micro")["tf_greedy_fixed_topv"][:, 0]
            eps = TAU["fp16"] * float(np.median(topv[:, 0] - topv[:, -1]))
            close = g[f"{key}_margins"] <= 2 * eps
            need = int(np.argmax(close)) if close.any() else len(ref)
        print(f"{key} fp16 agreement {agree}/{len(ref)} (required {need})")
        assert agree >= min(need, n)


@pytest.mark.parametrize("micro", ["fp32"], indirect=True)  # segment-exact parity is an fp32 claim
@pytest.mark.parametrize("run,schedule", [("clip_beam", "auto"), ("clip_greedy", "auto"), ("seq_greedy", "auto"), ("seq_beam", "auto"),
                                          ("clip_beam", "sequential"), ("clip_greedy", "sequential")])
def test_transcribe_segments(micro, run, schedule):
    """clip runs under "auto" take the batched schedule (all clips' windows through
    the encoder and step graph together); "sequential" is the reference's loop."""
    import whisper
    from whisper import synthetic as S
    m, _ = micro
    with open(os.path.join(GOLDEN, "micro_transcribe.json")) as f:
        gt = json.load(f)
    kw = dict(gt["runs"][run])
    audio = S.synthetic_audio(gt["audio_seconds"], seed=gt["audio_seed"])
    out = whisper.transcribe(m, audio, temperature=0.0, language="en", schedule=schedule, **kw)
    ref = gt["segments"][run]
    assert [s["tokens"] for s in out["segments"]] == [s["tokens"] for s in ref]
    assert [s["seek"] for s in out["segments"]] == [s["seek"] for s in ref]
    for a, b in zip(out["segments"], ref):
        assert a["start"] == pytest.approx(b["start"]) and a["end"] == pytest.approx(b["end"])


@pytest.mark.parametrize("micro", ["fp32"], indirect=True)  # segment-exact parity is an fp32 claim
@pytest.mark.parametrize("run", ["clip_greedy", "clip_beam"])
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_replay_equals_reference(micro, run, world):
    """whisper/distributed.py on one GPU: every rank's phase 1 (its mel frames +
    local max), the MAX reduction, then each rank's phase 2 in turn; the merged
    segments must equal the reference transcribe() of the whole file."""
    from whisper import distributed as D
    from whisper import synthetic as S
    m, _ = micro
    with open(os.path.join(GOLDEN, "micro_transcribe.json")) as f:
        gt = json.load(f)
    kw = dict(gt["runs"][run])
    kw.pop("clip_timestamps"), kw.pop("condition_on_previous_text", None)
    audio = S.synthetic_audio(gt["audio_seconds"], seed=gt["audio_seed"])
    states = [D.prepare_shard(m, audio, r, world) for r in range(world)]
    g = max(s.local_max for s in states)
    per_rank = [D.run_shard(m, s, g, audio=audio, temperature=0.0, language="en", **kw) for s in states]
    merged = D.merge_segments(per_rank)
    ref = gt["segments"][run]
    assert [s["tokens"] for s in merged] == [s["tokens"] for s in ref]
    assert [s["seek"] for s in merged] == [s["seek"] for s in ref]
    assert [s["id"] for s in merged] == list(range(len(ref)))


def test_time_stages(micro, window_mel):
    """The bench's live timers (wh_time_stage): every stage returns a positive
    per-launch time on a live beam-5 decode batch; an unknown stage fails loudly."""
    import math

    import whisper
    from whisper.backend_hip import HipBackendError
    from whisper.decoding import DecodingTask
    m, _ = micro
    m.ctx.mel_write(window_mel)
    m.ctx.encode([0], [3000])
    task = DecodingTask(m, whisper.DecodingOptions(language="en", beam_size=5))
    m.ctx.decode_begin(task.wh_opts(), [task.initial_tokens], [task.sot_index])
    for what in (0, 2, 3, 4, 5, 6, 7):
        ms = m.ctx.time_stage(what, 2)
        assert math.isfinite(ms) and 0.0 < ms < 100.0, (what, ms)
    with pytest.raises(HipBackendError):
        m.ctx.time_stage(99, 1)
