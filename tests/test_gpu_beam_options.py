"""Non-default beam options on the device path against the reference.

patience sets the finished-set cap max_candidates = round(beam_size * patience)
(reference decoding.py:334-345, 400-406), applied on the device by k_merge inside the
step graph; length_penalty picks among the finished candidates with
((5 + len) / 6) ** alpha (decoding.py:223-240), applied by the host finalize
(whisper/decoding.py DecodingTask.finalize).  Goldens: the reference's natural-mode
decodes of tests/golden/beam_options.json (oracle/gen_golden.py beam_option_goldens) on
the seeded weights with the EOT embedding row scaled so that candidates finish at many
lengths.  fp32 contexts: tokens exact, avg_logprob within 1e-3, the finished
candidates' lengths equal and their summed log-probabilities within 1e-3 — one window
per batch (the k_proj1 layers) and all three windows in one batch (split-K k_proj)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _golden():
    with open(os.path.join(GOLDEN, "beam_options.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module", params=["micro", "tiny.en"])
def model(request):
    import whisper
    from whisper import synthetic as S
    name = request.param
    gb = _golden()[name]
    dims = S.MODEL_DIMS[name]
    sd = S.synthetic_state_dict(dims, gb["seed"])
    S.scale_eot_embedding(sd, dims, gb["eot_scale"])
    m = whisper.Whisper(whisper.ModelDimensions(**dims), name, device=0, dtype="fp32", max_windows=3, max_group=5)
    m.load_state_dict(sd)
    yield m, name, gb
    m.close()


def _mels(m, seeds):
    import whisper
    from whisper import synthetic as S
    out = []
    for s in seeds:
        audio = S.synthetic_audio(30.0, seed=s)
        mel = whisper.log_mel_spectrogram(audio, m.dims.n_mels, padding=whisper.audio.N_SAMPLES)
        out.append(whisper.pad_or_trim(mel[:, :3000], 3000))
    return out


def _decode(m, mels, opts):
    """decode() of len(mels) windows in one batch, returning per window the result and the
    candidates the ranker saw (device finished set, then finalize's unfinished fill)."""
    import whisper
    from whisper.audio import N_FRAMES
    from whisper.decoding import DecodingTask
    n = len(mels)
    m.ctx.mel_write(np.concatenate(mels, axis=1))
    m.ctx.encode([i * N_FRAMES for i in range(n)], [N_FRAMES] * n)
    task = DecodingTask(m, whisper.DecodingOptions(language="en", **opts))
    m.ctx.decode_begin(task.wh_opts(), [task.initial_tokens] * n, [task.sot_index] * n)
    m.ctx.decode_steps(task.sample_len)
    out = []
    for i in range(n):
        raw = m.ctx.decode_read(i, task.n_group)
        toks, _, avg = task.finalize(raw)
        cands = [[int(L), float(sc)] for L, sc in zip(raw["fin_len"], raw["fin_score"])]
        if len(cands) < task.n_group:  # finalize's fill with the best unfinished rows
            for j in list(np.argsort(raw["sum_logprobs"]))[::-1]:
                cands.append([raw["length"] + 1, float(raw["sum_logprobs"][j])])
                if len(cands) >= task.n_group:
                    break
        out.append((toks, avg, raw["no_speech_prob"], cands))
    return out


def _check(got, case, where):
    toks, avg, nsp, cands = got
    assert toks == case["tokens"], where
    assert avg == pytest.approx(case["avg_logprob"], abs=1e-3), where
    assert nsp == pytest.approx(case["no_speech_prob"], rel=2e-2, abs=1e-6), where
    assert [c[0] for c in cands] == [c[0] for c in case["candidates"]], where
    np.testing.assert_allclose([c[1] for c in cands], [c[1] for c in case["candidates"]], atol=1e-3,
                               err_msg=str(where))


@pytest.mark.parametrize("key", ["patience2", "patience0.5", "beam3_patience1.5", "lp0.0", "lp0.6", "lp1.0",
                                 "patience2_lp0.6", "default"])
def test_beam_option_one_window(model, key):
    m, name, gb = model
    for s in gb["audio_seeds"]:
        case = gb["cases"][str(s)][key]
        (got,) = _decode(m, _mels(m, [s]), case["options"])
        _check(got, case, (name, s, key, "1 window"))


@pytest.mark.parametrize("key", ["patience2", "beam3_patience1.5", "patience2_lp0.6"])
def test_beam_option_batched(model, key):
    m, name, gb = model
    seeds = gb["audio_seeds"]
    res = _decode(m, _mels(m, seeds), gb["cases"][str(seeds[0])][key]["options"])
    for s, got in zip(seeds, res):
        _check(got, gb["cases"][str(s)][key], (name, s, key, f"{len(seeds)} windows"))


def test_length_penalty_changes_the_choice():
    """The golden set exercises the ranker: on micro, length_penalty picks another
    candidate than the default length normalisation (else the test above proves little)."""
    gb = _golden()["micro"]["cases"]["1"]
    assert gb["lp0.6"]["tokens"] != gb["default"]["tokens"]
    assert len(gb["patience2"]["candidates"]) == 10
