"""Pins the CPU oracle (oracle/ref_whisper.py) to golden vectors produced by the
reference itself (oracle/gen_golden.py).  CPU only."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import ref_whisper as R
from whisper import synthetic as S

from conftest import GOLDEN


def _golden(name):
    return np.load(os.path.join(GOLDEN, f"{name}.npz"))


@pytest.fixture(scope="module")
def micro():
    g = _golden("micro")
    dims = S.MODEL_DIMS["micro"]
    sd = S.synthetic_state_dict(dims, int(g["seed"]))
    assert S.state_dict_checksum(sd) == pytest.approx(float(g["weights_checksum"]), rel=1e-12)
    return R.OracleWhisper(dims, sd), g


def test_mel_cases():
    g = _golden("mel")
    for m in json.loads(str(g["meta"])):
        if m["seconds"] > 100:
            continue
        audio = S.synthetic_audio(m["seconds"], seed=m["seed"])
        mel = R.log_mel_spectrogram(audio, m["n_mels"], padding=m["padding"]).numpy()
        assert mel.shape[1] == m["frames"]
        tag = m["tag"]
        assert mel.max() == pytest.approx(float(g[f"{tag}_max"]), abs=1e-5)
        np.testing.assert_allclose(mel.astype(np.float64).sum(axis=0), g[f"{tag}_colsum"], rtol=1e-5, atol=1e-3)
        if f"{tag}_full" in g:
            np.testing.assert_allclose(mel, g[f"{tag}_full"], rtol=0, atol=1e-5)


def test_micro_encoder_and_first_pass(micro):
    model, g = micro
    audio = S.synthetic_audio(30.0, seed=int(g["audio_seed"]))
    mel = R.pad_or_trim(R.log_mel_spectrogram(audio, 80, padding=R.N_SAMPLES)[:, :3000])
    assert float(mel.double().sum()) == pytest.approx(float(g["mel_window_sum"]), rel=1e-9)
    xa = model.encode(mel)
    np.testing.assert_allclose(xa.numpy(), g["xa_full"], atol=2e-5, rtol=0)
    model.set_audio(xa)
    logits, _, _ = model.decoder_forward(torch.tensor([list(g["sot_sequence"])]), 0, None)
    np.testing.assert_allclose(logits[0, -1].numpy(), g["first_last_full"], atol=2e-5, rtol=0)
    np.testing.assert_array_equal(torch.topk(logits[0, 0], 64).indices.numpy(), g["first_sot_topi"])


@pytest.mark.parametrize("key,opts", [
    ("greedy", dict()),
    ("greedy_fixed", dict(suppress_tokens="-1,50257")),
    ("greedy_prompt", dict(prompt=list(range(1000, 1040)))),
    ("greedy_notime", dict(without_timestamps=True)),
    ("beam", dict(beam_size=5)),
    ("beam_fixed", dict(beam_size=5, suppress_tokens="-1,50257")),
])
def test_micro_decode(micro, key, opts):
    model, g = micro
    audio = S.synthetic_audio(30.0, seed=int(g["audio_seed"]))
    mel = R.pad_or_trim(R.log_mel_spectrogram(audio, 80, padding=R.N_SAMPLES)[:, :3000])
    res = R.decode(model, mel, R.Options(**opts))
    np.testing.assert_array_equal(np.asarray(res.tokens), g[f"{key}_tokens"])
    assert res.avg_logprob == pytest.approx(float(g[f"{key}_avg_logprob"]), abs=1e-4)
    assert res.no_speech_prob == pytest.approx(float(g[f"{key}_no_speech_prob"]), rel=1e-4, abs=1e-9)


@pytest.mark.parametrize("run", ["clip_beam", "clip_greedy", "seq_greedy", "seq_beam"])
def test_micro_transcribe(micro, run):
    model, _ = micro
    with open(os.path.join(GOLDEN, "micro_transcribe.json")) as f:
        gt = json.load(f)
    kw = dict(gt["runs"][run])
    audio = S.synthetic_audio(gt["audio_seconds"], seed=gt["audio_seed"])
    segs = R.transcribe(model, audio, **kw)
    ref = gt["segments"][run]
    assert [s["tokens"] for s in segs] == [s["tokens"] for s in ref]
    assert [s["seek"] for s in segs] == [s["seek"] for s in ref]
    for a, b in zip(segs, ref):
        assert a["start"] == pytest.approx(b["start"]) and a["end"] == pytest.approx(b["end"])
        assert a["avg_logprob"] == pytest.approx(b["avg_logprob"], abs=1e-4)


@pytest.mark.parametrize("name", ["micro", "tiny.en"])
def test_beam_options(name):
    """patience / length_penalty (decoding.py:223-240, 334-345, 400-431) against the
    reference's natural-mode decodes on the EOT-scaled seeded weights
    (tests/golden/beam_options.json, oracle/gen_golden.py beam_option_goldens): chosen
    tokens, avg_logprob, and every finished candidate (length, summed log-probability)."""
    with open(os.path.join(GOLDEN, "beam_options.json")) as f:
        gb = json.load(f)[name]
    dims = S.MODEL_DIMS[name]
    sd = S.synthetic_state_dict(dims, gb["seed"])
    S.scale_eot_embedding(sd, dims, gb["eot_scale"])
    model = R.OracleWhisper(dims, sd)
    for aseed in gb["audio_seeds"][:1 if name == "tiny.en" else None]:
        audio = S.synthetic_audio(30.0, seed=aseed)
        mel = R.pad_or_trim(R.log_mel_spectrogram(audio, dims["n_mels"], padding=R.N_SAMPLES)[:, :3000])
        xa = model.encode(mel)
        for key, case in gb["cases"][str(aseed)].items():
            res = R.decode(model, mel, R.Options(**case["options"]), xa=xa)
            assert res.tokens == case["tokens"], (aseed, key)
            assert res.avg_logprob == pytest.approx(case["avg_logprob"], abs=1e-4), (aseed, key)
            assert [c[0] for c in res.candidates] == [c[0] for c in case["candidates"]], (aseed, key)
            np.testing.assert_allclose([c[1] for c in res.candidates], [c[1] for c in case["candidates"]], atol=1e-3)


# ----------------------------------------------------------------------------- timing.py
def test_dtw_oracle_against_reference():
    """oracle/ref_timing.dtw_cpu vs the reference's dtw_cpu outputs (dtw.npz): planted
    paths (the construction of the reference's tests/test_timing.py) and random paths."""
    from oracle import ref_timing as RT
    g = _golden("dtw")
    for key in g.files:
        if key.startswith("planted_") and key.endswith("_x"):
            base = key[:-2]
            if base == "planted_123x1500":
                continue  # 184k cells in numpy: covered on the GPU (tests/test_gpu_words.py)
            np.testing.assert_array_equal(RT.dtw_cpu(g[key].astype(np.float64)), g[base + "_trace"])
        if key.startswith("rand_") and key.endswith("_x"):
            base = key[:-2]
            np.testing.assert_array_equal(RT.dtw_cpu(g[key].astype(np.float64)), g[base + "_path"])


def test_median_filter_oracle_against_reference():
    from oracle import ref_timing as RT
    g = _golden("dtw")
    for key in g.files:
        if key.startswith("med_") and key.endswith("_x"):
            base = key[:-2]
            x = torch.from_numpy(g[key])
            for w in (3, 5, 7, 13):
                np.testing.assert_array_equal(RT.median_filter(x, w).numpy(), g[f"{base}_w{w}"])


def test_word_split_matches_reference_alignment_words():
    """Product tokenizer word splitting (tokenizer.py:277-327 restated) reproduces the
    words/token groups of the reference's find_alignment (micro_words.json)."""
    from whisper import tokenizer as T
    with open(os.path.join(GOLDEN, "micro_words.json")) as f:
        gw = json.load(f)
    if True:  # the shipped rank file (whisper/assets/multilingual.tiktoken)
        tok = T.get_tokenizer(True, num_languages=S.MODEL_DIMS["micro"]["n_vocab"] - 51765 - 1, language="en",
                              task="transcribe")
        for case in gw["find_alignment"].values():
            words, word_tokens = tok.split_to_word_tokens(case["text_tokens"] + [tok.eot])
            ref = case["words"]
            if len(word_tokens) <= 1:
                assert ref == []
                continue
            # find_alignment zips words with len(word_tokens) - 1 boundaries: the eot word drops
            assert len(ref) == len(words) - 1
            assert [w["word"] for w in ref] == words[:-1]
            assert [w["tokens"] for w in ref] == word_tokens[:-1]
