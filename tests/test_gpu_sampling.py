"""SURVEY §8(f) rows 2 and 4 on the GPU (micro model, fp32):

* temperature sampling (decoding.py:307-311 draws from Categorical(logits / T)): the
  device sampler is a Gumbel-max draw with a counter-based RNG, so it cannot match
  torch's RNG stream token for token — it is held to the distribution instead: the
  empirical frequencies of the first sampled token over many seeds against
  softmax(filtered logits / T) computed from the same first-pass logits (4-sigma
  binomial bounds) and the sampled tokens' mean log-probability against the
  distribution's entropy;
* temperature fallback (transcribe.py:188-228): thresholds that can never be met
  walk every temperature and keep the last result; no thresholds keep T = 0;
* language detection (the fork's detect_language is broken, decoding.py:58; the
  upstream behaviour — one decoder pass over <|startoftranscript|>, softmax over
  the language tokens): probabilities against the CPU oracle on the same audio."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def micro32():
    import whisper
    m = whisper.load_model("micro", device=0, dtype="fp32", max_windows=4, max_group=5,
                             synthetic=True)
    yield m
    m.close()


@pytest.fixture(scope="module")
def window(micro32):
    import whisper
    from whisper import synthetic as S
    g = np.load(os.path.join(GOLDEN, "micro.npz"))
    audio = S.synthetic_audio(30.0, seed=int(g["audio_seed"]))
    mel = whisper.log_mel_spectrogram(audio, 80, padding=whisper.audio.N_SAMPLES)
    return whisper.pad_or_trim(mel[:, :3000], 3000)


def _first_step_probs(m, mel, T):
    """softmax((first-pass logits with the first-step filters) / T) for
    without_timestamps decoding: SuppressBlank + SuppressTokens(-1) (decoding.py:450-477)."""
    from whisper.decoding import DecodingOptions, DecodingTask
    task = DecodingTask(m, DecodingOptions(language="en", temperature=T, without_timestamps=True))
    m.ctx.mel_write(mel)
    m.ctx.encode([0], [3000])
    logits, _ = m.ctx.prefill_logits(0, list(task.initial_tokens))
    x = logits[-1].astype(np.float64)
    x[task.suppress_list()] = -np.inf
    x[task.tokenizer.encode_blank() + [task.tokenizer.eot]] = -np.inf
    z = x / T
    p = np.exp(z - z.max())
    return p / p.sum(), task


@pytest.mark.parametrize("T", [0.6, 1.0])
def test_sampling_matches_categorical(micro32, window, T):
    from whisper.decoding import DecodingOptions, decode
    m = micro32
    p, _ = _first_step_probs(m, window, T)
    n = 400
    draws = []
    for _ in range(n):
        r = decode(m, window, DecodingOptions(language="en", temperature=T, sample_len=1, without_timestamps=True))
        draws.append(r.tokens[0] if r.tokens else -1)
    draws = np.asarray(draws)
    assert np.all(p[draws[draws >= 0]] > 0), "sampled a filtered token"
    for tok in np.argsort(p)[::-1][:3]:
        f = float(np.mean(draws == tok))
        sd = np.sqrt(p[tok] * (1 - p[tok]) / n)
        assert abs(f - p[tok]) <= 4 * sd + 1e-3, (int(tok), f, float(p[tok]))
    # the sampled tokens' mean log-probability matches the distribution's -entropy
    lp = np.log(p[draws[draws >= 0]])
    ent = -np.sum(p[p > 0] * np.log(p[p > 0]))
    var = np.sum(p[p > 0] * np.log(p[p > 0]) ** 2) - ent ** 2
    assert abs(lp.mean() + ent) <= 4 * np.sqrt(var / len(lp)) + 1e-3


def test_temperature_fallback_walks_every_temperature(micro32):
    import whisper
    from whisper import synthetic as S
    audio = S.synthetic_audio(35.0, seed=7)
    temps = (0.0, 0.4, 0.8)
    # an avg_logprob threshold no result can meet: every window falls back to the last T
    out = whisper.transcribe(micro32, audio, temperature=temps, language="en", logprob_threshold=10.0,
                             no_speech_threshold=None, compression_ratio_threshold=None, sample_len=16)
    assert out["segments"] and all(s["temperature"] == 0.8 for s in out["segments"])
    # no thresholds: the first temperature is kept
    out = whisper.transcribe(micro32, audio, temperature=temps, language="en", logprob_threshold=None,
                             no_speech_threshold=None, compression_ratio_threshold=None, sample_len=16)
    assert out["segments"] and all(s["temperature"] == 0.0 for s in out["segments"])


def test_detect_language_matches_oracle(micro32, window):
    from oracle import ref_whisper as R
    from whisper import synthetic as S
    from whisper.decoding import detect_language
    from whisper.tokenizer import get_tokenizer
    m = micro32
    tokens, probs = detect_language(m, window)
    dims = S.MODEL_DIMS["micro"]
    om = R.OracleWhisper(dims, S.synthetic_state_dict(dims, 0))
    om.set_audio(om.encode(torch.from_numpy(np.asarray(window))))
    tok = get_tokenizer(True, num_languages=m.num_languages)
    logits, _, _ = om.decoder_forward(torch.tensor([[tok.sot]]), 0, None)
    lang = np.asarray(tok.all_language_tokens)
    sel = logits[0, 0].double().numpy()[lang]
    ref = np.exp(sel - sel.max())
    ref /= ref.sum()
    got = np.asarray([probs[c] for c in tok.all_language_codes])
    np.testing.assert_allclose(got, ref, atol=2e-4)
    assert tokens == int(lang[int(np.argmax(sel))])
