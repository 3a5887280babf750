"""DecodingOptions(prefix=...) against the reference (decoding.py:614-640).

The reference slices the prefix with ``prefix_tokens[-max_prefix_len:]`` where
``max_prefix_len = n_ctx // 2 - sample_len``: at the default sample_len (224) that is
``[-0:]``, which keeps the WHOLE prefix; sample_len = 200 keeps the last 24 tokens;
sample_len = 300 gives ``[76:]``, which drops the FIRST 76.  tests/golden/prefix.json
holds the reference's own decode results for those cases (oracle/gen_golden.py
prefix_goldens: micro and tiny.en, greedy and beam 5, list and string prefixes, a
prefix with a prompt).

* CPU: the initial token sequence equals the oracle's restatement
  (oracle/ref_whisper.py decode) for every golden case;
* GPU: fp32 decode tokens equal the reference's exactly.
"""
import json
import os
from types import SimpleNamespace

import numpy as np
import pytest

from conftest import GOLDEN


def _golden():
    with open(os.path.join(GOLDEN, "prefix.json")) as f:
        return json.load(f)


def _shell(name):
    import whisper
    from whisper import synthetic as S
    dims = whisper.ModelDimensions(**S.MODEL_DIMS[name])
    ml = dims.n_vocab >= 51865
    return SimpleNamespace(dims=dims, is_multilingual=ml, num_languages=dims.n_vocab - 51765 - int(ml))


def _options(case_opts):
    import whisper
    return whisper.DecodingOptions(language="en", temperature=0.0, **case_opts)


CASES = [(n, c) for n in ("micro", "tiny.en") for c in ("list_default", "list_len200", "list_len300", "str_default",
                                                        "list_default_beam", "prompt_prefix")]


@pytest.mark.parametrize("name,case", CASES)
def test_initial_tokens_match_oracle(name, case):
    from oracle import ref_whisper as R
    from whisper import synthetic as S
    from whisper.decoding import DecodingTask
    g = _golden()[name]["cases"][case]
    task = DecodingTask(_shell(name), _options(g["options"]))
    dims = S.MODEL_DIMS[name]
    st = R.SpecialTokens.for_model(dims)
    o = g["options"]
    pre = o["prefix"] if not isinstance(o["prefix"], str) else task.tokenizer.encode(" " + o["prefix"].strip())
    sample_len = o.get("sample_len") or dims["n_text_ctx"] // 2
    # the oracle's construction (ref_whisper.decode, decoding.py:614-640)
    want = list(st.sot_sequence) + list(pre)[-(dims["n_text_ctx"] // 2 - sample_len):]
    if o.get("prompt"):
        want = [st.sot_prev] + list(o["prompt"])[-(dims["n_text_ctx"] // 2 - 1):] + want
    assert list(task.initial_tokens) == want
    if case == "list_default":
        assert len(task.initial_tokens) == len(st.sot_sequence) + 100  # the whole prefix
    if case == "list_len300":
        assert list(task.initial_tokens[len(st.sot_sequence):]) == list(pre)[76:]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["micro", "tiny.en"])
def test_prefix_decode_matches_reference(name):
    """Every golden prefix case decodes (fp32, natural) to the reference's tokens."""
    import whisper
    from conftest import full_model, golden_window
    from whisper import synthetic as S
    gall = _golden()[name]
    if name == "micro":
        m = whisper.load_model("micro", device=0, dtype="fp32", max_windows=1, max_group=5, synthetic=True)
        audio = S.synthetic_audio(30.0, seed=gall["audio_seed"])
        mel = whisper.pad_or_trim(whisper.log_mel_spectrogram(audio, m.dims.n_mels, padding=whisper.audio.N_SAMPLES)
                                  [:, :3000], 3000)
    else:
        m = full_model(name, "fp32")
        mel = golden_window(name, gall["audio_seed"])
    try:
        for case, g in gall["cases"].items():
            res = whisper.decode(m, mel, _options(g["options"]))
            np.testing.assert_array_equal(np.asarray(res.tokens), np.asarray(g["tokens"]), err_msg=f"{name} {case}")
            assert res.avg_logprob == pytest.approx(g["avg_logprob"], abs=1e-3), case
    finally:
        if name == "micro":
            m.close()
