"""The checkpoint loader against a reference-format checkpoint.

tests/golden/micro_ckpt.pt was written by oracle/gen_golden.py checkpoint_goldens: the
reference's own Whisper.state_dict() of the seeded micro weights, every tensor fp16 as the
released checkpoints store them, saved as {"dims", "model_state_dict"}; the REFERENCE's
load_model(path) (reference __init__.py:151-166) loaded it back and decoded a seeded 30 s
window on its CPU path (tests/golden/micro_ckpt.json).  Here whisper.load_model(path)
(whisper/__init__.py: torch.load(weights_only=True) -> dims -> load_state_dict) must give
the reference's tokens exactly in fp32 (greedy and beam 5 with EOT suppressed, natural
greedy), from the file and from bytes (in_memory=True).  The CPU half checks the file
itself: its hash, its key set = the reference model's, fp16 tensors, loadable without
unpickling code."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

CKPT = os.path.join(GOLDEN, "micro_ckpt.pt")


def _golden():
    with open(os.path.join(GOLDEN, "micro_ckpt.json")) as f:
        return json.load(f)


def test_checkpoint_file_is_reference_format():
    import torch
    g = _golden()
    with open(CKPT, "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == g["sha256"]
    ck = torch.load(CKPT, map_location="cpu", weights_only=True)
    assert set(ck) == {"dims", "model_state_dict"}
    assert ck["dims"] == g["dims"]
    sd = ck["model_state_dict"]
    assert sorted(sd) == g["keys"]
    assert all(v.dtype == torch.float16 for v in sd.values())
    # the same key set as our seeded generator (what the GPU context's loader expects)
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(GOLDEN), "..", "whisper.coreml_amd"))
    from whisper import synthetic as S
    assert set(S.synthetic_state_dict(S.MODEL_DIMS["micro"], 0)) == set(sd)


@pytest.mark.gpu
@pytest.mark.parametrize("in_memory", [False, True])
def test_load_model_from_reference_checkpoint(in_memory):
    import whisper
    from whisper import synthetic as S
    g = _golden()
    m = whisper.load_model(CKPT, device=0, dtype="fp32", max_windows=1, max_group=5, in_memory=in_memory)
    try:
        assert m.dims.n_text_state == g["dims"]["n_text_state"] and m.dims.n_vocab == g["dims"]["n_vocab"]
        audio = S.synthetic_audio(30.0, seed=g["audio_seed"])
        mel = whisper.log_mel_spectrogram(audio, m.dims.n_mels, padding=whisper.audio.N_SAMPLES)
        seg = whisper.pad_or_trim(mel[:, :3000], 3000)
        for key, case in g["cases"].items():
            res = whisper.decode(m, seg, whisper.DecodingOptions(language="en", **case["options"]))
            np.testing.assert_array_equal(np.asarray(res.tokens), case["tokens"], err_msg=key)
            assert res.avg_logprob == pytest.approx(case["avg_logprob"], abs=1e-3), key
            assert res.no_speech_prob == pytest.approx(case["no_speech_prob"], abs=1e-4), key
    finally:
        m.close()
