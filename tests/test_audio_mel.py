"""Log-mel front end against the reference's own outputs (tests/golden/mel.npz,
written by oracle/gen_golden.py from /root/reference/whisper/audio.py:91-157).

CPU: the re-derived Slaney filterbank (whisper.audio.mel_filters) equals the
reference's mel_filters.npz values (filters_80 / filters_128).
GPU: k_mel_frames + k_mel_norm on all six reference cases — 1 s / 2 s / 0.5 s without
padding, 30 s / 31.5 s with the 30 s right pad, and the bench's 600 s / 128-mel file —
frame counts exact, the global max (audio.py:155, the whole padded file) within
1e-5, stored column slices within 2e-3 absolute (fp32 direct DFT vs pocketfft
rounding, amplified near the 1e-10 log clamp) and per-frame column sums within 1e-3
relative."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN


@pytest.fixture(scope="module")
def mel_golden():
    return np.load(os.path.join(GOLDEN, "mel.npz"))


@pytest.mark.parametrize("n_mels", [80, 128])
def test_mel_filters_equal_reference(mel_golden, n_mels):
    from whisper.audio import mel_filters
    got = mel_filters(None, n_mels)
    ref = mel_golden[f"filters_{n_mels}"]
    assert got.shape == ref.shape == (n_mels, 201)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-8)


CASES = ["a", "b", "c", "d", "e", "f"]


@pytest.mark.gpu
@pytest.mark.parametrize("tag", CASES)
def test_gpu_mel_matches_reference(mel_golden, tag):
    import whisper
    from whisper import synthetic as S
    meta = {m["tag"]: m for m in json.loads(str(mel_golden["meta"]))}[tag]
    audio = S.synthetic_audio(meta["seconds"], seed=meta["seed"])
    got = whisper.log_mel_spectrogram(audio, meta["n_mels"], padding=meta["padding"])
    assert got.shape == (meta["n_mels"], meta["frames"])
    assert float(got.max()) == pytest.approx(float(mel_golden[f"{tag}_max"]), abs=1e-5)
    n = 0
    for key in mel_golden.files:
        if key == f"{tag}_full":
            ref, lo = mel_golden[key], 0
        elif key.startswith(f"{tag}_") and key[len(tag) + 1:].isdigit():
            ref, lo = mel_golden[key], int(key[len(tag) + 1:])
        else:
            continue
        err = float(np.abs(got[:, lo:lo + ref.shape[1]] - ref).max())
        assert err < 2e-3, f"{key}: max abs err {err}"
        n += 1
    assert n >= 1
    cs = got.astype(np.float64).sum(axis=0)
    np.testing.assert_allclose(cs, mel_golden[f"{tag}_colsum"], rtol=1e-3, atol=1e-3)
    assert float(got.astype(np.float64).sum()) == pytest.approx(float(mel_golden[f"{tag}_sum"]), rel=2e-5)
