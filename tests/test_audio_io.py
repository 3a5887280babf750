"""load_audio without ffmpeg (reference whisper/audio.py:25-62; its test
tests/test_audio.py).  tests/golden/jfk.flac is the reference's own test file
(44.1 kHz stereo 24-bit FLAC, a fixture copied as data).

CPU: the library's host FLAC reader is bit-exact (the MD5 of the unencoded samples
that STREAMINFO carries), load_audio's shape / level checks of the reference test,
WAV input, loud failures.  GPU: the reference test's mel checks (file vs array path,
dynamic range <= 2.0) and the GPU log-mel of the file against the oracle's.
The ffmpeg resampler itself is not reproduced (parity unpinned for 44.1 -> 16 kHz;
documented in load_audio)."""
import hashlib
import os
import wave

import numpy as np
import pytest

from conftest import GOLDEN

JFK = os.path.join(GOLDEN, "jfk.flac")


def _streaminfo_md5(data: bytes) -> str:
    assert data[:4] == b"fLaC"
    assert data[4] & 127 == 0  # STREAMINFO comes first
    return data[8 + 18:8 + 34].hex()


def test_flac_decode_bit_exact():
    from whisper.backend_hip import decode_flac
    data = open(JFK, "rb").read()
    pcm, rate, bps = decode_flac(data)
    assert (rate, bps, pcm.shape) == (44100, 24, (485100, 2))
    # FLAC's MD5 is over the interleaved samples, little-endian, bps/8 bytes each
    le = pcm.astype("<i4").view(np.uint8).reshape(-1, 4)[:, : bps // 8].tobytes()
    assert hashlib.md5(le).hexdigest() == _streaminfo_md5(data)


def test_flac_decode_rejects_bad_streams():
    from whisper.backend_hip import HipBackendError, decode_flac
    data = open(JFK, "rb").read()
    with pytest.raises(HipBackendError):
        decode_flac(b"RIFF" + data[4:])
    with pytest.raises(HipBackendError):
        decode_flac(data[:8400])  # cut inside the first frame


def test_load_audio_jfk():
    # reference tests/test_audio.py:9-13
    from whisper.audio import SAMPLE_RATE, load_audio
    audio = load_audio(JFK)
    assert audio.dtype == np.float32 and audio.ndim == 1
    assert SAMPLE_RATE * 10 < audio.shape[0] < SAMPLE_RATE * 12
    assert 0 < audio.std() < 1
    # 16-bit quantised as ffmpeg's s16le output
    assert np.array_equal(audio * 32768.0, np.round(audio * 32768.0))


def test_load_audio_wav_exact(tmp_path):
    from whisper.audio import load_audio
    rng = np.random.default_rng(0)
    pcm = rng.integers(-20000, 20000, size=(16000, 2), dtype=np.int16)
    p = str(tmp_path / "x.wav")
    with wave.open(p, "wb") as w:
        w.setnchannels(2)
        w.setsampwidth(2)
        w.setframerate(16000)
        w.writeframes(pcm.tobytes())
    got = load_audio(p)
    want = np.clip(np.round(pcm.astype(np.float64).mean(axis=1)), -32768, 32767) / 32768.0
    np.testing.assert_array_equal(got, want.astype(np.float32))


def test_load_audio_unsupported(tmp_path):
    from whisper.audio import load_audio
    p = tmp_path / "x.mp3"
    p.write_bytes(b"\x00" * 16)
    with pytest.raises(RuntimeError):
        load_audio(str(p))


@pytest.mark.gpu
def test_mel_from_file_matches_array():
    # reference tests/test_audio.py:15-19, on the GPU log-mel
    from whisper.audio import load_audio, log_mel_spectrogram
    audio = load_audio(JFK)
    mel_from_audio = log_mel_spectrogram(audio)
    mel_from_file = log_mel_spectrogram(JFK)
    assert np.allclose(mel_from_audio, mel_from_file)
    assert mel_from_audio.max() - mel_from_audio.min() <= 2.0


@pytest.mark.gpu
@pytest.mark.parametrize("n_mels", [80, 128])
def test_mel_of_jfk_vs_oracle(n_mels):
    from oracle import ref_whisper as R
    from whisper.audio import N_SAMPLES, load_audio, log_mel_spectrogram
    audio = load_audio(JFK)
    got = log_mel_spectrogram(audio, n_mels, padding=N_SAMPLES)
    ref = R.log_mel_spectrogram(audio, n_mels, padding=R.N_SAMPLES).numpy()
    assert got.shape == ref.shape
    assert float(np.abs(got - ref).max()) < 2e-3


@pytest.mark.gpu
def test_config1_tiny_en_greedy_on_jfk():
    """BASELINE config 1 (tiny.en greedy on tests/jfk.flac): transcribe() of the file
    on the GPU in fp32 gives the oracle's segment tokens on the same decoded audio
    (seeded synthetic tiny.en weights: no checkpoint ships)."""
    import whisper
    from oracle import ref_whisper as R
    from whisper import synthetic as S
    from whisper.audio import load_audio
    dims = S.MODEL_DIMS["tiny.en"]
    sd = S.synthetic_state_dict(dims, 0)
    m = whisper.Whisper(whisper.ModelDimensions(**dims), "tiny.en", device=0, dtype="fp32", max_windows=1,
                        max_group=5)
    m.load_state_dict(sd)
    try:
        res = whisper.transcribe(m, JFK, temperature=0.0, language="en")
    finally:
        m.close()
    ref = R.transcribe(R.OracleWhisper(dims, sd), load_audio(JFK))
    assert len(res["segments"]) == len(ref) >= 1
    assert [s["tokens"] for s in res["segments"]] == [s["tokens"] for s in ref]
