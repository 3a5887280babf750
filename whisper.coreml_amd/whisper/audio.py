"""Audio front end (reference whisper/audio.py:13-157), computed on the GPU.

``log_mel_spectrogram`` keeps the reference signature and semantics (right zero
padding, centred reflect-padded 400-point periodic-Hann STFT at hop 160, last
frame dropped, |X|^2, Slaney mel projection, log10 clamp, floor at max-8,
(x+4)/4) but the work runs in the HIP kernel ``k_mel_frames`` of
libwhisper_hip; the returned array is a host copy.  There is no CPU path.
"""

import os
import wave
from functools import lru_cache
from typing import Optional, Union

import numpy as np

SAMPLE_RATE = 16000
N_FFT = 400
HOP_LENGTH = 160
CHUNK_LENGTH = 30
N_SAMPLES = CHUNK_LENGTH * SAMPLE_RATE  # 480000
N_FRAMES = N_SAMPLES // HOP_LENGTH  # 3000
N_SAMPLES_PER_TOKEN = HOP_LENGTH * 2
FRAMES_PER_SECOND = SAMPLE_RATE // HOP_LENGTH  # 100
TOKENS_PER_SECOND = SAMPLE_RATE // N_SAMPLES_PER_TOKEN  # 50


def load_audio(file: str, sr: int = SAMPLE_RATE) -> np.ndarray:
    """Mono float32 waveform at ``sr`` (audio.py:25-62).  The reference pipes the file
    through the ffmpeg CLI (``-ac 1 -ar sr -f s16le``), which neither this image nor
    the GPU box has.  Here: FLAC is decoded by the library's host FLAC reader
    (bit-exact, ``wh_flac_decode``) and 16-bit PCM WAV by ``wave``; then, as ffmpeg's
    command line asks, channels are averaged to mono, the rate is converted to ``sr``
    (polyphase FIR, ``scipy.signal.resample_poly``) and the result is quantised to
    16-bit PCM and scaled by 1/32768.  ffmpeg's own resampling filter is not
    reproduced, so samples differ from the reference's in the low bits wherever the
    file's rate is not ``sr`` (parity unpinned there; exact for 16-bit files at ``sr``)."""
    low = file.lower()
    if low.endswith(".flac"):
        from .backend_hip import decode_flac
        with open(file, "rb") as f:
            pcm, rate, bps = decode_flac(f.read())
        x = pcm.astype(np.float64) / float(1 << (bps - 1))
    elif low.endswith(".wav"):
        with wave.open(file, "rb") as w:
            if w.getsampwidth() != 2:
                raise RuntimeError(f"Failed to load audio: {file}: need 16-bit PCM WAV")
            rate = w.getframerate()
            x = np.frombuffer(w.readframes(w.getnframes()), np.int16).reshape(-1, w.getnchannels())
            x = x.astype(np.float64) / 32768.0
    else:
        raise RuntimeError(f"Failed to load audio: {file}: only .flac and 16-bit PCM .wav are supported without ffmpeg")
    x = x.mean(axis=1)
    if rate != sr:
        from math import gcd
        from scipy.signal import resample_poly
        g = gcd(int(rate), int(sr))
        x = resample_poly(x, sr // g, rate // g)
    pcm16 = np.clip(np.round(x * 32768.0), -32768, 32767).astype(np.int16)
    return pcm16.astype(np.float32) / 32768.0


def pad_or_trim(array, length: int = N_SAMPLES, *, axis: int = -1):
    """audio.py:65-88 (numpy arrays; torch tensors are accepted and converted)."""
    if hasattr(array, "numpy") and not isinstance(array, np.ndarray):
        array = array.detach().cpu().numpy()
    if array.shape[axis] > length:
        array = array.take(indices=range(length), axis=axis)
    if array.shape[axis] < length:
        pad = [(0, 0)] * array.ndim
        pad[axis] = (0, length - array.shape[axis])
        array = np.pad(array, pad)
    return array


def _hz_to_mel(f):
    f = np.asarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-10) / min_log_hz) / logstep, mels)


def _mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)


@lru_cache(maxsize=None)
def mel_filters(device=None, n_mels: int = 80) -> np.ndarray:
    """Slaney-normalised mel filterbank [n_mels][201] — the values the reference
    loads from assets/mel_filters.npz (audio.py:91-107, librosa.filters.mel with
    sr=16000, n_fft=400), re-derived here and pinned to the reference values by tests/test_audio_mel.py."""
    assert n_mels in {80, 128}, f"Unsupported n_mels: {n_mels}"
    fft_freqs = np.linspace(0, SAMPLE_RATE / 2, 1 + N_FFT // 2)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(0.0), _hz_to_mel(SAMPLE_RATE / 2), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fft_freqs[None, :]
    lower = -ramps[:-2] / fdiff[:-1, None]
    upper = ramps[2:] / fdiff[1:, None]
    w = np.maximum(0.0, np.minimum(lower, upper))
    w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    return w.astype(np.float32)


_mel_ctx = {}


def _mel_context(device: int):
    """A small HIP context used only for the free function ``log_mel_spectrogram``
    (a loaded model uses its own context)."""
    from .backend_hip import HipContext
    if device not in _mel_ctx:
        dims = dict(n_mels=80, n_audio_ctx=1500, n_audio_state=128, n_audio_head=2, n_audio_layer=1,
                    n_vocab=64, n_text_ctx=448, n_text_state=128, n_text_head=2, n_text_layer=1)
        ctx = HipContext(dims, device=device, dtype="fp32", max_windows=1, max_group=1)
        for nm in (80, 128):
            ctx.set_mel_filters(nm, mel_filters(None, nm))
        _mel_ctx[device] = ctx
    return _mel_ctx[device]


def _device_index(device) -> int:
    if device is None:
        return 0
    if isinstance(device, int):
        return device
    s = str(device)
    if s.startswith("cpu"):
        raise RuntimeError("the whisper HIP backend computes on an AMD GPU only (device='cpu' is not supported)")
    return int(s.split(":")[1]) if ":" in s else 0


def log_mel_spectrogram(audio: Union[str, np.ndarray], n_mels: int = 80, padding: int = 0,
                        device: Optional[Union[str, int]] = None, *, ctx=None) -> np.ndarray:
    """audio.py:110-157 on the GPU; returns float32 (n_mels, n_frames)."""
    if isinstance(audio, str):
        audio = load_audio(audio)
    if hasattr(audio, "numpy") and not isinstance(audio, np.ndarray):
        audio = audio.detach().cpu().numpy()
    audio = np.ascontiguousarray(audio, dtype=np.float32)
    c = ctx if ctx is not None else _mel_context(_device_index(device))
    nf = c.log_mel(audio, n_mels, padding, normalize=True)
    return c.mel_read(n_mels, 0, nf)
