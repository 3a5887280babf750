"""Seeded synthetic checkpoints and audio (no network, no downloaded weights).

There are no Whisper checkpoints on this machine or on the GPU box, so every
model used by tests and by ``bench.py`` is a *synthetic checkpoint*: a state
dict with the exact key set and shapes of the reference fork's model
(``/root/reference/whisper/model.py:31-68``, ``encoder.py:82-101``,
``decoder.py:131-170``), filled from a deterministic numpy generator.

The same function runs in the survey container (where the golden vectors are
produced by the reference) and on the GPU box (where the HIP path is checked
against them), so only the seed has to travel.  Each tensor gets its own
generator stream seeded by ``(seed, crc32(name))`` so the values do not depend
on iteration order.

Init (probe 8): Linear/Conv weights N(0, 1/fan_in), biases
N(0, 0.02^2), LayerNorm gamma = 1 + N(0, 0.05^2), beta N(0, 0.02^2), token /
positional embeddings N(0, 0.1^2).  This gives greedy top-2 logit margins far
above fp32 noise, which the token-for-token parity tests rely on.

This module is pure numpy on purpose: it is imported by file path from the
golden generator, which runs next to the reference's own ``whisper`` package.
"""

import zlib
from typing import Dict, Tuple

import numpy as np

# ModelDimensions of the official checkpoints (field order of
# reference whisper/model.py:18-29).  Head dim is 64 everywhere.
MODEL_DIMS: Dict[str, Dict[str, int]] = {
    "tiny.en": dict(n_mels=80, n_audio_ctx=1500, n_audio_state=384, n_audio_head=6, n_audio_layer=4,
                    n_vocab=51864, n_text_ctx=448, n_text_state=384, n_text_head=6, n_text_layer=4),
    "tiny": dict(n_mels=80, n_audio_ctx=1500, n_audio_state=384, n_audio_head=6, n_audio_layer=4,
                 n_vocab=51865, n_text_ctx=448, n_text_state=384, n_text_head=6, n_text_layer=4),
    "base.en": dict(n_mels=80, n_audio_ctx=1500, n_audio_state=512, n_audio_head=8, n_audio_layer=6,
                    n_vocab=51864, n_text_ctx=448, n_text_state=512, n_text_head=8, n_text_layer=6),
    "base": dict(n_mels=80, n_audio_ctx=1500, n_audio_state=512, n_audio_head=8, n_audio_layer=6,
                 n_vocab=51865, n_text_ctx=448, n_text_state=512, n_text_head=8, n_text_layer=6),
    "small.en": dict(n_mels=80, n_audio_ctx=1500, n_audio_state=768, n_audio_head=12, n_audio_layer=12,
                     n_vocab=51864, n_text_ctx=448, n_text_state=768, n_text_head=12, n_text_layer=12),
    "small": dict(n_mels=80, n_audio_ctx=1500, n_audio_state=768, n_audio_head=12, n_audio_layer=12,
                  n_vocab=51865, n_text_ctx=448, n_text_state=768, n_text_head=12, n_text_layer=12),
    "medium.en": dict(n_mels=80, n_audio_ctx=1500, n_audio_state=1024, n_audio_head=16, n_audio_layer=24,
                      n_vocab=51864, n_text_ctx=448, n_text_state=1024, n_text_head=16, n_text_layer=24),
    "medium": dict(n_mels=80, n_audio_ctx=1500, n_audio_state=1024, n_audio_head=16, n_audio_layer=24,
                   n_vocab=51865, n_text_ctx=448, n_text_state=1024, n_text_head=16, n_text_layer=24),
    "large-v1": dict(n_mels=80, n_audio_ctx=1500, n_audio_state=1280, n_audio_head=20, n_audio_layer=32,
                     n_vocab=51865, n_text_ctx=448, n_text_state=1280, n_text_head=20, n_text_layer=32),
    "large-v2": dict(n_mels=80, n_audio_ctx=1500, n_audio_state=1280, n_audio_head=20, n_audio_layer=32,
                     n_vocab=51865, n_text_ctx=448, n_text_state=1280, n_text_head=20, n_text_layer=32),
    "large-v3": dict(n_mels=128, n_audio_ctx=1500, n_audio_state=1280, n_audio_head=20, n_audio_layer=32,
                     n_vocab=51866, n_text_ctx=448, n_text_state=1280, n_text_head=20, n_text_layer=32),
    "large-v3-turbo": dict(n_mels=128, n_audio_ctx=1500, n_audio_state=1280, n_audio_head=20, n_audio_layer=32,
                           n_vocab=51866, n_text_ctx=448, n_text_state=1280, n_text_head=20, n_text_layer=4),
    # test-only shapes (not official): a micro model that the CPU oracle runs in seconds
    "micro": dict(n_mels=80, n_audio_ctx=1500, n_audio_state=128, n_audio_head=2, n_audio_layer=2,
                  n_vocab=51865, n_text_ctx=448, n_text_state=128, n_text_head=2, n_text_layer=2),
    "micro.en": dict(n_mels=80, n_audio_ctx=1500, n_audio_state=128, n_audio_head=2, n_audio_layer=2,
                     n_vocab=51864, n_text_ctx=448, n_text_state=128, n_text_head=2, n_text_layer=2),
}
MODEL_DIMS["large"] = MODEL_DIMS["large-v3"]
MODEL_DIMS["turbo"] = MODEL_DIMS["large-v3-turbo"]


def sinusoids(length: int, channels: int, max_timescale: float = 10000.0) -> np.ndarray:
    """Encoder positional embedding (reference encoder.py:10-16), float32."""
    assert channels % 2 == 0
    inc = np.log(max_timescale) / (channels // 2 - 1)
    # match torch: exp(-inc * arange) computed in float32
    inv = np.exp((-inc * np.arange(channels // 2, dtype=np.float32)).astype(np.float32)).astype(np.float32)
    t = np.arange(length, dtype=np.float32)[:, None] * inv[None, :]
    return np.concatenate([np.sin(t), np.cos(t)], axis=1).astype(np.float32)


def state_dict_shapes(d: Dict[str, int]) -> Dict[str, Tuple[int, ...]]:
    """Key -> shape for the fork's Whisper state dict (persistent entries only)."""
    na, nt = d["n_audio_state"], d["n_text_state"]
    s: Dict[str, Tuple[int, ...]] = {}
    s["encoder.conv1.weight"] = (na, d["n_mels"], 3)
    s["encoder.conv1.bias"] = (na,)
    s["encoder.conv2.weight"] = (na, na, 3)
    s["encoder.conv2.bias"] = (na,)
    s["encoder.positional_embedding"] = (d["n_audio_ctx"], na)

    def block(prefix: str, n: int, cross: bool):
        for att in (["attn", "cross_attn"] if cross else ["attn"]):
            s[f"{prefix}.{att}.query.weight"] = (n, n)
            s[f"{prefix}.{att}.query.bias"] = (n,)
            s[f"{prefix}.{att}.key.weight"] = (n, n)
            s[f"{prefix}.{att}.value.weight"] = (n, n)
            s[f"{prefix}.{att}.value.bias"] = (n,)
            s[f"{prefix}.{att}.out.weight"] = (n, n)
            s[f"{prefix}.{att}.out.bias"] = (n,)
            s[f"{prefix}.{att}_ln.weight"] = (n,)
            s[f"{prefix}.{att}_ln.bias"] = (n,)
        s[f"{prefix}.mlp.0.weight"] = (4 * n, n)
        s[f"{prefix}.mlp.0.bias"] = (4 * n,)
        s[f"{prefix}.mlp.2.weight"] = (n, 4 * n)
        s[f"{prefix}.mlp.2.bias"] = (n,)
        s[f"{prefix}.mlp_ln.weight"] = (n,)
        s[f"{prefix}.mlp_ln.bias"] = (n,)

    for i in range(d["n_audio_layer"]):
        block(f"encoder.blocks.{i}", na, False)
    s["encoder.ln_post.weight"] = (na,)
    s["encoder.ln_post.bias"] = (na,)
    s["decoder.token_embedding.weight"] = (d["n_vocab"], nt)
    s["decoder.positional_embedding"] = (d["n_text_ctx"], nt)
    for i in range(d["n_text_layer"]):
        block(f"decoder.blocks.{i}", nt, True)
    s["decoder.ln.weight"] = (nt,)
    s["decoder.ln.bias"] = (nt,)
    return s


def _tensor(name: str, shape: Tuple[int, ...], seed: int) -> np.ndarray:
    if name == "encoder.positional_embedding":
        return sinusoids(shape[0], shape[1])
    rng = np.random.default_rng([seed, zlib.crc32(name.encode())])
    if name.endswith("_ln.weight") or name.endswith("ln_post.weight") or name == "decoder.ln.weight":
        return (1.0 + 0.05 * rng.standard_normal(shape, dtype=np.float32)).astype(np.float32)
    if "embedding" in name:
        return (0.1 * rng.standard_normal(shape, dtype=np.float32)).astype(np.float32)
    if name.endswith(".bias"):
        return (0.02 * rng.standard_normal(shape, dtype=np.float32)).astype(np.float32)
    fan_in = int(np.prod(shape[1:]))
    return (rng.standard_normal(shape, dtype=np.float32) * np.float32(1.0 / np.sqrt(fan_in))).astype(np.float32)


def synthetic_state_dict(dims: Dict[str, int], seed: int = 0) -> Dict[str, np.ndarray]:
    """Checkpoint-format (un-prescaled) float32 state dict for ``dims``."""
    return {k: _tensor(k, shp, seed) for k, shp in state_dict_shapes(dims).items()}


def scale_eot_embedding(sd: Dict[str, np.ndarray], dims: Dict[str, int], scale: float) -> None:
    """Multiplies the EOT row of the decoder token embedding by ``scale`` in place (fp32).
    With the seeded random weights EOT never wins a natural decode; scaling its row (its
    logit is x . E[eot], reference decoder.py:319-320) makes candidates finish at many
    lengths — the test setting for patience / length_penalty (tests/golden/beam_options.json)."""
    eot = 50257 if dims["n_vocab"] >= 51865 else 50256
    E = sd["decoder.token_embedding.weight"]
    E[eot] = (E[eot] * np.float32(scale)).astype(np.float32)


def state_dict_checksum(sd: Dict[str, np.ndarray]) -> float:
    """Order-independent float64 checksum used to pin generator determinism."""
    tot = 0.0
    for k in sorted(sd):
        v = sd[k].astype(np.float64).ravel()
        tot += float(np.sum(v[::997])) + 1e-3 * float(np.sum(np.abs(v[::1009])))
    return tot


def synthetic_audio(seconds: float, seed: int = 0, sr: int = 16000, tone_hz: float = 440.0) -> np.ndarray:
    """Seeded 16 kHz float32 audio: N(0, 0.1^2) noise plus a 0.05-amplitude tone."""
    n = int(round(seconds * sr))
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(n, dtype=np.float32) * np.float32(0.1)
    if tone_hz:
        t = np.arange(n, dtype=np.float64) / sr
        x = x + (0.05 * np.sin(2 * np.pi * tone_hz * t)).astype(np.float32)
    return x.astype(np.float32)
