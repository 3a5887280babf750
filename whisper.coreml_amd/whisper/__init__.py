"""whisper — drop-in ``load_model()`` / ``transcribe()`` API on the MI355X HIP backend.

Mirrors the public surface of the reference package (whisper/__init__.py:102-179):
``available_models``, ``load_model``, ``transcribe``, ``decode``,
``DecodingOptions``, ``DecodingResult``, ``log_mel_spectrogram``, ``pad_or_trim``,
``load_audio``.  ``load_model(..., use_coreml=...)`` is accepted for call-site
compatibility and ignored: the compute backend is always libwhisper_hip.so.

There is no network: a model name resolves to ``<download_root>/<name>.pt``; a
missing checkpoint raises, as the reference's loader does without a download.
Seeded synthetic weights with the official dimensions (whisper/synthetic.py) are
opt-in: ``synthetic=True`` or ``WHISPER_HIP_SYNTHETIC=1``.  A path loads
``{"dims", "model_state_dict"}`` with ``torch.load(weights_only=True)``.
"""

import os
import warnings
from typing import List, Optional, Union

import numpy as np

from .audio import load_audio, log_mel_spectrogram, pad_or_trim
from .backend_hip import HipBackendError
from .decoding import DecodingOptions, DecodingResult, decode, detect_language
from .model import ModelDimensions, Whisper
from .synthetic import MODEL_DIMS, synthetic_state_dict
from .transcribe import transcribe

__version__ = "20240930+hip1"

# base85 alignment-head masks of the official checkpoints (reference __init__.py:39-55)
_ALIGNMENT_HEADS = {
    "tiny.en": b"ABzY8J1N>@0{>%R00Bk>$p{7v037`oCl~+#00",
    "tiny": b"ABzY8bu8Lr0{>%RKn9Fp%m@SkK7Kt=7ytkO",
    "base.en": b"ABzY8;40c<0{>%RzzG;p*o+Vo09|#PsxSZm00",
    "base": b"ABzY8KQ!870{>%RzyTQH3`Q^yNP!>##QT-<FaQ7m",
    "small.en": b"ABzY8>?_)10{>%RpeA61k&I|OI3I$65C{;;pbCHh0B{qLQ;+}v00",
    "small": b"ABzY8DmU6=0{>%Rpa?J`kvJ6qF(V^F86#Xh7JUGMK}P<N0000",
    "medium.en": b"ABzY8usPae0{>%R7<zz_OvQ{)4kMa0BMw6u5rT}kRKX;$NfYBv00*Hl@qhsU00",
    "medium": b"ABzY8B0Jh+0{>%R7}kK1fFL7w6%<-Pf*t^=N)Qr&0RR9",
    "large-v1": b"ABzY8r9j$a0{>%R7#4sLmoOs{s)o3~84-RPdcFk!JR<kSfC2yj",
    "large-v2": b"ABzY8zd+h!0{>%R7=D0pU<_bnWW*tkYAhobTNnu$jnkEkXqp)j;w1Tzk)UH3X%SZd&fFZ2fC2yj",
    "large-v3": b"ABzY8gWO1E0{>%R7(9S+Kn!D~%ngiGaR?*L!iJG9p-nab0JQ=-{D1-g00",
    "large": b"ABzY8gWO1E0{>%R7(9S+Kn!D~%ngiGaR?*L!iJG9p-nab0JQ=-{D1-g00",
    "large-v3-turbo": b"ABzY8j^C+e0{>%RARaKHP%t(lGR*)0g!tONPyhe`",
    "turbo": b"ABzY8j^C+e0{>%RARaKHP%t(lGR*)0g!tONPyhe`",
}


def available_models() -> List[str]:
    return list(_ALIGNMENT_HEADS.keys())


def _device_index(device) -> int:
    if device is None:
        return int(os.environ.get("LOCAL_RANK", 0))
    if isinstance(device, int):
        return device
    s = str(device)
    if s.startswith("cpu"):
        raise HipBackendError("device='cpu': this package runs Whisper on AMD GPUs only (no CPU fallback)")
    return int(s.split(":")[1]) if ":" in s else 0


def load_model(name: str, device: Optional[Union[str, int]] = None, download_root: Optional[str] = None,
               in_memory: bool = False, use_coreml: bool = False, *, dtype: str = "fp16", max_windows: int = 8,
               max_group: int = 5, synthetic: Optional[bool] = None, seed: int = 0) -> Whisper:
    """Load a model onto one MI355X (reference __init__.py:107-179)."""
    dev = _device_index(device)
    if download_root is None:
        default = os.path.join(os.path.expanduser("~"), ".cache")
        download_root = os.path.join(os.getenv("XDG_CACHE_HOME", default), "whisper")
    ckpt = None
    align = None
    if name in MODEL_DIMS:
        p = os.path.join(download_root, f"{name}.pt")
        if synthetic is None:
            synthetic = os.environ.get("WHISPER_HIP_SYNTHETIC", "0") == "1"
        if os.path.isfile(p) and not synthetic:
            ckpt = p
        elif not synthetic:
            raise RuntimeError(f"Model {name} not found in {download_root} (no network to download it; "
                               f"synthetic=True loads seeded random weights instead)")
        align = _ALIGNMENT_HEADS.get(name)
    elif os.path.isfile(name):
        ckpt = name
    else:
        raise RuntimeError(f"Model {name} not found; available models = {available_models()}")
    if ckpt is not None:
        import io
        import torch
        # the reference's loader (__init__.py:151-166): a released checkpoint is a torch.save'd
        # {"dims": dict, "model_state_dict": fp16 tensors}; loaded with weights_only=True (no
        # pickled code runs), optionally from bytes read up front (in_memory)
        if in_memory:
            with open(ckpt, "rb") as f:
                checkpoint = torch.load(io.BytesIO(f.read()), map_location="cpu", weights_only=True)
        else:
            checkpoint = torch.load(ckpt, map_location="cpu", weights_only=True)
        dims = ModelDimensions(**checkpoint["dims"])
        state = checkpoint["model_state_dict"]
    else:
        warnings.warn(f"{name!r}: seeded synthetic weights (seed={seed}), not a trained checkpoint")
        dims = ModelDimensions(**MODEL_DIMS[name])
        state = synthetic_state_dict(MODEL_DIMS[name], seed)
    model = Whisper(dims, name, device=dev, dtype=dtype, max_windows=max_windows, max_group=max_group)
    model.load_state_dict(state)
    del state
    if align is not None:
        model.set_alignment_heads(align)
    return model


__all__ = ["available_models", "load_model", "transcribe", "decode", "detect_language", "DecodingOptions",
           "DecodingResult", "log_mel_spectrogram", "pad_or_trim", "load_audio", "ModelDimensions", "Whisper",
           "HipBackendError"]
