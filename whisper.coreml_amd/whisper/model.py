"""Model container (reference whisper/model.py:18-135) backed by a HIP context.

The reference ``Whisper`` is an nn.Module holding the fork's encoder/decoder
(encoder.py, decoder.py); here the module is a thin host object: weights live
in HBM inside libwhisper_hip (loaded through ``wh_load_tensor`` with the
reference's state_dict names) and every forward pass runs there.
"""

import base64
import gzip
from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np

from .backend_hip import HipContext


@dataclass
class ModelDimensions:
    n_mels: int
    n_audio_ctx: int
    n_audio_state: int
    n_audio_head: int
    n_audio_layer: int
    n_vocab: int
    n_text_ctx: int
    n_text_state: int
    n_text_head: int
    n_text_layer: int


class Whisper:
    def __init__(self, dims: ModelDimensions, name: str = "", device: int = 0, dtype: str = "fp16",
                 max_windows: int = 8, max_group: int = 5):
        self.dims = dims
        self.name = name
        self.modelName = name
        self.device_index = device
        self.dtype = dtype
        self.ctx = HipContext(dims.__dict__, device=device, dtype=dtype, max_windows=max_windows,
                              max_group=max_group)
        # default alignment heads: last half of the decoder layers (model.py:51-56)
        heads = np.zeros((dims.n_text_layer, dims.n_text_head), dtype=bool)
        heads[dims.n_text_layer // 2:] = True
        self.alignment_heads = heads

    def load_state_dict(self, state_dict: Dict[str, np.ndarray]):
        for k, v in state_dict.items():
            if k in ("decoder.mask", "alignment_heads", "decoder.alignment_heads"):
                continue
            if hasattr(v, "detach"):
                v = v.detach().float().cpu().numpy()
            self.ctx.load_tensor(k, np.asarray(v, dtype=np.float32))
        self.ctx.finalize()
        from .audio import mel_filters
        self.ctx.set_mel_filters(self.dims.n_mels, mel_filters(None, self.dims.n_mels))

    def set_alignment_heads(self, dump: bytes):
        """model.py:70-78."""
        arr = np.frombuffer(gzip.decompress(base64.b85decode(dump)), dtype=bool).copy()
        self.alignment_heads = arr.reshape(self.dims.n_text_layer, self.dims.n_text_head)

    @property
    def device(self):
        return f"cuda:{self.device_index}"

    @property
    def is_multilingual(self):
        return self.dims.n_vocab >= 51865

    @property
    def num_languages(self):
        return self.dims.n_vocab - 51765 - int(self.is_multilingual)

    def close(self):
        self.ctx.close()

    _last_windows = ([], [])  # (seeks, sizes) of the windows in the encoder slots

    from .decoding import decode as decode  # noqa: E402
    from .decoding import detect_language as detect_language  # noqa: E402
    from .transcribe import transcribe as transcribe  # noqa: E402
