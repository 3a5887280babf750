"""The reference's ``Inference`` interface (whisper/decoding.py:127-204) over the
per-step C ABI, for a caller that keeps the reference's host decode loop
(``DecodingTask._main_loop``, decoding.py:707-737: logit filters and beam search in
Python, one library call per token).

``PyTorchInference`` of the reference runs the model itself or, with
``use_coreml``, calls ``decoder256Predict`` / ``decoder1Predict`` /
``rearrange_mkv`` of the CoreML library (coreml.h:15-31).  ``HipInference`` makes
the same three calls into libwhisper_hip: ``wh_prefill`` (first pass),
``wh_step`` (one token per row, logits back to the host) and ``wh_reorder_kv``
(the beam reorder, an index permutation on the device).  The production path
(``decoding.run_windows``) does not use it: there the loop itself runs on the
device inside one hipGraph per token.
"""

from typing import List, Optional, Sequence

import numpy as np


def _np(x) -> np.ndarray:
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    return np.asarray(x)


class HipInference:
    """Drop-in for ``PyTorchInference(model, initial_token_length)`` on windows already
    encoded into slots 0..n_audio-1 (``model.ctx.encode``).  Rows are
    ``w * group + b``, as the reference lays out ``tokens.repeat_interleave(n_group)``
    (decoding.py:761)."""

    def __init__(self, model, initial_token_length: int, group: int = 1, sot_index: int = 0):
        self.ctx = model.ctx
        self.V = model.dims.n_vocab
        self.initial_token_length = initial_token_length
        self.group = group
        self.sot_index = sot_index
        self._started = False

    def logits(self, tokens, audio_features=None):
        """Returns ``(logits [rows, n, V], None)`` like the fork's ``logits``
        (decoding.py:151-184).  The first call runs the first pass over all
        ``initial_token_length`` tokens; only the rows the loop reads are filled
        (positions ``sot_index`` and the last, decoding.py:719, 723), the others are NaN.
        Later calls take the last token of every row."""
        tok = _np(tokens).astype(np.int64)
        rows, n = tok.shape
        if rows % self.group:
            raise ValueError(f"{rows} rows are not a multiple of group {self.group}")
        if not self._started:
            if n != self.initial_token_length:
                raise ValueError("the first call must carry the initial tokens")
            n_win = rows // self.group
            init = [list(tok[w * self.group]) for w in range(n_win)]
            two = self.ctx.prefill(init, self.group, [self.sot_index] * n_win)
            out = np.full((rows, n, self.V), np.nan, dtype=np.float32)
            rep = np.repeat(two, self.group, axis=0)  # beams of a window share the first pass
            out[:, self.sot_index] = rep[:, 0]
            out[:, n - 1] = rep[:, 1]
            self._started = True
            return out, None
        n_win = rows // self.group
        lg = self.ctx.step(tok[:, -1], text_offsets=[n - 1] * n_win)
        return lg[:, None, :], None

    def rearrange_kv_cache(self, source_indices: Sequence[int]):
        src = [int(s) for s in source_indices]
        if src != list(range(len(src))):
            self.ctx.reorder_kv(src)

    def cleanup_caching(self):
        self._started = False
