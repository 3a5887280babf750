"""CPU restatement of the reference's word-timestamp numerics — TEST INFRASTRUCTURE ONLY.

Restates /root/reference/whisper/timing.py (the fork runs it on CPU: numba
``dtw_cpu`` on ``x.double()``, torch ``median_filter``) from reading it, not
copied.  Used by tests/ as the checker of csrc/wh_align.hip (wh_align / wh_dtw)
and by tests/test_oracle.py, which pins it against the reference's own outputs in
tests/golden/dtw.npz (planted-path DTW known answers as in the reference's
tests/test_timing.py, random DTW paths, median filters of several shapes/widths).
"""

from typing import List, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

TOKENS_PER_SECOND = 50  # audio.py:21-23


def median_filter(x: torch.Tensor, filter_width: int) -> torch.Tensor:
    """timing.py:19-54 (the CPU branch): reflect padding, median along the last dim."""
    pad_width = filter_width // 2
    if x.shape[-1] <= pad_width:
        return x
    ndim = x.ndim
    if ndim <= 2:
        x = x[None, None, :]
    x = F.pad(x, (pad_width, pad_width, 0, 0), mode="reflect")
    result = x.unfold(-1, filter_width, 1).sort()[0][..., pad_width]
    if ndim <= 2:
        result = result[0, 0]
    return result


def backtrace(trace: np.ndarray) -> np.ndarray:
    """timing.py:57-79."""
    i = trace.shape[0] - 1
    j = trace.shape[1] - 1
    trace[0, :] = 2
    trace[:, 0] = 1
    out = []
    while i > 0 or j > 0:
        out.append((i - 1, j - 1))
        t = trace[i, j]
        if t == 0:
            i -= 1
            j -= 1
        elif t == 1:
            i -= 1
        elif t == 2:
            j -= 1
        else:
            raise ValueError("unexpected trace value")
    return np.array(out)[::-1, :].T


def dtw_cpu(x: np.ndarray) -> np.ndarray:
    """timing.py:82-105: float64 input, float32 cost cells, ties -> the else branch.
    Vectorised over anti-diagonals (cell (i, j) needs diagonals d-1 and d-2 only),
    which leaves every cell's arithmetic and comparison unchanged."""
    x = np.asarray(x, dtype=np.float64)
    N, M = x.shape
    cost = np.full((N + 1, M + 1), np.inf, dtype=np.float32)
    trace = -np.ones((N + 1, M + 1), dtype=np.float32)
    cost[0, 0] = 0
    for d in range(2, N + M + 1):
        i = np.arange(max(1, d - M), min(N, d - 1) + 1)
        if len(i) == 0:
            continue
        j = d - i
        c0 = cost[i - 1, j - 1]
        c1 = cost[i - 1, j]
        c2 = cost[i, j - 1]
        t = np.where((c0 < c1) & (c0 < c2), 0, np.where((c1 < c0) & (c1 < c2), 1, 2))
        c = np.where(t == 0, c0, np.where(t == 1, c1, c2))
        cost[i, j] = (x[i - 1, j - 1] + c.astype(np.float64)).astype(np.float32)
        trace[i, j] = t
    return backtrace(trace)


def alignment_matrix(cross_qk: torch.Tensor, num_frames: int, n_sot: int, medfilt_width: int = 7,
                     qk_scale: float = 1.0) -> torch.Tensor:
    """timing.py:196-205: heads x tokens x frames -> the head-mean matrix rows
    [n_sot, -1)."""
    weights = cross_qk[:, :, : num_frames // 2]
    weights = (weights * qk_scale).softmax(dim=-1)
    std, mean = torch.std_mean(weights, dim=-2, keepdim=True, unbiased=False)
    weights = (weights - mean) / std
    weights = median_filter(weights, medfilt_width)
    matrix = weights.mean(axis=0)
    return matrix[n_sot:-1]


def find_alignment_path(model, sot_sequence: Sequence[int], no_timestamps: int, eot: int,
                        text_tokens: List[int], num_frames: int, medfilt_width: int = 7
                        ) -> Tuple[np.ndarray, np.ndarray, np.ndarray, torch.Tensor]:
    """timing.py:174-206 with the oracle model (audio already set): returns
    (text_token_probs, text_indices, time_indices, matrix)."""
    tokens = torch.tensor([[*sot_sequence, no_timestamps, *text_tokens, eot]])
    with torch.no_grad():
        logits, _, cross_qk = model.decoder_forward(tokens, 0, None)
    logits = logits[0]
    sampled = logits[len(sot_sequence):, :eot]
    probs = sampled.softmax(dim=-1)
    text_token_probs = probs[np.arange(len(text_tokens)), text_tokens].numpy()
    matrix = alignment_matrix(cross_qk, num_frames, len(sot_sequence), medfilt_width)
    text_indices, time_indices = dtw_cpu((-matrix).double().numpy())
    return text_token_probs, text_indices, time_indices, matrix
