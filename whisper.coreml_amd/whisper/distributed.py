"""One file transcribed by several GPUs, one process per GPU.

Exact sharding holds for ``condition_on_previous_text=False`` on a 30 s
``clip_timestamps`` grid (transcribe.py:172-181): each clip's seek is clip-local
(transcribe.py:277-287) and the prompt resets every window (transcribe.py:513-515),
so a clip's segments depend only on its own mel frames and on one file-global
scalar, the log-mel maximum (audio.py:155).  Each rank therefore

1. takes a contiguous block of clips (``shard_clips``),
2. computes only the mel frames of its block from the resident audio
   (``wh_log_mel_frames``; the last rank also covers the 30 s zero tail the
   reference appends, audio.py:145-146, since the max runs over it),
3. all-reduces the local maximum (MAX) — the only collective on the data path,
4. normalises and runs the batched schedule over its clips,
5. sends its segment records to rank 0 (gather), which renumbers the ids.

The two phases are exposed separately (``prepare_shard`` / ``run_shard``) so one
GPU can replay several ranks in turn, which is how the tests check that a sharded
run equals the unsharded one.

Two options would carry state across a rank boundary, so ``run_shard`` rejects them
instead of diverging from the reference: ``word_timestamps`` (each window's first-word
truncation reads the running ``last_speech_timestamp`` of the windows before it,
timing.py:337 / transcribe.py:485-486) and ``initial_prompt`` (the reference gives it
to the first window that is not skipped as silence, transcribe.py:299-321, which a
rank cannot know before the earlier ranks have decoded).
"""
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

from .audio import HOP_LENGTH, N_FRAMES, N_SAMPLES, SAMPLE_RATE

FRAMES_PER_SECOND = SAMPLE_RATE // HOP_LENGTH  # 100


def clip_grid(content_frames: int, clip_frames: int = N_FRAMES) -> List[Tuple[int, int]]:
    """The 30 s clip grid over the content, as (start, end) frames."""
    return [(s, min(s + clip_frames, content_frames)) for s in range(0, max(content_frames, 1), clip_frames)]


def shard_clips(n_clips: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced block [c0, c1) of clip indices for ``rank``."""
    if not (0 <= rank < world):
        raise ValueError(f"rank {rank} outside world {world}")
    return n_clips * rank // world, n_clips * (rank + 1) // world


BALANCES = ("clips", "tokens")


def rank_clips(n_clips: int, world: int, rank: int, balance: str = "clips") -> List[int]:
    """Clip indices of ``rank``: a contiguous block (``balance="clips"``: equal clip
    counts, the fixed-work case) or every world-th clip (``"tokens"``: natural decoding,
    where a window's EOT ends its decode early and speech density drifts along a file,
    so interleaved clips spread the long windows over the ranks)."""
    if balance == "clips":
        c0, c1 = shard_clips(n_clips, world, rank)
        return list(range(c0, c1))
    if balance == "tokens":
        if not (0 <= rank < world):
            raise ValueError(f"rank {rank} outside world {world}")
        return list(range(rank, n_clips, world))
    raise ValueError(f"balance must be one of {BALANCES}, not {balance!r}")


def mel_frame_range(clips: Sequence[Tuple[int, int]], c0: int, c1: int, total_frames: int,
                    last: bool) -> Tuple[int, int]:
    """(frame0, count) of mel frames rank needs: its clips, plus — for the last rank —
    every frame to the end of the padded file so the global max covers them all.
    (Interleaved clips: c0 / c1 - 1 are the rank's first / last clip; the span covers the
    clips between them, which other ranks decode — the log-mel is ~0.4 % of a window's
    time, and MAX over overlapping spans is still the file's maximum.)"""
    if c1 <= c0:
        return 0, 0
    f0 = clips[c0][0]
    f1 = total_frames if last else clips[c1 - 1][1]
    return f0, f1 - f0


def seconds_csv(clips: Sequence[Tuple[int, int]]) -> str:
    return ",".join(f"{s / FRAMES_PER_SECOND:.2f},{e / FRAMES_PER_SECOND:.2f}" for s, e in clips)


@dataclass
class ShardState:
    rank: int
    world: int
    n_samples: int
    total_frames: int
    clips: List[Tuple[int, int]]          # this rank's clips (absolute frames)
    frame0: int
    count: int
    local_max: float                      # -inf when the rank holds no frames


def prepare_shard(model, audio, rank: int, world: int, balance: str = "clips") -> ShardState:
    """Phase 1: this rank's mel frames and their (un-normalised) maximum."""
    from .backend_hip import DeviceAudio
    import numpy as np
    ctx = model.ctx
    n_mels = model.dims.n_mels
    if isinstance(audio, DeviceAudio):
        n, host = audio.n_samples, None
    else:
        host = np.ascontiguousarray(audio, dtype=np.float32)
        n = host.shape[0]
    total = (n + N_SAMPLES) // HOP_LENGTH
    content = total - N_FRAMES
    grid = clip_grid(content)
    mine = rank_clips(len(grid), world, rank, balance)
    # the rank that decodes the file's last clip also covers the padded tail (audio.py:145-146)
    holds_last = bool(mine) and mine[-1] == len(grid) - 1
    f0, cnt = mel_frame_range(grid, mine[0], mine[-1] + 1, total, last=holds_last) if mine else (0, 0)
    local_max = float("-inf")
    if cnt > 0:
        ctx.log_mel_frames(host, n, n_mels, f0, cnt, padding=N_SAMPLES, normalize=False)
        local_max = ctx.mel_max()
    return ShardState(rank, world, n, total, [grid[c] for c in mine], f0, cnt, local_max)


def run_shard(model, state: ShardState, global_max: float, audio=None, balance: str = "clips",
              **transcribe_kw) -> List[dict]:
    """Phase 2: normalise with the global max and transcribe this rank's clips
    (batched schedule).  ``audio`` re-supplies host audio when the context's mel
    buffer was reused by another shard since ``prepare_shard``."""
    from .transcribe import transcribe
    for key in ("word_timestamps", "initial_prompt", "carry_initial_prompt"):
        if transcribe_kw.get(key):
            raise ValueError(f"sharded transcription does not support {key} (it carries state across windows)")
    if not state.clips:
        return []
    if audio is not None:
        prepare_again = prepare_shard(model, audio, state.rank, state.world, balance)
        assert prepare_again.frame0 == state.frame0 and prepare_again.count == state.count
    model.ctx.mel_normalize(global_max)
    kw = dict(transcribe_kw)
    kw.update(condition_on_previous_text=False, clip_timestamps=seconds_csv(state.clips), schedule="batched")
    out = transcribe(model, None, _mel_prepared=(state.total_frames, state.frame0, state.count), **kw)
    return out["segments"]


def merge_segments(per_rank: Sequence[Sequence[dict]]) -> List[dict]:
    """The ranks' segments in file order with ids renumbered (transcribe.py:468-480): a
    stable sort by window seek, so interleaved clips (balance "tokens") come back in clip
    order and a window's segments keep their order (contiguous blocks are already sorted)."""
    flat = [s for segs in per_rank for s in segs]
    flat.sort(key=lambda s: s["seek"])
    return [{**s, "id": i} for i, s in enumerate(flat)]


def global_max(local: float, group=None) -> float:
    """All-reduce MAX of the local log-mel maximum (RCCL on GPU tensors, gloo on CPU)."""
    import torch
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([local], dtype=torch.float32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def gather_segments(segments: List[dict], group=None, dst: int = 0) -> Optional[List[dict]]:
    """Segment records of every rank to ``dst`` (a few KB per window)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    bucket = [None] * world if rank == dst else None
    dist.gather_object(segments, bucket, dst=dst, group=group)
    return merge_segments(bucket) if rank == dst else None


def transcribe_sharded(model, audio, group=None, reduce_max: Optional[Callable[[float], float]] = None,
                       **transcribe_kw) -> Optional[dict]:
    """``transcribe()`` of one file over the ranks of ``group`` (torch.distributed
    initialised by the caller; backend "nccl" = RCCL).  Returns the merged result on
    rank 0 and None elsewhere."""
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    st = prepare_shard(model, audio, rank, world)
    g = (reduce_max or (lambda x: global_max(x, group)))(st.local_max)
    segs = run_shard(model, st, g, **transcribe_kw)
    merged = gather_segments(segs, group)
    if merged is None:
        return None
    return {"segments": merged, "language": transcribe_kw.get("language")}
