"""Host logic of the multi-GPU path (whisper/distributed.py) on CPU: clip sharding,
mel frame ranges, and the two collectives (all-reduce MAX of the log-mel maximum,
gather of segment records) over gloo with world size 2."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from whisper import distributed as D
from whisper.audio import HOP_LENGTH, N_FRAMES, N_SAMPLES


@pytest.mark.parametrize("seconds", [1.0, 29.99, 30.0, 65.0, 600.0, 3600.0])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shards_cover_every_clip_and_frame_once(seconds, world):
    n = int(seconds * 16000)
    total = (n + N_SAMPLES) // HOP_LENGTH
    content = total - N_FRAMES
    grid = D.clip_grid(content)
    assert grid[0][0] == 0 and grid[-1][1] == content
    assert all(a[1] == b[0] for a, b in zip(grid, grid[1:]))
    seen_clips, covered = [], []
    for r in range(world):
        c0, c1 = D.shard_clips(len(grid), world, r)
        seen_clips += list(range(c0, c1))
        f0, cnt = D.mel_frame_range(grid, c0, c1, total, last=r == world - 1)
        if cnt:
            covered.append((f0, f0 + cnt))
            # the rank holds every frame its windows read
            for s, e in grid[c0:c1]:
                assert f0 <= s and e <= f0 + cnt
    assert seen_clips == list(range(len(grid)))
    # frames of all ranks tile [0, total) — the global max sees every frame
    covered.sort()
    assert covered[0][0] == 0 and covered[-1][1] == total
    assert all(a[1] == b[0] for a, b in zip(covered, covered[1:]))


@pytest.mark.parametrize("seconds", [1.0, 65.0, 600.0, 3600.0])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("balance", D.BALANCES)
def test_rank_clips_partition_and_frames(seconds, world, balance):
    """Both balances deal every clip to exactly one rank; each rank's mel span holds its
    clips, and the rank holding the last clip covers the padded tail (the max sees it)."""
    n = int(seconds * 16000)
    total = (n + N_SAMPLES) // HOP_LENGTH
    grid = D.clip_grid(total - N_FRAMES)
    dealt = []
    spans = []
    for r in range(world):
        mine = D.rank_clips(len(grid), world, r, balance)
        assert mine == sorted(mine)
        dealt += mine
        if mine:
            f0, cnt = D.mel_frame_range(grid, mine[0], mine[-1] + 1, total, last=mine[-1] == len(grid) - 1)
            spans.append((f0, f0 + cnt))
            assert all(f0 <= grid[c][0] and grid[c][1] <= f0 + cnt for c in mine)
    assert sorted(dealt) == list(range(len(grid)))
    if balance == "tokens":
        assert all(len(D.rank_clips(len(grid), world, r, balance)) in (len(grid) // world, -(-len(grid) // world))
                   for r in range(world))
    assert max(e for _, e in spans) == total and min(s for s, _ in spans) == 0


def test_merge_interleaved_ranks_in_file_order():
    a = [{"id": 0, "seek": 0}, {"id": 1, "seek": 0, "x": 1}, {"id": 2, "seek": 6000}]
    b = [{"id": 0, "seek": 3000}, {"id": 1, "seek": 9000}]
    m = D.merge_segments([a, b])
    assert [s["seek"] for s in m] == [0, 0, 3000, 6000, 9000] and [s["id"] for s in m] == list(range(5))
    assert m[1].get("x") == 1  # a window's segments keep their order


def test_seconds_csv_round_trips_to_frames():
    grid = D.clip_grid(6500)
    ts = [float(x) for x in D.seconds_csv(grid).split(",")]
    assert [round(t * 100) for t in ts] == [f for c in grid for f in c]


def test_merge_renumbers_in_rank_order():
    a = [{"id": 0, "seek": 0}, {"id": 1, "seek": 0}]
    b = [{"id": 0, "seek": 3000}]
    m = D.merge_segments([a, [], b])
    assert [s["id"] for s in m] == [0, 1, 2] and [s["seek"] for s in m] == [0, 0, 3000]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = D.global_max([-3.5, 1.25][rank])
        segs = [{"id": i, "seek": 3000 * rank, "tokens": [rank, i]} for i in range(rank + 1)]
        merged = D.gather_segments(segs)
        q.put((rank, g, merged))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_collectives():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict()
    for _ in procs:
        r, g, merged = q.get(timeout=120)
        out[r] = (g, merged)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0][0] == out[1][0] == 1.25
    assert out[1][1] is None
    assert [s["id"] for s in out[0][1]] == [0, 1, 2]
    assert [s["tokens"] for s in out[0][1]] == [[0, 0], [1, 0], [1, 1]]


@pytest.mark.parametrize("opt", [dict(word_timestamps=True), dict(initial_prompt="hello"),
                                 dict(carry_initial_prompt=True)])
def test_run_shard_rejects_cross_window_state(opt):
    """Options whose reference semantics carry state from window to window across a
    rank boundary are refused rather than silently diverging (distributed.py header)."""
    st = D.ShardState(rank=1, world=2, n_samples=0, total_frames=0, clips=[(0, 3000)], frame0=0, count=0,
                      local_max=0.0)
    with pytest.raises(ValueError):
        D.run_shard(object(), st, 0.0, language="en", **opt)
