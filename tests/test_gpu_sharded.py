"""Config 4 (large-v3, beam 5, 3600 s of audio over 8 GPUs) replayed on one GPU.

whisper/distributed.py runs each rank in two phases (prepare_shard: its mel frames and
their local max; run_shard: normalise with the all-reduced max, batched schedule over
its clips).  Here the eight ranks run in turn on one context: 120 clips, 15 windows per
rank — the per-rank batch of config 4 (75 decoder rows per step) — and the merged
segments are compared with the unsharded transcribe() of the same file on the same
context (batches of 20 windows).

Bar: identical segments (tokens, seeks, timestamps) in the production fp16 context.
That holds because a window's decoder step is batch-invariant for batches of >= 2
windows (DESIGN.md §2 "batch invariance"): every reduction a window's logits go
through is ordered by the model shape, never by how many windows share the batch.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SECONDS = 3600.0
WORLD = 8


@pytest.mark.parametrize("balance", ["clips", "tokens"])
def test_config4_sharded_replay_equals_unsharded(balance, dtype="fp16"):
    """balance "clips": contiguous 15-clip blocks; "tokens": every 8th clip per rank
    (bench.py --balance tokens), merged back into file order by window seek."""
    import whisper
    from conftest import full_model
    from whisper import distributed as D
    from whisper import synthetic as S
    m = full_model("large-v3", dtype)
    audio = S.synthetic_audio(SECONDS, seed=0)
    kw = dict(temperature=0.0, language="en", beam_size=5)
    states = [D.prepare_shard(m, audio, r, WORLD, balance) for r in range(WORLD)]
    assert [len(s.clips) for s in states] == [15] * WORLD
    g = max(s.local_max for s in states)
    per_rank = [D.run_shard(m, s, g, audio=audio, balance=balance, **kw) for s in states]
    merged = D.merge_segments(per_rank)
    ref = whisper.transcribe(m, audio, condition_on_previous_text=False,
                             clip_timestamps=D.seconds_csv(D.clip_grid(int(SECONDS * 100))), **kw)["segments"]
    print(f"config 4 replay ({balance}): {len(merged)} segments sharded, {len(ref)} unsharded")
    assert len(merged) == len(ref)
    assert [s["seek"] for s in merged] == [s["seek"] for s in ref]
    assert [s["tokens"] for s in merged] == [s["tokens"] for s in ref]
    np.testing.assert_array_equal([s["start"] for s in merged], [s["start"] for s in ref])
    np.testing.assert_array_equal([s["end"] for s in merged], [s["end"] for s in ref])
    np.testing.assert_array_equal([s["avg_logprob"] for s in merged], [s["avg_logprob"] for s in ref])
