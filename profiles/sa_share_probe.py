"""Probe (round 5): is the late-context step self-attention bound by the bytes of its
K/V rows or by its per-wave round trips?  At 20 windows x beam 5, after advancing the
decode (step graphs) to several context lengths, time k_self_attn_qkv of every layer
(wh_time_stage 8) with the decode's ancestry, then with every row reading beam slot 0's
history (stage 9: the 5 beams of a (window, head) fetch identical rows — what an L2 that
deduplicated shared history rows perfectly would fetch).  If 9 is much faster than 8 the
kernel is byte-bound and beam-shared loads would pay; if equal, its round trips bound it.
    python profiles/sa_share_probe.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "whisper.coreml_amd"), REPO]
import whisper  # noqa: E402
from whisper import synthetic as S  # noqa: E402
from whisper.decoding import DecodingTask  # noqa: E402

W = 20
dims = S.MODEL_DIMS["large-v3"]
m = whisper.Whisper(whisper.ModelDimensions(**dims), "large-v3", device=0, dtype="fp16", max_windows=W, max_group=5)
m.load_state_dict(S.synthetic_state_dict(dims, 0))
m.ctx.log_mel(S.synthetic_audio(30.0 * W, seed=1000), dims["n_mels"], padding=whisper.audio.N_SAMPLES)
m.ctx.encode([3000 * i for i in range(W)], [3000] * W)
task = DecodingTask(m, whisper.DecodingOptions(language="en", beam_size=5))
m.ctx.decode_begin(task.wh_opts(), [task.initial_tokens] * W, [task.sot_index] * W)
done = 0
for target in (8, 50, 100, 150, 200):
    m.ctx.time_stage(0, target - done)  # advance (graph steps)
    done = target
    t8 = [m.ctx.time_stage(8, 3) for _ in range(3)]
    t9 = [m.ctx.time_stage(9, 3) for _ in range(3)]
    t8b = m.ctx.time_stage(8, 3)
    ctx_len = 4 + target
    logical = 100 * 20 * 2 * ctx_len * 64 * 2
    print(f"context ~{ctx_len:3d}: own ancestry {min(t8) * 1e3:6.2f} us ({t8b * 1e3:6.2f} after), "
          f"all beams on slot 0 {min(t9) * 1e3:6.2f} us; logical K/V {logical / 1e6:6.1f} MB "
          f"-> {logical / (min(t8) * 1e-3) / 1e12:5.2f} TB/s at own ancestry", flush=True)
m.close()
