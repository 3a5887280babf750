"""Probe (round 5): how much of a 100-row split-K projection's time is its weights' HBM
latency?  wh_time_stage 2 runs the six projections of every layer back to back (weights
from HBM: 32 layers x 46 MB do not fit the 256 MB Infinity Cache); stage 5 repeats layer
0's six (weights Infinity-Cache / L2 warm).  Per-launch us, 20 windows x beam 5.
    python profiles/warm_proj_probe.py
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
m.ctx.time_stage(0, 2)
for rep in range(3):
    cold = m.ctx.time_stage(2, 3)
    warm = m.ctx.time_stage(5, 3)
    xc = m.ctx.time_stage(3, 3)
    xw = m.ctx.time_stage(6, 3)
    print(f"k_proj per launch: HBM-cold {cold * 1e3:6.2f} us, layer-0 warm {warm * 1e3:6.2f} us; "
          f"k_xattn_seg: cold {xc * 1e3:6.2f} us, warm {xw * 1e3:6.2f} us", flush=True)
m.close()
