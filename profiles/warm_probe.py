"""Probe: how much would Infinity-Cache residency (256 MiB L3) buy the step's two
dominant kernels?  Times k_cross_attn1 and the six k_proj projections at the bench
batch (20 windows x beam 5, large-v3 fp16) over all 32 layers (operands HBM-cold,
as in the step: wh_time_stage 2/3) and on layer 0 repeated (operands L3-warm:
wh_time_stage 5/6).
    python profiles/warm_probe.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "whisper.coreml_amd"))

import whisper  # noqa: E402
from whisper import synthetic as S  # noqa: E402
from whisper.decoding import DecodingTask  # noqa: E402

dims = S.MODEL_DIMS["large-v3"]
sd = S.synthetic_state_dict(dims, 0)
audio = S.synthetic_audio(600.0, seed=1000)
nwin = 20
m = whisper.Whisper(whisper.ModelDimensions(**dims), "large-v3", device=0, dtype="fp16", max_windows=nwin,
                    max_group=5)
m.load_state_dict(sd)
m.ctx.log_mel(audio, dims["n_mels"], padding=480000)
m.ctx.encode([3000 * i for i in range(nwin)], [3000] * nwin)
task = DecodingTask(m, whisper.DecodingOptions(language="en", beam_size=5, suppress_tokens="-1,50257"))
m.ctx.decode_begin(task.wh_opts(), [task.initial_tokens] * nwin, [task.sot_index] * nwin)
for what, name in ((7, "k_proj in-step"), (2, "k_proj cold"), (5, "k_proj L3-warm"), (3, "k_cross_attn1 cold"),
                   (6, "k_cross_attn1 L3-warm")):
    m.ctx.time_stage(what, 1)
    print(f"{name:24s} {m.ctx.time_stage(what, 5) * 1e3:8.2f} us/launch", flush=True)
print(f"step graph               {m.ctx.time_stage(0, 20):8.3f} ms", flush=True)
