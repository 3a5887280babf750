"""Per-kernel-family timings at one decode batch via wh_time_stage (events around back-to-back
launches): 0 = step graph, 2 = the six projections of every layer (per launch), 3 = cross-
attention (per launch), 4 = token selection alone (k_logit_part + k_logit_combine).
  python3 profiles/stage_probe.py [model] [windows]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "whisper.coreml_amd"), REPO]

import whisper  # noqa: E402
from whisper import synthetic as S  # noqa: E402
from whisper.decoding import DecodingTask  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "turbo"
nwin = int(sys.argv[2]) if len(sys.argv) > 2 else 1
dims = S.MODEL_DIMS[name]
m = whisper.Whisper(whisper.ModelDimensions(**dims), name, device=0, dtype="fp16", max_windows=max(nwin, 1), max_group=5)
m.load_state_dict(S.synthetic_state_dict(dims, 0))
audio = S.synthetic_audio(30.0 * nwin, seed=1000)
m.ctx.log_mel(audio, dims["n_mels"], padding=whisper.audio.N_SAMPLES)
m.ctx.encode([3000 * i for i in range(nwin)], [3000] * nwin)
task = DecodingTask(m, whisper.DecodingOptions(language="en", beam_size=5))
m.ctx.decode_begin(task.wh_opts(), [task.initial_tokens] * nwin, [task.sot_index] * nwin)
for st, what in ((0, "step graph"), (2, "projection (avg of 6)"), (3, "cross-attention"), (4, "token selection")):
    m.ctx.time_stage(st, 3)
    print(f"{name} {nwin} win  {what:24s} {m.ctx.time_stage(st, 20) * 1e3:8.1f} us")
