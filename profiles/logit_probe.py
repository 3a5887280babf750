"""Time k_logit_rows alone (wh_time_stage 4) at the bench batch (20 windows x beam 5)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "whisper.coreml_amd"))
import whisper  # noqa: E402
from whisper import synthetic as S  # noqa: E402
from whisper.decoding import DecodingTask  # noqa: E402

dims = S.MODEL_DIMS["large-v3"]
m = whisper.Whisper(whisper.ModelDimensions(**dims), "large-v3", device=0, dtype="fp16", max_windows=20, max_group=5)
m.load_state_dict(S.synthetic_state_dict(dims, 0))
m.ctx.log_mel(S.synthetic_audio(600.0, seed=1000), dims["n_mels"], padding=480000)
m.ctx.encode([3000 * i for i in range(20)], [3000] * 20)
for ts in (True, False):
    task = DecodingTask(m, whisper.DecodingOptions(language="en", beam_size=5, without_timestamps=not ts))
    m.ctx.decode_begin(task.wh_opts(), [task.initial_tokens] * 20, [task.sot_index] * 20)
    m.ctx.decode_steps(50)
    m.ctx.time_stage(4, 3)
    print(f"timestamps={ts}: k_logit_rows {m.ctx.time_stage(4, 20) * 1e3:.1f} us/launch "
          f"(step {m.ctx.time_stage(0, 10):.3f} ms)")
