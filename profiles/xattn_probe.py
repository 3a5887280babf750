"""Step cross-attention (k_xattn_seg) time per launch against the number of decode
windows, and the whole step graph per window count.  With the tuning build
(WHISPER_HIP_LIB=.../libwhisper_hip_tune.so) a third argument lists the per-wave segment
counts to force (WHISPER_HIP_XS_K, read per launch; 0 = the default grid)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "whisper.coreml_amd"), REPO]
import whisper  # noqa: E402
from whisper import synthetic as S  # noqa: E402
from whisper.decoding import DecodingTask  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "large-v3"
dims = S.MODEL_DIMS[name]
m = whisper.Whisper(whisper.ModelDimensions(**dims), name, device=0, dtype="fp16", max_windows=24, max_group=5)
m.load_state_dict(S.synthetic_state_dict(dims, 0))
audio = S.synthetic_audio(30.0 * 24, seed=1000)
m.ctx.log_mel(audio, dims["n_mels"], padding=whisper.audio.N_SAMPLES)
m.ctx.encode([3000 * i for i in range(24)], [3000] * 24)
task = DecodingTask(m, whisper.DecodingOptions(language="en", beam_size=5))
wins = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2, 4, 6, 8, 10, 12, 13, 14, 16, 18, 20, 24]
ks = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0]
for nw in wins:
    m.ctx.decode_begin(task.wh_opts(), [task.initial_tokens] * nw, [task.sot_index] * nw)
    for k in ks:
        os.environ["WHISPER_HIP_XS_K"] = str(k)
        xa = m.ctx.time_stage(3, 5)
        step = m.ctx.time_stage(0, 10) if k == ks[0] else float("nan")
        mb = nw * 2 * 1500 * dims["n_text_state"] * 2 / 1e6
        print(f"windows {nw:2d} k {k}: cross-attn {xa * 1e3:6.1f} us ({mb / xa / 1e3:5.2f} TB/s)  step {step:.3f} ms",
              flush=True)
