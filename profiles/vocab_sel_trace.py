"""Probe (round 4): where the time of the single-window fused token tail (k_vocab_sel)
goes.  The tuning build records, per workgroup, wall-clock marks (s_memrealtime, 100 MHz)
at the phase boundaries of the last launch; this replays one live step graph at a time and
prints, per mark, the median and maximum over the 256 workgroups of the time since the
first workgroup started (the last workgroup's combine and merge: marks 7 and 8).
    WHISPER_HIP_LIB=whisper.coreml_amd/lib/libwhisper_hip_tune.so python profiles/vocab_sel_trace.py [model]
"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "whisper.coreml_amd"), REPO]
import whisper  # noqa: E402
from whisper import synthetic as S  # noqa: E402
from whisper.decoding import DecodingTask  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "large-v3"
dims = S.MODEL_DIMS[name]
m = whisper.Whisper(whisper.ModelDimensions(**dims), name, device=0, dtype="fp16", max_windows=1, max_group=5)
m.load_state_dict(S.synthetic_state_dict(dims, 0))
audio = S.synthetic_audio(30.0, seed=1000)
m.ctx.log_mel(audio, dims["n_mels"], padding=whisper.audio.N_SAMPLES)
m.ctx.encode([0], [3000])
task = DecodingTask(m, whisper.DecodingOptions(language="en", beam_size=5))
eot = task.tokenizer.eot
task = DecodingTask(m, whisper.DecodingOptions(language="en", beam_size=5, suppress_tokens=f"-1,{eot}"))
m.ctx.decode_begin(task.wh_opts(), [task.initial_tokens], [task.sot_index])
print("step kernels", m.ctx.step_kernels(1, 5))
lib = m.ctx.lib
lib.wh_tune_vs_trace.restype = ctypes.c_int
lib.wh_tune_vs_trace.argtypes = [ctypes.c_void_p]
NAMES = ["start", "state loaded", "projection done", "logits in LDS", "records issued", "records drained",
         "arrival counted", "combine done (last)", "merge done (last)"]
buf = np.zeros((256, 10), dtype=np.uint64)
m.ctx.time_stage(0, 3)  # capture + warm
acc = {k: [] for k in range(9)}
for it in range(12):
    ms = m.ctx.time_stage(0, 1)
    assert lib.wh_tune_vs_trace(buf.ctypes.data) == 0
    t = buf.astype(np.int64)
    t0 = t[:, 0].min()
    last = int(np.argmax(t[:, 6]))
    for k in range(9):
        col = (t[:, k] - t0) * 0.01  # us
        if k >= 7:
            acc[k].append((col[last], col[last]))
        else:
            acc[k].append((float(np.median(col)), float(col.max())))
    if it == 0:
        print(f"step graph {ms:.3f} ms")
for k in range(9):
    a = np.asarray(acc[k])
    print(f"mark {k} {NAMES[k]:26s}: median over workgroups {np.median(a[:, 0]):7.2f} us, max {np.median(a[:, 1]):7.2f} us")
