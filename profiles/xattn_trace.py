"""Probe (round 4): where the time of the step cross-attention (k_xattn_seg) goes.  The
tuning build records, per workgroup, wall-clock marks (s_memrealtime, 100 MHz) at the
phase boundaries of the last launch: 0 start, 1 query rows staged (LDS barrier), 2 wave 0's
tiles done, 3 every tile done (barrier), 4 merge from LDS / records stored and drained,
5 arrival counted, 6 cut pair merged by the last arriver.  Runs all 32 layers
(wh_time_stage 3, HBM-cold as in the step) and reads the last launch; prints, per mark,
the median and maximum over workgroups of the time since the first workgroup started.
    WHISPER_HIP_LIB=whisper.coreml_amd/lib/libwhisper_hip_tune.so python profiles/xattn_trace.py [windows,...]
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

wins = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [20, 1]
dims = S.MODEL_DIMS["large-v3"]
W = max(wins)
m = whisper.Whisper(whisper.ModelDimensions(**dims), "large-v3", device=0, dtype="fp16", max_windows=W, max_group=5)
m.load_state_dict(S.synthetic_state_dict(dims, 0))
m.ctx.log_mel(S.synthetic_audio(30.0 * W, seed=1000), dims["n_mels"], padding=whisper.audio.N_SAMPLES)
m.ctx.encode([3000 * i for i in range(W)], [3000] * W)
task = DecodingTask(m, whisper.DecodingOptions(language="en", beam_size=5))
lib = m.ctx.lib
lib.wh_tune_xs_trace.restype = ctypes.c_int
lib.wh_tune_xs_trace.argtypes = [ctypes.c_void_p]
NAMES = ["start", "query staged", "wave 0 tiles done", "all tiles done", "merged / records drained",
         "arrival counted", "cut pair merged", "(qproj) X rows staged", "(qproj) W_q landed, MFMAs done"]
NM = 10  # marks per workgroup (wh_kernels.hip XS_MARKS)
for nw in wins:
    m.ctx.decode_begin(task.wh_opts(), [task.initial_tokens] * nw, [task.sot_index] * nw)
    m.ctx.time_stage(3, 1)
    acc = {k: [] for k in range(9)}
    spans = []
    for it in range(10):
        us_launch = m.ctx.time_stage(3, 1) * 1e3
        buf = np.zeros((256, NM), dtype=np.uint64)
        assert lib.wh_tune_xs_trace(buf.ctypes.data) == 0
        t = buf.astype(np.int64)
        live = t[:, 0] > 0
        # only the workgroups of the last launch: their start within 1 ms of the latest start
        live &= t[:, 0] >= t[live, 0].max() - 100000
        t = t[live]
        t0 = t[:, 0].min()
        for k in range(9):
            col = t[:, k]
            ok = col >= t0
            if k >= 6:
                ok &= col > 0
            if ok.any():
                v = (col[ok] - t0) * 0.01
                acc[k].append((float(np.median(v)), float(v.max()), int(ok.sum())))
        spans.append((us_launch, (t[:, 5].max() - t0) * 0.01, (t[:, 0].max() - t0) * 0.01))
    sp = np.asarray(spans)
    print(f"windows {nw}: {len(t)} workgroups; launch (events, 32 layers) {np.median(sp[:, 0]):.2f} us, "
          f"first start -> last mark 5 {np.median(sp[:, 1]):.2f} us, last workgroup starts at {np.median(sp[:, 2]):.2f} us")
    for k in range(9):
        if acc[k]:
            a = np.asarray(acc[k])
            print(f"  mark {k} {NAMES[k]:26s}: median {np.median(a[:, 0]):6.2f} us, max {np.median(a[:, 1]):6.2f} us "
                  f"({int(np.median(a[:, 2]))} workgroups)")
m.close()
