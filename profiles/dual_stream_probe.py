"""Probe: do two half-batch decode steps on two streams overlap on MI355X?

Two contexts (10 windows x beam 5 each, their own weights and HIP stream) replay
their step graphs from two host threads at once, against one context with all 20
windows.  If the pair finishes 20-window-equivalent steps faster, a dual-stream step
(one context, two window groups, shared weights) is worth building.
    python profiles/dual_stream_probe.py
"""
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "whisper.coreml_amd"))

import whisper  # noqa: E402
from whisper import synthetic as S  # noqa: E402
from whisper.decoding import DecodingTask  # noqa: E402

dims = S.MODEL_DIMS["large-v3"]
sd = S.synthetic_state_dict(dims, 0)
audio = S.synthetic_audio(600.0, seed=1000)


def make(nwin):
    m = whisper.Whisper(whisper.ModelDimensions(**dims), "large-v3", device=0, dtype="fp16", max_windows=nwin,
                        max_group=5)
    m.load_state_dict(sd)
    m.ctx.log_mel(audio, dims["n_mels"], padding=480000)
    m.ctx.encode([3000 * i for i in range(nwin)], [3000] * nwin)
    task = DecodingTask(m, whisper.DecodingOptions(language="en", beam_size=5, suppress_tokens="-1,50257"))
    m.ctx.decode_begin(task.wh_opts(), [task.initial_tokens] * nwin, [task.sot_index] * nwin)
    return m


full = make(20)
full.ctx.time_stage(0, 5)
t_full = full.ctx.time_stage(0, 40)
print(f"one context, 20 windows: {t_full:.3f} ms/step")
full.close()
a, b = make(10), make(10)
a.ctx.time_stage(0, 5)
b.ctx.time_stage(0, 5)
t_half = a.ctx.time_stage(0, 40)
print(f"one context, 10 windows alone: {t_half:.3f} ms/step")
res = {}


def run(m, k):
    t0 = time.perf_counter()
    m.ctx.time_stage(0, 40)
    res[k] = (time.perf_counter() - t0) * 1e3 / 40


ta = threading.Thread(target=run, args=(a, "a"))
tb = threading.Thread(target=run, args=(b, "b"))
t0 = time.perf_counter()
ta.start(); tb.start(); ta.join(); tb.join()
wall = (time.perf_counter() - t0) * 1e3 / 40
print(f"two contexts x 10 windows concurrently: {wall:.3f} ms per (pair of) steps; per-thread {res}")
print(f"speedup vs one 20-window context: {t_full / wall:.3f}x")
