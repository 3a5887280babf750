"""Probe (round 4): two window groups of one file decoding on two streams, sharing ONE
weight copy, with group B's step graphs started a fixed delay after group A's.

The 100-row step is a chain of ~390 dependent launches, most of them latency-bound
(projections, reductions) and one per layer bandwidth-bound (the cross-attention over
20 windows' cross-KV, 36 us).  Two 10-window groups whose chains run offset from each
other could overlap one group's cross-attention with the other's latency-bound
launches.  Round 2's probe ran two contexts with their OWN weights, started together
(dual_stream_probe.py: 3.96 vs 3.68 ms); here B reads A's weights (tuning build:
wh_tune_share_weights) and starts `delay` ms later.
    WHISPER_HIP_LIB=whisper.coreml_amd/lib/libwhisper_hip_tune.so python profiles/stagger_probe.py
"""
import ctypes
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
ITERS = 40


def prepare(m, nwin, first):
    m.ctx.log_mel(audio, dims["n_mels"], padding=480000)
    m.ctx.encode([3000 * (first + i) for i in range(nwin)], [3000] * nwin)
    task = DecodingTask(m, whisper.DecodingOptions(language="en", beam_size=5, suppress_tokens="-1,50257"))
    m.ctx.decode_begin(task.wh_opts(), [task.initial_tokens] * nwin, [task.sot_index] * nwin)
    m.ctx.time_stage(0, 3)  # capture + warm


def new_model(nwin, load):
    m = whisper.Whisper(whisper.ModelDimensions(**dims), "large-v3", device=0, dtype="fp16", max_windows=nwin,
                        max_group=5)
    if load:
        m.load_state_dict(sd)
    return m


full = new_model(20, True)
prepare(full, 20, 0)
t_full = full.ctx.time_stage(0, ITERS)
print(f"one context, 20 windows: {t_full:.3f} ms/step", flush=True)
full.close()

a = new_model(10, True)
b = new_model(10, False)
lib = a.ctx.lib
lib.wh_tune_share_weights.restype = ctypes.c_int
lib.wh_tune_share_weights.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
assert lib.wh_tune_share_weights(b.ctx.h, a.ctx.h) == 0, lib.wh_last_error()
b.ctx.set_mel_filters(dims["n_mels"], whisper.audio.mel_filters(None, dims["n_mels"]))
prepare(a, 10, 0)
prepare(b, 10, 10)
t_half = a.ctx.time_stage(0, ITERS)
print(f"one 10-window group alone: {t_half:.3f} ms/step", flush=True)

for delay_ms in (0.0, 0.05, 0.3, 0.8, 1.5):
    res = {}

    def run(m, k, d):
        if d:
            time.sleep(d / 1e3)
        t0 = time.perf_counter()
        m.ctx.time_stage(0, ITERS)
        res[k] = (t0, time.perf_counter())

    ta = threading.Thread(target=run, args=(a, "a", 0.0))
    tb = threading.Thread(target=run, args=(b, "b", delay_ms))
    ta.start()
    tb.start()
    ta.join()
    tb.join()
    span = (max(res["a"][1], res["b"][1]) - min(res["a"][0], res["b"][0])) * 1e3 / ITERS
    print(f"delay {delay_ms:4.2f} ms: {span:.3f} ms per pair of 10-window steps "
          f"(= 20-window equivalent; one context {t_full:.3f}) -> {t_full / span:.3f}x", flush=True)
