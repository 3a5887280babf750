"""Host-side time of one bench step (config 3): cProfile of transcribe_sharded's pieces on
one GPU, to separate Python / ctypes overhead from GPU time.
  python3 profiles/host_profile.py"""
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "whisper.coreml_amd"), REPO]

import whisper  # noqa: E402
from whisper import distributed as D  # noqa: E402
from whisper import synthetic as S  # noqa: E402

dims = S.MODEL_DIMS["large-v3"]
m = whisper.Whisper(whisper.ModelDimensions(**dims), "large-v3", device=0, dtype="fp16", max_windows=20, max_group=5)
m.load_state_dict(S.synthetic_state_dict(dims, 0))
audio = S.synthetic_audio(600.0, seed=1000)
dev = m.ctx.audio_upload(audio)
kw = dict(temperature=0.0, beam_size=5, language="en")


def step():
    st = D.prepare_shard(m, dev, 0, 1)
    segs = D.run_shard(m, st, st.local_max, **kw)
    return D.merge_segments([segs])


step()
m.ctx.sync()
s0 = m.ctx.stats()
t0 = time.perf_counter()
pr = cProfile.Profile()
pr.enable()
step()
m.ctx.sync()
pr.disable()
el = time.perf_counter() - t0
s1 = m.ctx.stats()
print(f"wall {el * 1e3:.1f} ms; decode_steps {s1['steps_ms'] - s0['steps_ms']:.1f} ms; encode {s1['encode_ms'] - s0['encode_ms']:.1f} ms")
pstats.Stats(pr).sort_stats("cumulative").print_stats(30)
