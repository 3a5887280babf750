"""Per-window cost of word timestamps (config 5) on large-v3 fp16: wall time of
wh_align (first pass + alignment + DTW) vs the host half of find_alignment.
    python profiles/align_timing.py
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "whisper.coreml_amd"))

import whisper  # noqa: E402
from whisper import synthetic as S  # noqa: E402
from whisper import tokenizer as T  # noqa: E402
from whisper.timing import _alignment_head_ids, find_alignment  # noqa: E402

dims = S.MODEL_DIMS["large-v3"]
m = whisper.Whisper(whisper.ModelDimensions(**dims), "large-v3", device=0, dtype="fp16", max_windows=4, max_group=5)
m.load_state_dict(S.synthetic_state_dict(dims, 0))
m.set_alignment_heads(whisper._ALIGNMENT_HEADS["large-v3"])
T.set_token_bytes("multilingual", {i: b" w%d" % i for i in range(dims["n_vocab"])})
tok = T.get_tokenizer(True, num_languages=m.num_languages, language="en", task="transcribe")
audio = S.synthetic_audio(30.0, seed=3)
m.ctx.log_mel(audio, dims["n_mels"], padding=480000)
m.ctx.encode([0], [3000])
rng = np.random.default_rng(0)
text = [int(t) for t in rng.integers(0, tok.eot, 220)]
toks = [*tok.sot_sequence, tok.no_timestamps, *text, tok.eot]
heads = _alignment_head_ids(m)
for _ in range(2):
    m.ctx.align(0, toks, len(tok.sot_sequence), 3000, heads)
n = 5
t0 = time.perf_counter()
for _ in range(n):
    m.ctx.align(0, toks, len(tok.sot_sequence), 3000, heads)
t_align = (time.perf_counter() - t0) / n
t0 = time.perf_counter()
for _ in range(n):
    find_alignment(m, tok, text, 3000)
t_find = (time.perf_counter() - t0) / n
t0 = time.perf_counter()
for _ in range(n):
    m.ctx.prefill_logits(0, toks[:4])
t_pre4 = (time.perf_counter() - t0) / n
print(f"wh_align {t_align*1e3:.2f} ms  find_alignment {t_find*1e3:.2f} ms  (host half {1e3*(t_find-t_align):.2f} ms)"
      f"  prefill_logits(4 tokens) {t_pre4*1e3:.2f} ms  heads={len(heads)} T={len(text)}")
m.close()
