"""Diagnostic (round 5): which interleaved call changes a chunked device-loop decode."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "whisper.coreml_amd"), REPO, os.path.join(REPO, "tests")]
import test_gpu_resume as T  # noqa: E402
import whisper  # noqa: E402
from whisper.timing import _alignment_head_ids  # noqa: E402
from whisper.tokenizer import get_tokenizer  # noqa: E402

m = whisper.load_model("micro", device=0, dtype="fp32", max_windows=4, max_group=5, synthetic=True)
for n in (3, 1):
    task = T._setup(m, n)
    init = [task.initial_tokens] * n
    m.ctx.decode_begin(task.wh_opts(), init, [task.sot_index] * n)
    m.ctx.decode_steps(task.sample_len)
    ref = T._read(m, task, n)
    tok = get_tokenizer(m.is_multilingual, num_languages=m.num_languages, language="en", task="transcribe")
    heads = _alignment_head_ids(m)
    seq = [*tok.sot_sequence, tok.no_timestamps, *range(100, 140), tok.eot]
    ops = {"none": lambda: None,
           "align": lambda: m.ctx.align_batch([3], [seq], len(tok.sot_sequence), [3000], heads),
           "prefill": lambda: m.ctx.prefill_logits(3, list(task.initial_tokens) + list(range(200, 230))),
           "stage2": lambda: m.ctx.time_stage(2, 1)}
    for name, op in ops.items():
        m.ctx.decode_begin(task.wh_opts(), init, [task.sot_index] * n)
        m.ctx.decode_steps(9)
        op()
        m.ctx.decode_steps(17)
        op()
        m.ctx.decode_steps(task.sample_len)
        got = T._read(m, task, n)
        bad = []
        for w in range(n):
            for a, b, what in zip(got[w], ref[w], ("tokens", "slp", "len", "fin_len", "fin_score")):
                a, b = np.asarray(a), np.asarray(b)
                if not np.array_equal(a, b):
                    nz = np.argwhere(a != b)
                    bad.append(f"w{w}:{what}:{len(nz)} first {nz[0].tolist()}")
        print(f"n={n} op={name}: {'OK' if not bad else bad}", flush=True)
m.close()
