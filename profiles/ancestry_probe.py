"""Probe (round 4): how the 100-row step time grows with the decoded context, and how much
of the self-attention's cached K/V the 5 beams of a window share.

Beam histories form a tree: two beams whose ancestries name the same (slot, position)
row share every earlier row too.  Per checkpoint this prints the step graph time
(time_stage 0, which advances the decode), the mean length of the prefix all 5 beams
share, and the mean number of distinct cached rows per position over the context
(1 = every beam reads the same row, 5 = all different): the self-attention's per-wave K/V
loads could shrink by that factor if a window's beams loaded each distinct row once.
    python profiles/ancestry_probe.py [model] [windows]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "whisper.coreml_amd"), REPO]
import whisper  # noqa: E402
from whisper import synthetic as S  # noqa: E402
from whisper.decoding import DecodingTask  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "large-v3"
nw = int(sys.argv[2]) if len(sys.argv) > 2 else 20
G = 5
dims = S.MODEL_DIMS[name]
m = whisper.Whisper(whisper.ModelDimensions(**dims), name, device=0, dtype="fp16", max_windows=nw, max_group=G)
m.load_state_dict(S.synthetic_state_dict(dims, 0))
audio = S.synthetic_audio(30.0 * nw, seed=1000)
m.ctx.log_mel(audio, dims["n_mels"], padding=whisper.audio.N_SAMPLES)
m.ctx.encode([3000 * i for i in range(nw)], [3000] * nw)
S_EOT = DecodingTask(m, whisper.DecodingOptions(language="en", beam_size=G)).tokenizer.eot
task = DecodingTask(m, whisper.DecodingOptions(language="en", beam_size=G, suppress_tokens="-1,%d" % S_EOT))
m.ctx.decode_begin(task.wh_opts(), [task.initial_tokens] * nw, [task.sot_index] * nw)


def sharing():
    pcs, dist = [], []
    for w in range(nw):
        r = m.ctx.decode_read(w, G)
        ln = r["length"]
        h = r["tokens"][:, :ln]
        same = np.all(h == h[0:1], axis=0)
        pc = int(np.argmin(same)) if not same.all() else ln
        pcs.append(pc / ln)
        # distinct ancestors per position = distinct token prefixes ending there
        d = [len({tuple(h[b, :p + 1]) for b in range(G)}) for p in range(ln)]
        dist.append(float(np.mean(d)))
    return ln, float(np.mean(pcs)), float(np.mean(dist))


done = 0
for target in (8, 32, 64, 96, 128, 160, 192, 216):
    while done < target - 4:
        m.ctx.decode_steps(min(8, target - 4 - done))
        done += min(8, target - 4 - done)
    ms = m.ctx.time_stage(0, 4)
    done += 4
    ln, pc, dist = sharing()
    print(f"len {ln:3d}: step {ms:.3f} ms  shared prefix {pc:.2f} of the context  distinct rows per position {dist:.2f}",
          flush=True)
