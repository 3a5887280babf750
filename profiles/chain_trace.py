"""Probe (round 5): the 100-row decoder step's chain, priced per launch.  The tuning build
records per-workgroup wall-clock marks (s_memrealtime, 100 MHz) in every step kernel
(wh_common.h CT_MARK): mark 0 = workgroup start, 1 / 2 = phase ends (k_proj: X staged in
LDS / MFMAs done, i.e. the weights landed; k_resid_ln: the loads landed), 3 = thread 0
done with its stores drained.  Every launch of a role overwrites its slot, so after one
replayed step graph each slot holds the role's LAST launch: layer 31's qkv, self-attention,
cross-attention, cross-out (the n x n slot), fc1, reduce+GELU, fc2, the final residual +
LayerNorm, then the vocabulary projection and the token selection.  Printed per launch:
the first / last workgroup start, the phase marks (median over workgroups) and the last
end, relative to qkv's first start, and the gap from the previous launch's last end to
this launch's first start (the kernel boundary as the chain pays it).
    WHISPER_HIP_LIB=whisper.coreml_amd/lib/libwhisper_hip_tune.so python profiles/chain_trace.py [windows] [reps]
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

W = int(sys.argv[1]) if len(sys.argv) > 1 else 20
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ADVANCE = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # steps replayed before tracing (context length)
model_name = os.environ.get("CT_MODEL", "large-v3")
dims = S.MODEL_DIMS[model_name]
m = whisper.Whisper(whisper.ModelDimensions(**dims), model_name, device=0, dtype="fp16", max_windows=W, max_group=5)
m.load_state_dict(S.synthetic_state_dict(dims, 0))
m.ctx.log_mel(S.synthetic_audio(30.0 * W, seed=1000), dims["n_mels"], padding=whisper.audio.N_SAMPLES)
m.ctx.encode([3000 * i for i in range(W)], [3000] * W)
task = DecodingTask(m, whisper.DecodingOptions(language="en", beam_size=5))
lib = m.ctx.lib
UNITS = ["proj", "kernels", "gemm", "decode"]
for u in UNITS:
    getattr(lib, f"wh_tune_ct_trace_{u}").argtypes = [ctypes.c_void_p]
    getattr(lib, f"wh_tune_ct_trace_{u}").restype = ctypes.c_int
    getattr(lib, f"wh_tune_ct_clear_{u}").restype = ctypes.c_int
SLOT_UNIT = {0: "proj", 1: "proj", 2: "proj", 3: "proj", 4: "kernels", 5: "kernels", 6: "kernels", 7: "kernels",
             8: "gemm", 9: "decode", 10: "decode", 11: "decode"}
ORDER = [(0, "qkv k_proj", ("X staged", "MFMA done")), (6, "self-attn (+qkv reduce)", None),
         (7, "cross-attn k_xattn_seg", None), (1, "cross-out k_proj", ("X staged", "MFMA done")),
         (2, "fc1 k_proj", ("X staged", "MFMA done")), (5, "reduce+GELU", None),
         (3, "fc2 k_proj", ("X staged", "MFMA done")), (4, "resid+LN (final)", ("loads landed", None)),
         (8, "vocab k_vocab_2p / k_vocab1", ("epilogue start", "half 1 staged")), (9, "selection k_logit_part", ("row combine", "window merge")),
         (10, "  merge_window (in it)", ("staged", "ranked")),
         (11, "  selection slices (marks)", ("loads", "top-k"))]

m.ctx.decode_begin(task.wh_opts(), [task.initial_tokens] * W, [task.sot_index] * W)
m.ctx.time_stage(0, 2 + ADVANCE)  # graph captured, warm; ADVANCE more tokens of context
rows = {s: [] for s, _, _ in ORDER}
steps = []
for rep in range(REPS):
    for u in UNITS:
        assert getattr(lib, f"wh_tune_ct_clear_{u}")() == 0
    steps.append(m.ctx.time_stage(0, 1))
    tr = {}
    for u in UNITS:
        buf = np.zeros((12, 2048, 4), dtype=np.uint64)
        assert getattr(lib, f"wh_tune_ct_trace_{u}")(buf.ctypes.data) == 0
        tr[u] = buf.astype(np.int64)
    base = None
    for slot, name, phases in ORDER:
        t = tr[SLOT_UNIT[slot]][slot]
        t = t[t[:, 0] > 0]
        if len(t) == 0:
            continue
        if base is None:
            base = t[:, 0].min()
        rel = (t - base) * 0.01  # us
        ends = rel[:, 3][t[:, 3] > 0]
        rows[slot].append(dict(n=len(t), s0=rel[:, 0].min(), s1=rel[:, 0].max(),
                               p1=np.median(rel[:, 1][t[:, 1] > 0]) if (t[:, 1] > 0).any() else np.nan,
                               p2=np.median(rel[:, 2][t[:, 2] > 0]) if (t[:, 2] > 0).any() else np.nan,
                               e_med=np.median(ends) if len(ends) else np.nan, e1=ends.max() if len(ends) else np.nan,
                               p1max=rel[:, 1][t[:, 1] > 0].max() if (t[:, 1] > 0).any() else np.nan,
                               p2max=rel[:, 2][t[:, 2] > 0].max() if (t[:, 2] > 0).any() else np.nan))
print(f"{model_name} fp16, {W} windows x beam 5 ({5 * W} rows), after {2 + ADVANCE} steps: "
      f"step graph {np.median(steps):.3f} ms "
      f"(median of {REPS}); times in us from layer 31's qkv first workgroup start, medians over {REPS} steps")
print(f"{'launch':28s} {'WGs':>5s} {'gap':>6s} {'start0':>7s} {'startN':>7s} {'phase1':>7s} {'phase2':>7s} "
      f"{'end med':>7s} {'end max':>7s} {'span':>6s}")
prev_end = None
for slot, name, phases in ORDER:
    if not rows[slot]:
        continue
    agg = {k: float(np.nanmedian([r[k] for r in rows[slot]])) for k in rows[slot][0]}
    gap = agg["s0"] - prev_end if prev_end is not None else float("nan")
    print(f"{name:28s} {int(agg['n']):5d} {gap:6.2f} {agg['s0']:7.2f} {agg['s1']:7.2f} {agg['p1']:7.2f} "
          f"{agg['p2']:7.2f} {agg['e_med']:7.2f} {agg['e1']:7.2f} {agg['e1'] - agg['s0']:6.2f}"
          f"   (phase maxima {agg['p1max']:.2f} / {agg['p2max']:.2f})")
    prev_end = agg["e1"]
