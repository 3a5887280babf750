"""One decoder-step batch replayed as the hipGraph, for rocprofv3 kernel traces of graph
mode: rocprofv3 --kernel-trace segfaults once a process has dispatched somewhere
between 8k and 80k graph-launched kernels (tools/graph_prof_repro.hip reproduces it
with trivial kernels: profiles/r02/graph_prof_repro.txt), and a bench transcribe()
dispatches ~80k, so this replays only `--steps` step graphs (~370 kernels each).
  python3 profiles/step_profile.py [--model large-v3] [--windows 20] [--steps 16]"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "whisper.coreml_amd"), REPO]

p = argparse.ArgumentParser()
p.add_argument("--model", default="large-v3")
p.add_argument("--windows", type=int, default=20)
p.add_argument("--beam", type=int, default=5)
p.add_argument("--steps", type=int, default=16)
p.add_argument("--dtype", default="fp16")
p.add_argument("--encode", type=int, default=0, help="also run this many encoder passes of 1 window")
args = p.parse_args()

import numpy as np  # noqa: E402

import whisper  # noqa: E402
from whisper import synthetic as S  # noqa: E402
from whisper.decoding import DecodingTask  # noqa: E402

dims = S.MODEL_DIMS[args.model]
m = whisper.Whisper(whisper.ModelDimensions(**dims), args.model, device=0, dtype=args.dtype,
                    max_windows=args.windows, max_group=args.beam)
m.load_state_dict(S.synthetic_state_dict(dims, 0))
audio = S.synthetic_audio(30.0 * args.windows, seed=1000)
m.ctx.log_mel(audio, dims["n_mels"], padding=whisper.audio.N_SAMPLES)
m.ctx.encode([3000 * i for i in range(args.windows)], [3000] * args.windows)
task = DecodingTask(m, whisper.DecodingOptions(language="en", beam_size=args.beam if args.beam > 1 else None))
m.ctx.decode_begin(task.wh_opts(), [task.initial_tokens] * args.windows, [task.sot_index] * args.windows)
m.ctx.time_stage(0, 3)  # capture + warm
t0 = time.perf_counter()
ms = m.ctx.time_stage(0, args.steps)
print(f"{args.model} {args.windows}x{args.beam} {args.dtype}: {ms:.4f} ms per step graph over {args.steps} replays "
      f"(wall {1e3 * (time.perf_counter() - t0) / args.steps:.4f})")
if args.encode:
    print(f"encoder: {m.ctx.time_stage(1, args.encode):.3f} ms per window")
m.close()
