"""Encoder ms per window for a batch of windows, by encoder chunk size (tuning library:
WHISPER_HIP_LIB=.../libwhisper_hip_tune.so WHISPER_HIP_ENC_CHUNK=c).
  python3 profiles/enc_chunk_probe.py [--model large-v3] [--windows 20] [--reps 3]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "whisper.coreml_amd"), REPO]

p = argparse.ArgumentParser()
p.add_argument("--model", default="large-v3")
p.add_argument("--windows", type=int, default=20)
p.add_argument("--reps", type=int, default=3)
args = p.parse_args()

import whisper  # noqa: E402
from whisper import synthetic as S  # noqa: E402

dims = S.MODEL_DIMS[args.model]
m = whisper.Whisper(whisper.ModelDimensions(**dims), args.model, device=0, dtype="fp16",
                    max_windows=args.windows, max_group=5)
m.load_state_dict(S.synthetic_state_dict(dims, 0))
audio = S.synthetic_audio(30.0 * args.windows, seed=1000)
m.ctx.log_mel(audio, dims["n_mels"], padding=whisper.audio.N_SAMPLES)
seeks, segs = [3000 * i for i in range(args.windows)], [3000] * args.windows
m.ctx.encode(seeks, segs)  # warm
t0 = m.ctx.stats()["encode_ms"]
for _ in range(args.reps):
    m.ctx.encode(seeks, segs)
ms = (m.ctx.stats()["encode_ms"] - t0) / args.reps
print(f"{args.model} {args.windows} windows, chunk {os.environ.get('WHISPER_HIP_ENC_CHUNK', 'default')}: "
      f"{ms:.2f} ms per batch = {ms / args.windows:.3f} ms per window")
m.close()
