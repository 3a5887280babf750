"""The multi-GPU path's collectives on the GPU backend: torch.distributed "nccl" (RCCL
on ROCm) with one rank on the box's one GPU, in a fresh child process (the rank owns
its torch / RCCL state, as a torchrun rank does).  whisper/distributed.transcribe_sharded
runs its real exchange steps -- the all-reduce MAX of the log-mel maximum over a
device tensor and the gather of segment records -- and its merged segments equal the
reference transcribe() of the whole file (micro_transcribe.json, the golden the
replayed-rank test in test_gpu_micro.py also uses).  World sizes > 1 are covered on
CPU (gloo, tests/test_distributed.py) and by the driver's 8-GPU bench."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import GOLDEN, PKG_ROOT, REPO

pytestmark = pytest.mark.gpu

_CHILD = r"""
import json, os, sys
sys.path[:0] = [os.environ["PKG_ROOT"], os.environ["REPO"]]
import torch
import torch.distributed as dist
torch.cuda.set_device(0)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:" + os.environ["PORT"], rank=0, world_size=1)
import whisper
from whisper import distributed as D
from whisper import synthetic as S
gt = json.load(open(os.environ["GOLDEN_FILE"]))
kw = dict(gt["runs"][os.environ["RUN"]])
kw.pop("clip_timestamps"), kw.pop("condition_on_previous_text", None)
audio = S.synthetic_audio(gt["audio_seconds"], seed=gt["audio_seed"])
m = whisper.load_model("micro", device=0, dtype="fp32", max_windows=4, max_group=5, synthetic=True)
backend = dist.get_backend()
gmax = D.global_max(1.25)
res = D.transcribe_sharded(m, audio, temperature=0.0, language="en", **kw)
dist.destroy_process_group()
m.close()
print("RESULT " + json.dumps({"backend": backend, "gmax": gmax,
                              "tokens": [s["tokens"] for s in res["segments"]],
                              "seek": [s["seek"] for s in res["segments"]]}))
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("run", ["clip_beam"])
def test_rccl_world1_transcribe_sharded(run):
    gfile = os.path.join(GOLDEN, "micro_transcribe.json")
    env = dict(os.environ, PKG_ROOT=PKG_ROOT, REPO=REPO, PORT=str(_free_port()), GOLDEN_FILE=gfile, RUN=run,
               MASTER_ADDR="127.0.0.1")
    p = subprocess.run([sys.executable, "-c", _CHILD], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    out = json.loads(line[len("RESULT "):])
    assert out["backend"] == "nccl"
    assert out["gmax"] == 1.25
    with open(gfile) as f:
        ref = json.load(f)["segments"][run]
    assert out["tokens"] == [s["tokens"] for s in ref]
    assert out["seek"] == [s["seek"] for s in ref]
