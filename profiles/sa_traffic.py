"""HBM traffic of the step self-attention (k_self_attn_qkv) at late context (round 5):
does the L2 dedupe the beams' shared history rows, or does every (row, head) wave pull its
whole history from HBM?  Workload (`run`): large-v3 fp16, 20 windows x beam 5, eager
steps (WHISPER_HIP_EAGER=1, tuning library: rocprofv3 follows eager dispatches) advanced
to ~205 tokens of context; `parse <fetch dir> <write dir>` reports the LAST step's 32
self-attention dispatches (FETCH_SIZE x 2 gfx950 read correction, WRITE_SIZE exact) beside
the logical K/V bytes (rows x heads x 2 x t x 64 x 2 B).

Round 5's form (200 EAGER steps under `--pmc FETCH_SIZE --kernel-trace`) died with SIGSEGV
inside the HIP launch path, in the profiler's interception of a k_proj dispatch, after
~80 k dispatches (gpurun_out/sa_f.log): the same range in which rocprofv3's kernel trace
crashes with trivial kernels (tools/graph_prof_repro.hip).  Round 6: the
context is advanced by replaying the captured step graph (ADVANCE steps: no per-kernel host
dispatch), then ONE eager step runs (the library reads WHISPER_HIP_EAGER per call), and the
profiler counts only the self-attention (--kernel-include-regex), without --kernel-trace:
  cd /tmp && export TMPDIR=/tmp
  WHISPER_HIP_LIB=... rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_self_attn_qkv -d D -o run \
      --output-format csv -- python3 sa_traffic.py run
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# context steps before the traced one; SA_GRAPH=1 advances them by graph replays.  Round 6:
# under --pmc the graph replay itself crashed rocprofv3 (SIGSEGV in the first hipGraphLaunch
# after HSA init, profiles/r06/sa_traffic_crash.log), so the default is eager with a
# context short enough to stay under the dispatch counts where its crashes begin
STEPS = int(os.environ.get("SA_STEPS", "100"))
GRAPH = os.environ.get("SA_GRAPH", "0") == "1"


def run():
    sys.path.insert(0, os.path.join(REPO, "whisper.coreml_amd"))
    import whisper
    from whisper import synthetic as S
    from whisper.decoding import DecodingTask
    dims = S.MODEL_DIMS["large-v3"]
    m = whisper.Whisper(whisper.ModelDimensions(**dims), "large-v3", device=0, dtype="fp16", max_windows=20, max_group=5)
    m.load_state_dict(S.synthetic_state_dict(dims, 0))
    m.ctx.log_mel(S.synthetic_audio(600.0, seed=1000), dims["n_mels"], padding=480000)
    m.ctx.encode([3000 * i for i in range(20)], [3000] * 20)
    task = DecodingTask(m, whisper.DecodingOptions(language="en", beam_size=5))
    m.ctx.decode_begin(task.wh_opts(), [task.initial_tokens] * 20, [task.sot_index] * 20)
    if GRAPH:
        os.environ.pop("WHISPER_HIP_EAGER", None)
    else:
        os.environ["WHISPER_HIP_EAGER"] = "1"
    print("context steps ms", m.ctx.time_stage(0, STEPS - 1), flush=True)
    os.environ["WHISPER_HIP_EAGER"] = "1"
    print("eager step ms", m.ctx.time_stage(0, 1), flush=True)  # the traced step: 32 self-attention dispatches
    m.close()


def _per_dispatch(d, counter):
    per, names = defaultdict(float), {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter:
                k = int(r["Dispatch_Id"])
                per[k] += float(r["Counter_Value"])
                names[k] = r["Kernel_Name"]
    return per, names


def parse(dfetch, dwrite):
    out = {}
    for counter, d, scale in (("FETCH_SIZE", dfetch, 2 * 1024), ("WRITE_SIZE", dwrite, 1024)):
        per, names = _per_dispatch(d, counter)
        ids = sorted(k for k in per if "k_self_attn_qkv" in names[k])[-32:]
        out[counter] = scale * sum(per[k] for k in ids) / max(len(ids), 1)
        out[counter + "_dispatches"] = len(ids)
    t = 4 + STEPS  # context positions of the traced step (sot sequence + generated)
    out["logical_kv_bytes"] = 100 * 20 * 2 * t * 64 * 2
    out["context"] = t
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    run() if sys.argv[1] == "run" else parse(sys.argv[2], sys.argv[3])
