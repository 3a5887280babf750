"""HBM traffic per launch of the decoder-step kernels from rocprofv3 PMC counters.

Workload (`run`): large-v3 fp16 at the bench batch (20 windows x beam 5 = 100 rows),
encode (k_gemm_256) + decode_begin, then wh_time_stage 2 (the six split-K projections
(k_proj) of every decoder layer) and 3 (cross-attention of every layer) once each; then
one window (5 rows) and stage 2 again (the k_proj1 projections).

Collected in two separate passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass
on gfx950, MI355X_MICROARCH.md "rocprofv3 PMC slots"):

  cd /tmp && export TMPDIR=/tmp
  rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/pmc_f -o run --output-format csv -- \
      python $R/profiles/pmc_traffic.py run
  rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/pmc_w -o run --output-format csv -- \
      python $R/profiles/pmc_traffic.py run
  python profiles/pmc_traffic.py parse gpurun_out/pmc_f gpurun_out/pmc_w > profiles/r02/traffic.json

Correction (same guide, "HBM [CDNA4]"): FETCH_SIZE counts half the bytes of 16 B/lane
streaming reads on gfx950, so reads = 2 x FETCH_SIZE; WRITE_SIZE is exact for 16 B
stores.  Both are in KiB.  Infinity-Cache hits are counted, not excluded.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

KERNELS = {
    # short name -> regex on the mangled kernel name
    "k_proj": r"k_projIDF16_",                # fp16 split-K projections (all tile variants), 100 rows
    "k_proj1": r"k_proj1IDF16_",              # single-window projections (5 rows, all six shapes)
    "k_xattn_seg": r"k_xattn_segIDF16_",      # the step's cross-attention (round 3), 20 windows
    "k_resid_ln": r"k_resid_lnIDF16_",        # split-K reduction + residual + LayerNorm, 100 rows
    "k_gemm_256": r"k_gemm_256",              # encoder GEMMs of the 20-window encode (all epilogues)
}


def run():
    sys.path.insert(0, os.path.join(REPO, "whisper.coreml_amd"))
    import whisper
    from whisper import synthetic as S
    from whisper.decoding import DecodingTask
    dims = S.MODEL_DIMS["large-v3"]
    model = whisper.Whisper(whisper.ModelDimensions(**dims), "large-v3", device=0, dtype="fp16",
                            max_windows=20, max_group=5)
    model.load_state_dict(S.synthetic_state_dict(dims, 0))
    audio = S.synthetic_audio(600.0, seed=1000)
    model.ctx.log_mel(audio, padding=480000, n_mels=dims["n_mels"], normalize=True)
    model.ctx.encode([3000 * i for i in range(20)], [3000] * 20)
    task = DecodingTask(model, whisper.DecodingOptions(language="en", beam_size=5))
    model.ctx.decode_begin(task.wh_opts(), [task.initial_tokens] * 20, [task.sot_index] * 20)
    print("gemv ms/launch", model.ctx.time_stage(2, 1))
    print("cross-attn ms/launch", model.ctx.time_stage(3, 1))
    print("step ms", model.ctx.time_stage(0, 2))  # k_resid_ln (and every step kernel) in the graph
    # one window (5 rows): the six projections of every layer as k_proj1 launches
    model.ctx.decode_begin(task.wh_opts(), [task.initial_tokens], [task.sot_index])
    print("k_proj1 ms/launch", model.ctx.time_stage(2, 1))
    model.close()


def _counters(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(float)
    names = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            key = (f, r["Dispatch_Id"])
            per[key] += float(r["Counter_Value"])
            names[key] = r["Kernel_Name"]
    return per, names


def parse(dir_fetch, dir_write):
    fetch, fn = _counters(dir_fetch, "FETCH_SIZE")
    write, wn = _counters(dir_write, "WRITE_SIZE")
    out = {}
    for short, pat in KERNELS.items():
        f = [v for k, v in fetch.items() if re.search(pat, fn[k])]
        w = [v for k, v in write.items() if re.search(pat, wn[k])]
        if not f or not w:
            continue
        rd = 2 * 1024 * sum(f) / len(f)   # KiB -> bytes, x2 gfx950 read correction
        wr = 1024 * sum(w) / len(w)
        out[short] = {"hbm_bytes_per_launch": round(rd + wr), "read_bytes": round(rd), "write_bytes": round(wr),
                      "dispatches": [len(f), len(w)], "pattern": pat}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        parse(sys.argv[2], sys.argv[3])
