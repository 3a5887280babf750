"""Per-kernel summary of a rocprofv3 PMC pass (``--pmc ... --kernel-trace --output-format csv``).

  python3 profiles/pmc_summary.py <rocprof output dir> [kernel regex ...] > out.json

For every kernel name matching a regex (default: every kernel): dispatches, mean
duration (kernel trace), and the mean of each collected counter per dispatch.  Derived,
where the counters are present (MI355X_MICROARCH.md "rocprofv3 PMC slots" and the
DVFS note: GRBM_GUI_ACTIVE is summed over the 8 XCDs):
  * mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs):
    the share of all SIMD cycles the matrix pipes were busy;
  * eff_clock_ghz = GRBM_GUI_ACTIVE / 8 / duration;
  * lds_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE: extra LDS cycles from
    bank conflicts over all LDS-array cycles.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def main(d, pats):
    counters = defaultdict(lambda: defaultdict(float))
    names = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            key = (os.path.dirname(f), r["Dispatch_Id"])
            counters[key][r["Counter_Name"]] += float(r["Counter_Value"])
            names[key] = r["Kernel_Name"]
    dur = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[(os.path.dirname(f), r["Dispatch_Id"])] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    groups = defaultdict(list)
    for key, nm in names.items():
        short = nm if not pats else next((p for p in pats if re.search(p, nm)), None)
        if short is not None:
            groups[short].append(key)
    out = {}
    for short, keys in groups.items():
        agg = defaultdict(float)
        for k in keys:
            for c, v in counters[k].items():
                agg[c] += v / len(keys)
        ds = [dur[k] for k in keys if k in dur]
        rec = {"dispatches": len(keys), "mean_ns": round(sum(ds) / len(ds), 1) if ds else None}
        rec.update({c: round(v, 1) for c, v in sorted(agg.items())})
        if "GRBM_GUI_ACTIVE" in agg and agg["GRBM_GUI_ACTIVE"] > 0:
            xcd_cycles = agg["GRBM_GUI_ACTIVE"] / 8
            if "SQ_VALU_MFMA_BUSY_CYCLES" in agg:
                rec["mfma_busy_frac"] = round(agg["SQ_VALU_MFMA_BUSY_CYCLES"] / (xcd_cycles * 1024), 4)
            if rec["mean_ns"]:
                rec["eff_clock_ghz"] = round(xcd_cycles / rec["mean_ns"], 3)
        if agg.get("SQ_LDS_IDX_ACTIVE", 0) > 0 and "SQ_LDS_BANK_CONFLICT" in agg:
            rec["lds_conflict_frac"] = round(agg["SQ_LDS_BANK_CONFLICT"] / agg["SQ_LDS_IDX_ACTIVE"], 4)
        out[short[:120]] = rec
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
