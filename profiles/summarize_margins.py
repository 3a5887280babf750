"""Fold one GPU run's tolerance margins (gpurun_out/margins.jsonl, written by the GPU
tests through tests/conftest.py:record_margin) into a committed JSON:

    python profiles/summarize_margins.py gpurun_out/margins.jsonl profiles/r06/fp16_margins.json

The summary lists every teacher-forced case with its worst relative error as a fraction of
its bound (tau), the step / row where it occurred and the top-1 agreement, the first-pass
logit cases, the free-running agreement cases and the word-timestamp cases, and flags every
case above half its bound."""
import json
import sys


def main(src, dst):
    recs = [json.loads(line) for line in open(src) if line.strip()]
    tf = [r for r in recs if r["test"] == "teacher_forced"]
    logit = [r for r in recs if r["test"] in ("first_step_logits", "prompt_prefill_logits")]
    out = {
        "source": src,
        "cases": len(recs),
        "teacher_forced": sorted(tf, key=lambda r: -r["frac_of_tau"]),
        "first_pass_logits": sorted(logit, key=lambda r: -r["frac_of_tau"]),
        "free_running": [r for r in recs if r["test"] in ("fp16_natural_greedy", "fp16_fixed_greedy")],
        "words": [r for r in recs if r["test"].startswith("fp16_words") or r["test"] == "fp16_beam_words_tokens"],
    }
    summ = {}
    for dt in ("fp16", "fp32"):
        c = [r for r in tf if r["dtype"] == dt]
        if c:
            w = max(c, key=lambda r: r["frac_of_tau"])
            summ[dt] = {"cases": len(c), "worst_rel": w["worst_rel"], "tau": w["tau"], "frac_of_tau": w["frac_of_tau"],
                        "worst_case": {k: w[k] for k in ("model", "kind", "windows", "mixed", "worst_step", "worst_row")},
                        "min_top1_agreement": min(r["top1_agreement"] for r in c)}
    out["summary"] = summ
    out["above_half_tau"] = [r for r in tf + logit if r["frac_of_tau"] > 0.5]
    json.dump(out, open(dst, "w"), indent=1)
    for dt, s in summ.items():
        print(f"{dt}: {s['cases']} teacher-forced cases, worst rel {s['worst_rel']:.3e} = {s['frac_of_tau']:.3f} tau "
              f"({s['worst_case']}), min top-1 agreement {s['min_top1_agreement']:.4f}")
    print(f"cases above 0.5 tau: {len(out['above_half_tau'])}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
