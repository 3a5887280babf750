import json, os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "tests")]
import numpy as np
from conftest import full_model, GOLDEN
import whisper
from whisper import synthetic as S
g = json.load(open(os.path.join(GOLDEN, "large-v3_words.json")))
m = full_model("large-v3", "fp32")
audio = S.synthetic_audio(65.0, seed=7)
out = {}
for sched in ["batched", "sequential"]:
    r = whisper.transcribe(m, audio, temperature=0.0, language="en", schedule=sched, **g["runs"]["clip_greedy_words"])
    out[sched] = [dict(seek=s["seek"], start=s["start"], end=s["end"], tokens=s["tokens"], words=s["words"])
                  for s in r["segments"]]
    print(sched, len(r["segments"]), flush=True)
# decode-only, no words
r = whisper.transcribe(m, audio, temperature=0.0, language="en", condition_on_previous_text=False,
                       clip_timestamps="0,30,30,60,60")
out["nowords"] = [dict(seek=s["seek"], start=s["start"], end=s["end"], tokens=s["tokens"]) for s in r["segments"]]
os.makedirs("gpurun_out", exist_ok=True)
json.dump(out, open("gpurun_out/lv3_words_dbg.json", "w"))
