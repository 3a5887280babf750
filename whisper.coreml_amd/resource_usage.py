"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin) as a table."""
import re
import sys

cur = {}
rows = []
for line in sys.stdin:
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                  r"SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    else:
        cur[k] = v
for r in rows:
    print(f"{r.get('VGPRs','?'):>4} vgpr {r.get('VGPRs Spill','?'):>3} spill {r.get('ScratchSize [bytes/lane]','?'):>4} scr "
          f"{r.get('Occupancy [waves/SIMD]','?'):>2} occ {r.get('LDS Size [bytes/block]','?'):>6} lds  {r['name'][:90]}")
