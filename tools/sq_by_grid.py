"""Mean of each PMC counter per launch grid of one kernel over the
rocprofv3 counter_collection.csv files under a directory (tools/gpu_sq_rollwaves.sh)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root, name = sys.argv[1], sys.argv[2]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    per = defaultdict(float)   # (dispatch, grid, counter) -> value summed over dimensions
    for r in csv.DictReader(open(f)):
        if name not in r.get("Kernel_Name", ""):
            continue
        per[(r["Dispatch_Id"], r["Grid_Size"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, g, c), v in per.items():
        acc[g][c].append(v)
out = {g: {c: sum(v) / len(v) for c, v in cs.items()} for g, cs in acc.items()}
for g, cs in out.items():
    w = cs.get("SQ_WAVE_CYCLES")
    if w:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in cs:
                cs[c + "_frac"] = cs[c] / w
    if cs.get("SQ_BUSY_CYCLES") and cs.get("SQ_VALU_MFMA_BUSY_CYCLES"):
        cs["mfma_busy_frac"] = cs["SQ_VALU_MFMA_BUSY_CYCLES"] / cs["SQ_BUSY_CYCLES"]
print(json.dumps(out, indent=1, sort_keys=True))
