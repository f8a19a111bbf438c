"""Per-kernel mean of every counter in rocprofv3 --pmc CSV passes:
python tools/pmc_summary.py DIR [kernel-substring]  (DIR holds p1/, p2/, ... run_counter_collection.csv)"""
import collections
import csv
import glob
import json
import os
import sys

src = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else ""
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(src, "*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if want and want not in k:
            continue
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in vals.items()}
print(json.dumps(out, indent=1))
