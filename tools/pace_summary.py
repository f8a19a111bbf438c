"""Summary of tools/pace_pmc.sh: per variant (paced, grid) the int8 SYRK's counters averaged per
launch, its kernel-trace duration, the L2 hit rate and MFMA busy fraction.
    python tools/pace_summary.py DIR > profiles/r5/pace_pmc.json"""
import csv
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1]
out = {}
for v in ("paced", "grid"):
    ctr = defaultdict(list)
    dur = []
    for grp in ("l2", "mfma"):
        base = os.path.join(d, v, grp)
        per = defaultdict(float)
        with open(os.path.join(base, "run_counter_collection.csv")) as f:
            for r in csv.DictReader(f):
                if "syrk" in r["Kernel_Name"]:
                    per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, name), val in per.items():
            ctr[name].append(val)
        with open(os.path.join(base, "run_kernel_trace.csv")) as f:
            for r in csv.DictReader(f):
                if "syrk" in r["Kernel_Name"]:
                    dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    avg = {k: sum(x) / len(x) for k, x in ctr.items()}
    hit = avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    # GRBM_GUI_ACTIVE is summed over the 8 XCD instances; 1024 SIMDs
    gui = avg["GRBM_GUI_ACTIVE"] / 8
    out[v] = {"launches": len(ctr["TCC_HIT_sum"]), "avg_duration_ms": sum(dur) / len(dur),
              "counters_per_launch": avg, "l2_hit_rate": hit,
              "l2_miss_bytes_per_launch_128B": avg["TCC_MISS_sum"] * 128,
              "gui_active_cycles_per_xcd": gui,
              "mfma_busy_frac": avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui * 1024),
              "wait_inst_frac": avg["SQ_WAIT_INST_ANY"] / avg["SQ_WAVE_CYCLES"]}
out["note"] = ("tools/pace_pmc.sh on tools/corr_i8_probe.py 256 256 4096 (C3 correlation, two passes); "
               "paced = k_syrk_i8_paced (persistent, XCD-paced), grid = k_syrk_i8 (PODS_SYRK_PACE=0); "
               "mfma_busy_frac assumes GRBM_GUI_ACTIVE summed over 8 XCDs and counts in the counter's own units: "
               "compare the two variants, not against the roofline")
print(json.dumps(out, indent=1))
