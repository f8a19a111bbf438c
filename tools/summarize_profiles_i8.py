"""Summarize a profile_round_i8.sh output dir into profiles/ (committed):
   python tools/summarize_profiles_i8.py gpurun_out/round_i8 r4 c3
Writes profiles/<tag>_<config>_kernel_stats.{csv,txt} and profiles/pmc_corr_i8_<config>.json
(k_syrk_i8's L2-to-fabric bytes per launch: the roofline 'traffic' bench.py reports)."""
import collections
import csv
import json
import os
import shutil
import sys

src, tag, config = sys.argv[1], sys.argv[2], sys.argv[3]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(ROOT, "profiles")
stats = os.path.join(src, "stats", "bench_kernel_stats.csv")
rows = list(csv.DictReader(open(stats)))
shutil.copy(stats, os.path.join(dst, "%s_%s_kernel_stats.csv" % (tag, config)))
lines = ["# rocprofv3 --kernel-trace --stats -- python bench.py --steps 3 --warmup 2 --no-cpu  (%s, %s)" % (tag, config),
         "%-70s %8s %12s %12s %8s" % ("kernel", "calls", "avg_us", "total_ms", "pct")]
for r in rows[:40]:
    lines.append("%-70s %8s %12.1f %12.2f %8.2f" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3,
                                                    float(r["TotalDurationNs"]) / 1e6, float(r["Percentage"])))
open(os.path.join(dst, "%s_%s_kernel_stats.txt" % (tag, config)), "w").write("\n".join(lines) + "\n")


def pmc(d, counter):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(src, d, "run_counter_collection.csv"))):
        if r["Counter_Name"] == counter:
            vals[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return vals


f = pmc("pmc_fetch", "FETCH_SIZE")
w = pmc("pmc_write", "WRITE_SIZE")
ns, K = 4096, 3 * 256 * 256
res = {"tag": tag, "config": config,
       "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over tools/corr_i8_probe.py "
                 "256 256 4096; bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (FETCH_SIZE reads half of 16-B/lane "
                 "streaming loads, LDS-DMA included, on gfx950: MI355X_MICROARCH.md HBM section); FETCH_SIZE counts "
                 "Infinity-Cache-served lines too, so this is L2-miss traffic (HBM + Infinity Cache)",
       "kernels": {}}
total = 0.0
for k in sorted(set(f) | set(w)):
    fk = sum(f.get(k, [0])) / max(len(f.get(k, [1])), 1)
    wk = sum(w.get(k, [0])) / max(len(w.get(k, [1])), 1)
    b = (2 * fk + wk) * 1024
    res["kernels"][k] = {"FETCH_SIZE_kB": fk, "WRITE_SIZE_kB": wk, "bytes": b}
    if "k_syrk_i8" in k:
        total += b
res["hbm_bytes_per_launch"] = total
res["algorithmic_bytes_per_launch"] = 16 * ns * K + 16 * ns * ns  # residues read once + one byte per modulus out
json.dump(res, open(os.path.join(dst, "pmc_corr_i8_%s.json" % config), "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))
print("\n".join(lines[:16]))
