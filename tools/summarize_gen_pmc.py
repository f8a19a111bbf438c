"""Summarize tools/gen_pmc_c2.sh output into profiles/ (committed):
   python tools/summarize_gen_pmc.py gpurun_out/c2 r6
Writes profiles/<tag>/c2_kernel_stats.txt and profiles/pmc_gen_c2.json: per generator kernel the
L2-miss bytes per launch, (2*FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md HBM section: on
gfx950 FETCH_SIZE reports half the bytes of 16-B/lane streaming reads), and the algorithmic bytes."""
import collections
import csv
import glob
import json
import os
import sys

src, tag = sys.argv[1], sys.argv[2]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.makedirs(os.path.join(ROOT, "profiles", tag), exist_ok=True)
stats = glob.glob(os.path.join(src, "stats", "**", "*kernel_stats.csv"), recursive=True)[0]
rows = list(csv.DictReader(open(stats)))
lines = ["# rocprofv3 --kernel-trace --stats -- python3 bench.py --config c2 --steps 4 --warmup 1 --no-cpu (%s)" % tag,
         "%-70s %8s %12s %12s %8s" % ("kernel", "calls", "avg_us", "total_ms", "pct")]
for r in rows[:30]:
    lines.append("%-70s %8s %12.1f %12.2f %8.2f" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3,
                                                    float(r["TotalDurationNs"]) / 1e6, float(r["Percentage"])))
open(os.path.join(ROOT, "profiles", tag, "c2_kernel_stats.txt"), "w").write("\n".join(lines) + "\n")


def pmc(d, counter):
    vals = collections.defaultdict(list)
    f = glob.glob(os.path.join(src, d, "**", "*counter_collection.csv"), recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter:
            vals[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return vals


import bench  # noqa: E402
f = pmc("pmc_fetch", "FETCH_SIZE")
w = pmc("pmc_write", "WRITE_SIZE")
J, K, ns = 256, 256, 4096
bpu = bench.gen_bytes_per_unit(J, K, ns, 6, 6, 6)
alg = {"k_mt_generate_full": bpu["gen_planes"], "k_filter_x2": bpu["gen_xpass"], "k_filter_yz": bpu["gen_yzpass"]}
res = {"tag": tag, "config": "c2",
       "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over bench.py --config c2; "
                 "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 per launch (FETCH_SIZE reads half of 16-B/lane streaming "
                 "loads on gfx950: MI355X_MICROARCH.md HBM section); FETCH_SIZE counts Infinity-Cache-served lines "
                 "too, so this is L2-miss traffic (HBM + Infinity Cache)",
       "kernels": {}}
for k in sorted(set(f) | set(w)):
    if "pods::" not in k:
        continue
    fk = sum(f.get(k, [0])) / max(len(f.get(k, [1])), 1)
    wk = sum(w.get(k, [0])) / max(len(w.get(k, [1])), 1)
    ent = {"FETCH_SIZE_kB": fk, "WRITE_SIZE_kB": wk, "bytes": (2 * fk + wk) * 1024}
    for name, b in alg.items():
        if name in k:
            ent["algorithmic_bytes"] = b * J * K * ns
    res["kernels"][k] = ent
res["total_bytes_per_step"] = sum(v["bytes"] for v in res["kernels"].values())
res["output_bytes_per_step"] = 24.0 * J * K * ns
json.dump(res, open(os.path.join(ROOT, "profiles", "pmc_gen_c2.json"), "w"), indent=1)
print(json.dumps({k: v for k, v in res.items()}, indent=1))
print("\n".join(lines[:12]))
