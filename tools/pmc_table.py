"""Per-kernel FETCH/WRITE bytes from tools/gen_pmc.sh output: python tools/pmc_table.py gpurun_out/genpmc"""
import collections, csv, os, sys
src = sys.argv[1]
def pmc(d, counter):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(src, d, "run_counter_collection.csv"))):
        if r["Counter_Name"] == counter:
            vals[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return vals
f, w = pmc("fetch", "FETCH_SIZE"), pmc("write", "WRITE_SIZE")
for k in sorted(set(f) | set(w), key=lambda k: -sum(f.get(k, [0]))):
    fk = sum(f.get(k, [0])) / max(len(f.get(k, [1])), 1)
    wk = sum(w.get(k, [0])) / max(len(w.get(k, [1])), 1)
    print("%-55s fetch(x2) %8.2f GB  write %8.2f GB" % (k[:55], 2 * fk * 1024 / 1e9, wk * 1024 / 1e9))
