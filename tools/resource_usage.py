"""Per-kernel register/LDS/spill report from hipcc -Rpass-analysis=kernel-resource-usage (the same
flags as csrc/Makefile), one row per kernel instantiation:
    python tools/resource_usage.py podsgen_eigen podsgen_corr_i8 ... > profiles/r5/resource_usage.txt"""
import re
import subprocess
import sys

CSRC = "pods-digital-filter_amd/csrc"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-I../../include", "-Wno-unused-function",
         "--offload-arch=gfx950", "-Rpass-analysis=kernel-resource-usage", "-c", "-o", "/dev/null"]
FIELDS = ("VGPRs", "AGPRs", "TotalSGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]",
          "Occupancy [waves/SIMD]", "LDS Size [bytes/block]")
print("%-72s %5s %5s %5s %6s %6s %7s %4s %7s" % ("kernel", "vgpr", "agpr", "sgpr", "vspill", "sspill",
                                                 "scratch", "occ", "lds"))
for src in sys.argv[1:]:
    r = subprocess.run(["/opt/rocm/bin/hipcc", src + ".hip"] + FLAGS, cwd=CSRC, capture_output=True, text=True)
    cur, rows = None, []
    for line in r.stderr.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([^:]+): (\S+) \[", line)
        if m and cur is not None and m.group(1) in FIELDS:
            cur[m.group(1)] = m.group(2)
    dem = subprocess.run(["c++filt"], input="\n".join(x["name"] for x in rows),
                         capture_output=True, text=True).stdout.splitlines()
    print("# %s.hip" % src)
    for x, d in zip(rows, dem):
        d = re.sub(r"\(.*\)$", "", d.replace("pods::", ""))
        print("%-72s %5s %5s %5s %6s %6s %7s %4s %7s" % ((d[:72],) + tuple(x.get(f, "?") for f in FIELDS)))
