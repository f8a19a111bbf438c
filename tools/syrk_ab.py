"""A/B of libpodsgen variants (tools/lib_variants.sh) on pods_corr at C3 (tools/syrk_probe.py),
one process per variant, alternating twice: python tools/syrk_ab.py reps default prio ..."""
import os
import re
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..")


def run(name, reps):
    env = dict(os.environ)
    if name != "default":
        env["PODSGEN_LIB"] = os.path.join(ROOT, "pods-digital-filter_amd", "podsgen", "variants",
                                          "libpodsgen_%s.so" % name)
    r = subprocess.run([sys.executable, os.path.join(HERE, "syrk_probe.py"), "256", "256", "4096", str(reps)],
                       env=env, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        print(name, "FAILED", r.stderr[-2000:], flush=True)
        sys.exit(1)
    chk = re.findall(r"check max rel err (\S+) symmetric (\S+)", r.stdout)
    print(name, "check", chk, flush=True)
    return [float(m) for m in re.findall(r"corr ([0-9.]+) ms", r.stdout)][2:]


def main(reps, names):
    res = {n: [] for n in names}
    for _ in range(2):
        for n in names:
            res[n] += run(n, reps)
    for n in names:
        print("%-10s corr median %.2f ms  min %.2f ms  (%d runs)" % (n, statistics.median(res[n]), min(res[n]),
                                                                   len(res[n])), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]), sys.argv[2:])
