#!/bin/bash
# rocprofv3 kernel stats of pods_syev2 at one n (values + 20 vectors, then values only):
#   bash tools/syev2_prof.sh N OUTDIR
set -o pipefail
N=${1:-8192}; OUT=${2:-gpurun_out/syev2_$N}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python tools/syev2_probe.py $N > $OUT.log 2>&1 || exit 1
echo prof-ok
