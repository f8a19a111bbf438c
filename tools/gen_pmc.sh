#!/bin/bash
# PMC traffic of the generator kernels (one pass per counter group), from the repo root on the box:
#   bash tools/gen_pmc.sh gpurun_out/genpmc
set -o pipefail
OUT=${1:-gpurun_out/genpmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- python tools/stage_probe.py 256 256 4096 1 > $OUT/fetch.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv -- python tools/stage_probe.py 256 256 4096 1 > $OUT/write.log 2>&1 || exit 3
echo pmc-done
