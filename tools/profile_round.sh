#!/bin/bash
# Round profiling recipe (run on the GPU box from the repo root):
#   bench JSON, rocprofv3 kernel-trace --stats of the bench command, and separate
#   --pmc passes (FETCH_SIZE, WRITE_SIZE) for the SYRK traffic.
set -o pipefail
OUT=${1:-gpurun_out/round}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/stats -o bench --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu > $OUT/stats.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python tools/syrk_probe.py 256 256 4096 2 > $OUT/pmc_fetch.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python tools/syrk_probe.py 256 256 4096 2 > $OUT/pmc_write.log 2>&1 || exit 4
echo profile-done
