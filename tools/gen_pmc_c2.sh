#!/bin/bash
# BASELINE config 2 (generation only) on the GPU box, from the repo root:
#   bash tools/gen_pmc_c2.sh gpurun_out/c2
# kernel-trace --stats of the c2 bench, then one rocprofv3 --pmc pass per counter (FETCH_SIZE,
# WRITE_SIZE) over the same command; python tools/summarize_gen_pmc.py OUT TAG writes
# profiles/pmc_gen_c2.json (the per-kernel traffic bench.py --config c2 reports).
set -o pipefail
OUT=${1:-gpurun_out/c2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CMD="python3 bench.py --config c2 --steps 4 --warmup 1 --no-cpu"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- $CMD > $OUT/stats.log 2>&1 || exit 2
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- $CMD > $OUT/pmc_fetch.log 2>&1 || exit 3
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- $CMD > $OUT/pmc_write.log 2>&1 || exit 4
echo c2-profile-done
