#!/bin/bash
# Round profiling recipe for the int8 correlation (run on the GPU box from the repo root):
#   rocprofv3 kernel-trace --stats of the bench command, and separate --pmc passes (FETCH_SIZE,
#   WRITE_SIZE) of the correlation probe for k_syrk_i8's traffic.  Summary:
#   python tools/summarize_profiles_i8.py OUT TAG c3
set -o pipefail
OUT=${1:-gpurun_out/round_i8}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/stats -o bench --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu > $OUT/stats.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python tools/corr_i8_probe.py 256 256 4096 2 > $OUT/pmc_fetch.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python tools/corr_i8_probe.py 256 256 4096 2 > $OUT/pmc_write.log 2>&1 || exit 4
echo profile-done
