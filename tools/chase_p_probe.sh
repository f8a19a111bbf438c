#!/bin/bash
# pods_syev2 at n = 4096 with the bulge chase on all CUs and on 64 / 32 / 16 workgroups
# (PODS_CHASE_P): kernel stats per setting.  bash tools/chase_p_probe.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/chasep}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for p in 256 64 32 16; do
  PODS_CHASE_P=$p timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/p$p -o run --output-format csv -- python tools/syev2_probe.py 4096 > $OUT/p$p.log 2>&1 || exit 1
done
echo chase-done
