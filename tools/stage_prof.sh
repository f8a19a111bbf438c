# Kernel-trace profile of one generate pass (tools/stage_probe.py) on the GPU box.
# usage (inside gpurun): bash tools/yz_prof.sh [outdir]
set -o pipefail
OUT=${1:-gpurun_out/stageprof}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT -o stage --output-format csv -- python tools/stage_probe.py 256 256 4096 1 > $OUT.log 2>&1 || exit 2
echo done
