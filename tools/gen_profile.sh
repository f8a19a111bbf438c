set -o pipefail
OUT=${1:-gpurun_out/genprof}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o gen --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu > $OUT.log 2>&1 || exit 2
echo done
