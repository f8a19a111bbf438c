#!/bin/bash
# Round validation on the box: the whole GPU suite, smoke(), the default bench line (C3, N = 1, the
# CPU baseline included), a rocprofv3 kernel-stats pass over a short C3 bench, the c2 line.
set -o pipefail
O=${1:-gpurun_out/r6round}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $O/gputests.log 2>&1 || exit 2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/c3_bench.json 2> $O/c3_bench.err || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o bench --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-cpu > $O/stats.log 2>&1 || exit 5
timeout -k 10 300 python3 -u bench.py --config c2 --steps 20 --warmup 3 > $O/c2_bench.json 2> $O/c2_bench.err || exit 6
echo round-done
