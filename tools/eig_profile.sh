# rocprofv3 kernel stats of pods_syev at n = 4096 (run inside gpurun from the repo root)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/eigprof -o eig --output-format csv -- python tools/eig_probe.py 4096 > gpurun_out/eigprof.log 2>&1 || exit 2
echo done
