set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/eig_probe.py 513 1000 1025 2048 2049 2500 3000 3585 4096 > gpurun_out/eig2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/eigprof -o eig --output-format csv -- python tools/eig_probe.py 4096 > gpurun_out/eigprof.log 2>&1 || exit 2
echo done
