set -o pipefail
mkdir -p gpurun_out/r6a
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_corr_i8.py tests/test_gpu_dropin.py -k "world1 or tiny or schedules or c2_generation or pipelined or prefetch or two_ranks_one_device or exact" > gpurun_out/r6a/tests.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r6a/c3_bench.json 2> gpurun_out/r6a/c3_bench.err || exit 3
bash tools/gen_pmc_c2.sh gpurun_out/r6a/c2 || exit 4
echo all-done
