#!/bin/bash
# r6 measurement call: k_trd per-column trace and hop view at n = 4096; the int8 SYRK of this build
# against the r5 build (same box, alternating processes); MFMA counter calibration.
set -o pipefail
O=gpurun_out/r6b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=pods-digital-filter_amd/podsgen/variants
timeout -k 10 200 python -u tools/trd_trace.py 4096 0 100 255 > $O/trd_trace.log 2>&1 || exit 2
timeout -k 10 200 python -u tools/trd_hop.py 4096 > $O/trd_hop.log 2>&1 || exit 3
for i in 1 2; do
  timeout -k 10 200 python -u tools/corr_i8_ab.py 5 - > $O/syrk_new_$i.log 2>&1 || exit 4
  PODSGEN_LIB=$V/r5/libpodsgen.so timeout -k 10 200 python -u tools/corr_i8_ab.py 5 - > $O/syrk_r5_$i.log 2>&1 || exit 5
done
PODSGEN_LIB=$V/libpodsgen_diag.so timeout -k 10 300 python -u tools/corr_i8_ab.py 5 - PODS_SYRK_I8=g PODS_SYRK_I8=9d PODS_SYRK_I8=9m > $O/syrk_diag.log 2>&1 || exit 6
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -o "SQ_INSTS_VALU_MFMA[A-Z0-9_]*\|SQ_VALU_MFMA[A-Z0-9_]*\|SQ_INSTS_MFMA[A-Z0-9_]*" $O/counters.txt | sort -u > $O/mfma_counters.txt || true
if grep -q "^SQ_INSTS_VALU_MFMA_MOPS_I8$" $O/mfma_counters.txt; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_mops -o run --output-format csv -- python tools/corr_i8_probe.py 256 256 4096 2 > $O/pmc_mops.log 2>&1 || exit 7
fi
if grep -q "^SQ_INSTS_VALU_MFMA_I8$" $O/mfma_counters.txt; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_I8 SQ_INSTS_MFMA --kernel-trace -d $O/pmc_insts -o run --output-format csv -- python tools/corr_i8_probe.py 256 256 4096 2 > $O/pmc_insts.log 2>&1 || exit 8
fi
echo call2-done
