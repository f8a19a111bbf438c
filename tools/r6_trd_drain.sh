#!/bin/bash
# Is the hand-off wait the consumer's own store queue?  The same k_trd with every wave's stores
# drained at the top of each column (variant 'drain') against the product build: traces + syev time.
set -o pipefail
O=${1:-gpurun_out/r6e}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=pods-digital-filter_amd/podsgen/variants
timeout -k 10 120 python -u tools/syev_ab.py 10 > $O/syev_prod.log 2>&1 || exit 2
PODSGEN_LIB=$V/libpodsgen_drain.so timeout -k 10 120 python -u tools/syev_ab.py 10 > $O/syev_drain.log 2>&1 || exit 3
timeout -k 10 200 python -u tools/trd_trace.py 4096 0 > $O/trace_prod.log 2>&1 || exit 4
PODSGEN_LIB=$V/libpodsgen_drain.so timeout -k 10 200 python -u tools/trd_trace.py 4096 0 > $O/trace_drain.log 2>&1 || exit 5
PODSGEN_LIB=$V/libpodsgen_drain.so timeout -k 10 200 python -u tools/trd_hop.py 4096 > $O/hop_drain.log 2>&1 || exit 6
timeout -k 10 200 python -u tools/trd_hop.py 4096 > $O/hop_prod.log 2>&1 || exit 7
echo drain-done
