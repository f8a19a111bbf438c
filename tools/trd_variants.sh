#!/bin/bash
# Build libpodsgen variants of the tridiagonalisation (podsgen_eigen.hip compile-time switches)
# into pods-digital-filter_amd/podsgen/variants/ for A/B runs (PODSGEN_LIB=...):
#   bash tools/trd_variants.sh NAME "-DPODS_TRD_SKIP_MIN_K=99" [NAME2 "FLAGS2" ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/pods-digital-filter_amd/csrc
OUT=$ROOT/pods-digital-filter_amd/podsgen/variants
mkdir -p $OUT/obj
FLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -I$ROOT/include -Wall -Wno-unused-function"
OBJ=$ROOT/pods-digital-filter_amd/podsgen/.obj
while [ $# -ge 2 ]; do
  name=$1; extra=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $FLAGS $extra -c $CS/podsgen_eigen.hip -o $OUT/obj/eigen_$name.o
  objs=$(ls $OBJ/*.o | grep -v podsgen_eigen.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs $OUT/obj/eigen_$name.o -pthread -o $OUT/libpodsgen_$name.so
  echo built $OUT/libpodsgen_$name.so
done
