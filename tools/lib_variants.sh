#!/bin/bash
# Build libpodsgen variants with compile-time switches of the kernel files (podsgen_kernels.hip,
# podsgen_eigen.hip) into pods-digital-filter_amd/podsgen/variants/ for A/B runs in one GPU call
# (PODSGEN_LIB=.../libpodsgen_NAME.so):
#   bash tools/lib_variants.sh NAME "-DPODS_SYRK_SETPRIO=1" [NAME2 "FLAGS2" ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/pods-digital-filter_amd/csrc
OUT=$ROOT/pods-digital-filter_amd/podsgen/variants
OBJ=$ROOT/pods-digital-filter_amd/podsgen/.obj
mkdir -p $OUT/obj
FLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -I$ROOT/include -Wall -Wno-unused-function"
while [ $# -ge 2 ]; do
  name=$1; extra=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $FLAGS $extra -c $CS/podsgen_eigen.hip -o $OUT/obj/eigen_$name.o &
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $FLAGS $extra -c $CS/podsgen_kernels.hip -o $OUT/obj/kernels_$name.o &
  wait
  objs=$(ls $OBJ/*.o | grep -v -e podsgen_eigen.o -e podsgen_kernels.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs $OUT/obj/eigen_$name.o $OUT/obj/kernels_$name.o \
    -pthread -o $OUT/libpodsgen_$name.so
  echo built $OUT/libpodsgen_$name.so
done
