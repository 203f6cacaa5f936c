#!/bin/bash
# Dev A/B of solve-kernel variants (NOT product code): the working-tree library built
# with extra -D flags into tools/ab/libals_<tag>.so (same ABI; loaded through ALS_HIP_LIB
# by tools/ab_solve.py).  Usage: bash tools/ab/build_solve.sh tag='-DX=1 -DY=0' ...
set -e
cd "$(dirname "$0")"
CSRC=${CSRC:-../../recommender-system-using-apache-spark-mllib-_amd/csrc}
for a in "$@"; do
  t=${a%%=*}; f=${a#*=}
  mkdir -p obj_$t
  for s in csr_build gram_solve predict topk; do
    /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 $f -c $CSRC/$s.hip -o obj_$t/$s.o &
  done
  wait
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 obj_$t/*.o -o libals_$t.so
  rm -rf obj_$t
  echo "built libals_$t.so ($f)"
done
