#!/bin/bash
# Dev A/B of top-k kernel variants (NOT product code): each variant's topk.hip is
# compiled into its own tools/ab/libtk_<tag>.so exposing ab_topk() = its als_topk.
#   base = the committed kernel (git HEAD)
#   new  = the working-tree kernel
#   TAG='sed expression' arguments: the working-tree kernel with that edit applied
set -e
cd "$(dirname "$0")"
CSRC=../../recommender-system-using-apache-spark-mllib-_amd/csrc
rm -f libtk_*.so tk_*.hip ab_*.hip
git show HEAD:recommender-system-using-apache-spark-mllib-_amd/csrc/topk.hip > tk_base.hip
cp $CSRC/topk.hip tk_new.hip
tags="base new"
for a in "$@"; do
  t=${a%%=*}; e=${a#*=}
  sed "$e" $CSRC/topk.hip > tk_$t.hip
  if cmp -s tk_$t.hip $CSRC/topk.hip; then echo "variant $t: sed changed nothing" >&2; exit 1; fi
  tags="$tags $t"
done
for v in $tags; do
  cat > ab_$v.hip <<EOT
#include "tk_$v.hip"
namespace als { void set_error(const char*, ...) {} }
extern "C" int ab_topk(const float* Q, int64_t n_q, const float* V, int64_t n_v, int ld, int k,
                       int top, int32_t* idx, float* sc, void* ws, size_t ws_bytes, void* st) {
  return als_topk(Q, n_q, V, n_v, ld, k, top, idx, sc, ws, ws_bytes, st);
}
extern "C" size_t ab_ws(int64_t n_q, int64_t n_v, int k, int top) {
  return als_topk_workspace_bytes(n_q, n_v, k, top);
}
EOT
  /opt/rocm/bin/hipcc -O3 -fPIC -shared -std=c++17 --offload-arch=gfx950 -I$CSRC ab_$v.hip -o libtk_$v.so &
done
wait
ls libtk_*.so
echo "$tags" > variants.txt
