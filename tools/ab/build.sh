#!/bin/bash
# Dev A/B of top-k kernel variants (NOT product code): each variant's topk.hip is
# compiled into its own tools/ab/libtk_<tag>.so exposing ab_topk() = its als_topk.
#   v0 = round-2 kernel (register staging, quad lists with one row group)
#   v1 = bf088e3 (register staging, quad lists with two row groups)
#   v2 = HEAD (LDS-DMA staging, quad two row groups)
#   v3 = HEAD with one row group for quad lists
set -e
cd "$(dirname "$0")"
CSRC=../../recommender-system-using-apache-spark-mllib-_amd/csrc
git show ad16911:recommender-system-using-apache-spark-mllib-_amd/csrc/topk.hip > tk_v0.hip
git show bf088e3:recommender-system-using-apache-spark-mllib-_amd/csrc/topk.hip > tk_v1.hip
cp $CSRC/topk.hip tk_v2.hip
sed 's|  if (quad) return 2;  // quad lists: two row groups (each V tile feeds 128 query rows)|  if (quad) return 1;|' $CSRC/topk.hip > tk_v3.hip
grep -q "if (quad) return 1;" tk_v3.hip
for v in v0 v1 v2 v3; do
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
ls -la libtk_*.so
