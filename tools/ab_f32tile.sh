#!/bin/bash
# fp32 GEMM tile variants (build_variant.sh gemm.hip -DND_F32_TILE=...) on the encoder's shapes, microbench "enc"
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for v in "$@"; do
  echo "== $v"
  NANODEC_AB=1 NANODEC_LIB=$R/tools/_ab/$v.so timeout -k 10 200 python -u tools/microbench.py enc > $O/ab_f32tile_$v.log 2>&1 || exit $?
  grep -v split $O/ab_f32tile_$v.log | grep gemm
done
