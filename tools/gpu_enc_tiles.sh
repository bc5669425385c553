# encoder GEMM tile A/B (split-fp16 and fp32): default 256x256 vs ND_GEMM_TILE=128
set -u
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for t in 256 128; do
  ND_GEMM_TILE=$t timeout -k 10 120 python tools/microbench.py enc > gpurun_out/enc_tile_$t.log 2>&1
  rc=$?; echo "== tile $t rc=$rc"; grep gemm gpurun_out/enc_tile_$t.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
