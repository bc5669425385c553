# encoder GEMM XCD-aware tile order A/B (ND_GEMM_XCD 1 / 0) + GEMM parity
set -u
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "gemm_vs_fp64" > gpurun_out/xcd_test.log 2>&1
rc=$?; tail -3 gpurun_out/xcd_test.log; [ $rc -ne 0 ] && exit $rc
for x in 1 0; do
  ND_GEMM_XCD=$x timeout -k 10 120 python tools/microbench.py enc > gpurun_out/xcd_$x.log 2>&1
  rc=$?; echo "== xcd $x rc=$rc"; grep gemm gpurun_out/xcd_$x.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
