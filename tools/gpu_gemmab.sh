# encoder GEMM A/B: 256x256 tiles (default) vs 128x128 (ND_GEMM_TILE=128), then the GEMM parity tests
set -u
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "gemm" > gpurun_out/gemmtest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gemmtest.log; if [ $rc -ne 0 ]; then exit $rc; fi
for t in 256 128; do
  ND_GEMM_TILE=$t timeout -k 10 120 python tools/microbench.py enc > gpurun_out/gemmab_$t.log 2>&1
  rc=$?; echo "== tile $t rc=$rc"; grep gemm gpurun_out/gemmab_$t.log; if [ $rc -ne 0 ]; then exit $rc; fi
done
