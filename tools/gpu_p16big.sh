# P16 GEMMs: parity incl. the large-M route, then decoder-shape timing
set -u
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "gemm_p16" > gpurun_out/p16big_test.log 2>&1
rc=$?; tail -4 gpurun_out/p16big_test.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/microbench.py dec256 > gpurun_out/p16big.log 2>&1
rc=$?; grep gemm gpurun_out/p16big.log; exit $rc
