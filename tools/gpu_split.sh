# split-fp16 GEMMs: parity (GEMM + split images), timing (encoder + decoder shapes), full GPU suite
set -u
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "gemm_vs_fp64 or split_weight or gemm_p16" > gpurun_out/split_test.log 2>&1
rc=$?; tail -5 gpurun_out/split_test.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/microbench.py enc > gpurun_out/split_bench.log 2>&1
rc=$?; grep gemm gpurun_out/split_bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/microbench.py dec256 > gpurun_out/split_dec.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/split_dec.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/split_all.log 2>&1
rc=$?; tail -5 gpurun_out/split_all.log; exit $rc
