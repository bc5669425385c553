# encoder GEMM A/B of an environment knob: KNOB=ND_GEMM_XCD VALS="1 0" bash tools/gpu_knob.sh
set -u
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "${TESTS:-gemm_vs_fp64}" > gpurun_out/knob_test.log 2>&1
rc=$?; tail -3 gpurun_out/knob_test.log; [ $rc -ne 0 ] && exit $rc
for x in ${VALS:-1 0}; do
  env $KNOB=$x timeout -k 10 120 python tools/microbench.py ${MODE:-enc} > gpurun_out/knob_$x.log 2>&1
  rc=$?; echo "== $KNOB=$x rc=$rc"; grep "gemm\|attn" gpurun_out/knob_$x.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
