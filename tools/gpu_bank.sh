# memory-bank attention: op-level parity (fp32 + split-fp16 forms) and the microbench
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "mem_attention or bank_h3 or greedy" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $O/bank_test.log 2>&1; rc=$?
tail -15 $O/bank_test.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/microbench.py mem > $O/bank_mb.log 2>&1; rc=$?
grep -E "mem-attn|bank-h3" $O/bank_mb.log; exit $rc
