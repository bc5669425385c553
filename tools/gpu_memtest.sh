# memory-bank attention: kernel parity, greedy parity, then the microbench
set -u
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "mem_attention or greedy_vs_golden or memory_bank or nano_greedy" > gpurun_out/memtest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/memtest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python tools/microbench.py mem > gpurun_out/mem.log 2>&1
rc=$?; echo "mem rc=$rc"; grep mem-attn gpurun_out/mem.log; exit $rc
