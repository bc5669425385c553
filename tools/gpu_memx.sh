# memory-bank attention: kernel parity, then timing experiments ND_MEM_EXPT 0/1/2/3 (1 no loads, 2 no MFMA; timing only)
set -u
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "mem_attention or greedy_vs_golden or memory_bank or nano_greedy" > gpurun_out/memtest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/memtest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for x in ${EXPTS:-0 1 2 3}; do
  ND_MEM_EXPT=$x timeout -k 10 120 python tools/microbench.py mem > gpurun_out/memx_$x.log 2>&1
  rc=$?; echo "== EXPT=$x rc=$rc"; grep mem-attn gpurun_out/memx_$x.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
