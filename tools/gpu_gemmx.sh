# encoder GEMM timing experiments: ND_GEMM_EXPT 0/1/2/4/6 (1 no epilogue, 2 no MFMA, 4 no loads; timing only)
set -u
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for x in ${EXPTS:-0 1 2 4 6}; do
  ND_GEMM_EXPT=$x timeout -k 10 120 python tools/microbench.py enc > gpurun_out/gemmx_$x.log 2>&1
  rc=$?; echo "== EXPT=$x rc=$rc"; grep gemm gpurun_out/gemmx_$x.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
