# k-step depth of the 64x64 long-K GEMM tiles (ND_GEMM_BKL): parity per value, microbench, beam bench
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/bkl; mkdir -p $O; cd $R
for x in ${VALS:-32 64 128}; do
  ND_GEMM_BKL=$x timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "gemm or beam_vs_golden" > $O/t$x.log 2>&1
  rc=$?; echo "== BKL=$x tests rc=$rc"; tail -1 $O/t$x.log; [ $rc -ne 0 ] && exit $rc
  ND_GEMM_BKL=$x timeout -k 10 200 python tools/microbench.py dec256 > $O/mb$x.log 2>&1
  rc=$?; grep "rm .*M= 5120.*K= 2048\|rm .*M= 1280.*K= 2048" $O/mb$x.log; [ $rc -ne 0 ] && exit $rc
  ND_GEMM_BKL=$x timeout -k 10 300 python bench.py --mode beam --batch 1024 --steps 2 --warmup 1 --cpu-baseline 0 --no-roofline > $O/b$x.json 2> $O/b$x.err
  rc=$?; python -c "import json; d=json.load(open('$O/b$x.json')); print('beam ms/call', d['ms_per_step'])"; [ $rc -ne 0 ] && exit $rc
done
exit 0
