# A/B a tuning knob: microbench (dec256) under each ENV setting given as args, then the tests
set -u
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for kv in "$@"; do
  env $kv timeout -k 10 300 python tools/microbench.py dec256 > gpurun_out/ab.log 2>&1
  rc=$?; echo "== $kv rc=$rc"; grep -E "attn|gemm" gpurun_out/ab.log
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab.log; exit $rc; fi
done
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/t.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/t.log
