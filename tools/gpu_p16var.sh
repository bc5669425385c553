# decoder P16 GEMM slicing A/B (ND_P16_VARIANT bits; the knob was removed from
# gemm.hip after this A/B showed no change): GEMM parity
# under each variant, then the greedy bench alternating variants, then a
# kernel trace of the best guess
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/p16var; mkdir -p $O; cd $R
for v in 3; do
  ND_P16_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "p16 or greedy" -p no:cacheprovider > $O/t$v.log 2>&1
  rc=$?; echo "tests v=$v rc=$rc"; tail -1 $O/t$v.log; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/t$v.log | head; exit $rc; }
done
for v in 0 1 2 3 0 1 2 3; do
  ND_P16_VARIANT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-baseline 0 --no-roofline > $O/b$v.json 2> $O/b$v.err
  rc=$?; python -c "import json; d=json.load(open('$O/b$v.json')); print('v=$v ms/call', d['ms_per_step'])"; [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp
ND_P16_VARIANT=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --no-roofline > $O/trace.log 2>&1
echo "trace rc=$?"
