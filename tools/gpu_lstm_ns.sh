# BiLSTM sequences per workgroup A/B (ND_LSTM_SEQ = 16 / 8 / 4): every GPU
# test on the default, the nano tests on each value, the nano bench
# alternating, a kernel trace of NS=4
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/lstmns; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "assert|Error|FAIL" $O/tests.log | head -20; exit $rc; }
for v in 4 16; do
  ND_LSTM_SEQ=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k nano -p no:cacheprovider > $O/t$v.log 2>&1
  rc=$?; echo "SEQ=$v tests rc=$rc"; tail -1 $O/t$v.log; [ $rc -ne 0 ] && { grep -E "assert|Error|FAIL" $O/t$v.log | head -20; exit $rc; }
done
for v in 8 4 8 4; do
  ND_LSTM_SEQ=$v timeout -k 10 300 python bench.py --encoder nano --steps 5 --warmup 1 --cpu-baseline 0 > $O/b$v.json 2> $O/b$v.err
  rc=$?; python -c "import json; d=json.load(open('$O/b$v.json')); print('SEQ=$v nano ms/call', d['ms_per_step'], d['value'])"; [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp
ND_LSTM_SEQ=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --encoder nano --steps 3 --warmup 1 --cpu-baseline 0 > $O/trace.log 2>&1
echo "trace rc=$?"
