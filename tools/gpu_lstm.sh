# BiLSTM cell activations A/B (ND_LSTM_LIBM 0 / 1): nano parity per value, then the nano bench
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/lstm; mkdir -p $O; cd $R
for x in 0 1; do
  ND_LSTM_LIBM=$x timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "nano" > $O/t$x.log 2>&1
  rc=$?; echo "== LSTM_LIBM=$x tests rc=$rc"; tail -1 $O/t$x.log; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/t$x.log | head; exit $rc; }
done
for x in 0 1 0 1; do
  ND_LSTM_LIBM=$x timeout -k 10 300 python bench.py --encoder nano --steps 3 --warmup 1 --cpu-baseline 0 --no-roofline > $O/b$x.json 2> $O/b$x.err
  rc=$?; python -c "import json; d=json.load(open('$O/b$x.json')); print('LSTM_LIBM=$x nano ms/call', d['ms_per_step'])"; [ $rc -ne 0 ] && exit $rc
done
exit 0
