# op-level BiLSTM parity (nd_op_lstm_layer vs torch.nn.LSTM) at every
# sequences-per-workgroup setting, the whole GPU suite, the nano bench with
# its lstm_kernel view
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/lstmop; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "assert|Error|FAIL" $O/tests.log | head -20; exit $rc; }
for v in 8 16; do
  ND_LSTM_SEQ=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k nano -p no:cacheprovider > $O/t$v.log 2>&1
  rc=$?; echo "SEQ=$v tests rc=$rc"; tail -1 $O/t$v.log; [ $rc -ne 0 ] && { grep -E "assert|Error|FAIL" $O/t$v.log | head -20; exit $rc; }
done
timeout -k 10 300 python bench.py --encoder nano --steps 5 --warmup 1 --cpu-chunks 256 > $O/nano.json 2> $O/nano.err
rc=$?; echo "nano bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
python -c "import json; d=json.load(open('$O/nano.json')); print(d['ms_per_step'], d['value'], d['roofline']['lstm_kernel'])"
