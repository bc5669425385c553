# BiLSTM recurrence: parity (nano golden, ragged oracle, op-level vs torch.nn.LSTM) + the nano bench's per-step timing
cd $GRAFT_REPO_ROOT && O=$GRAFT_REPO_ROOT/gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "nano or lstm" > $O/t_lstm.log 2>&1; rc=$?; tail -2 $O/t_lstm.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --encoder nano --steps 40 --warmup 3 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 > $O/b_lstm.json 2> $O/b_lstm.err; rc=$?
python3 -c "
import json; d=json.loads(open('$O/b_lstm.json').read().strip().splitlines()[-1]); l=d['roofline']['lstm_kernel']
print('nano %.3f ms/call, lstm layer %.3f ms, %.3f us/step' % (d['ms_per_step'], l['avg_launch_ms'], l['us_per_step']))"
exit $rc
