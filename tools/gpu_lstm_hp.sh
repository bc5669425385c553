# BiLSTM h exchanged as split-fp16 planes: every GPU test, the nano bench
# twice, and a kernel trace of the nano bench (lstm_dir_kernel durations)
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/lstmhp; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "assert|Error|FAIL" $O/tests.log | head -20; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --encoder nano --steps 5 --warmup 1 --cpu-baseline 0 > $O/b$i.json 2> $O/b$i.err
  rc=$?; python -c "import json; d=json.load(open('$O/b$i.json')); print('nano ms/call', d['ms_per_step'], d['value'])"; [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --encoder nano --steps 3 --warmup 1 --cpu-baseline 0 > $O/trace.log 2>&1
echo "trace rc=$?"
