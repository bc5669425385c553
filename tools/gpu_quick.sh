# GPU suite + quick greedy bench with kernel stats
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/q; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-baseline 0 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 $O/bench.json; [ $rc -ne 0 ] && { tail -5 $O/bench.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --no-roofline > $O/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
