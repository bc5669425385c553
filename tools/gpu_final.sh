# end-of-session check on the committed tree: smoke, every GPU test, the three
# bench lines, a kernel trace of the headline bench
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/final; mkdir -p $O; cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $O/bench_greedy.json 2> $O/bench_greedy.err
rc=$?; echo "bench greedy rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --mode beam --batch 1024 --steps 3 --warmup 1 > $O/bench_beam.json 2> $O/bench_beam.err
rc=$?; echo "bench beam rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --encoder nano --steps 5 --warmup 1 --cpu-chunks 256 > $O/bench_nano.json 2> $O/bench_nano.err
rc=$?; echo "bench nano rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --cpu-baseline 0 > $O/trace.log 2>&1
echo "trace rc=$?"
