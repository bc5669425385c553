# full measurement pass: tests, benches (greedy / beam / nano), kernel trace, PMC
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/full
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > $O/bench_greedy.json 2> $O/bench_greedy.err
rc=$?; echo "bench greedy rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --mode beam --batch 1024 --steps 3 --warmup 1 > $O/bench_beam.json 2> $O/bench_beam.err
rc=$?; echo "bench beam rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --encoder nano --steps 5 --warmup 1 --cpu-chunks 256 > $O/bench_nano.json 2> $O/bench_nano.err
rc=$?; echo "bench nano rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --cpu-baseline 0 > $O/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --cpu-baseline 0 > $O/pmc_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --cpu-baseline 0 > $O/pmc_write.log 2>&1
echo "pmc write rc=$?"
