# quick iteration: GPU parity tests, decoder-shape microbench, short bench
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/quick; mkdir -p $O; cd $R
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider -x > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/microbench.py ${MICRO:-dec256} > $O/micro.log 2>&1; echo "micro rc=$?"
if [ $? -gt 1 ]; then exit 1; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --no-roofline > $O/bench.json 2> $O/bench.err
echo "bench rc=$?"
