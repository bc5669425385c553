# quick greedy bench + kernel stats (rocprofv3 --kernel-trace --stats)
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/b1; mkdir -p $O; cd $R
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-baseline 0 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json | cut -c1-400; if [ $rc -ne 0 ]; then tail -5 $O/bench.err; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --no-roofline > $O/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
