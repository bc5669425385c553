set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/trace; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --no-roofline ${BENCH_ARGS:-} > $O/log 2>&1
echo "trace rc=$?"
