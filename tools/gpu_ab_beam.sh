# beam-bench A/B of an environment knob with per-kernel times (kernel trace)
# KNOB=ND_SELF_XCD VALS="1 0" bash tools/gpu_ab_beam.sh
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/abb; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for x in ${VALS:-1 0}; do
  env $KNOB=$x timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t$x -o run --output-format csv -- python3 $R/bench.py --mode beam --batch 1024 --steps 1 --warmup 1 --cpu-baseline 0 --no-roofline > $O/b$x.json 2> $O/b$x.err
  rc=$?; echo "== $KNOB=$x rc=$rc"; cut -c1-200 $O/b$x.json; [ $rc -ne 0 ] && exit $rc
done
exit 0
