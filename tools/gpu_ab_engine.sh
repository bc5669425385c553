# engine A/B of an environment knob: per-kernel times from a kernel trace of the greedy bench
# KNOB=ND_GEMM_XCD VALS="1 0" bash tools/gpu_ab_engine.sh
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/abe; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for x in ${VALS:-1 0}; do
  env $KNOB=$x timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t$x -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --no-roofline > $O/b$x.json 2> $O/b$x.err
  rc=$?; echo "== $KNOB=$x rc=$rc"; cut -c1-200 $O/b$x.json; [ $rc -ne 0 ] && exit $rc
done
exit 0
