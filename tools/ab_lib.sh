# same-box A/B of two builds of the library on the greedy bench:
#   bash tools/ab_lib.sh [bench args]     (tools/_ab/A.so, tools/_ab/B.so; interleaved A B A B)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
L=nanodecoder_amd/libnanodec_hip.so
for rep in 1 2; do
  for v in A B; do
    cp tools/_ab/$v.so $L || exit 1
    timeout -k 10 300 python -u bench.py --steps 60 --warmup 3 --cpu-baseline 0 --exact 0 --host-inclusive 0 \
      --read-shard 0 "$@" > $O/ab_lib_${v}_$rep.json 2> $O/ab_lib_${v}_$rep.err || exit $?
    python3 -c "
import json; d=json.loads(open('$O/ab_lib_${v}_$rep.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}
print('$v rep $rep: %.3f ms/step  %s %.2f us' % (d['ms_per_step'], r.get('kernel'), 1e3*r.get('avg_launch_ms', 0)))"
  done
done
cp tools/_ab/B.so $L
