# same-box A/B of two builds of the library on the greedy bench:
#   bash tools/ab_lib.sh A B [bench args]   (tools/_ab/A.so, tools/_ab/B.so via NANODEC_LIB; interleaved A B A B)
a=$1; b=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for rep in 1 2; do
  for v in $a $b; do
    NANODEC_AB=1 NANODEC_LIB=$R/tools/_ab/$v.so timeout -k 10 300 python -u bench.py --allow-switches --steps 60 --warmup 3 \
      --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 --config-legs 0 "$@" \
      > $O/ab_lib_${v}_$rep.json 2> $O/ab_lib_${v}_$rep.err || exit $?
    python3 -c "
import json; d=json.loads(open('$O/ab_lib_${v}_$rep.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}
rp = d.get('roofline_pooled') or {}
print('$v rep $rep: %.3f ms/step  one call %s  %s %.2f us  pooled %.2f us' % (d['ms_per_step'], (d.get('one_call_in_flight') or {}).get('ms_per_step'), r.get('kernel'), 1e3*r.get('avg_launch_ms', 0), 1e3*rp.get('avg_launch_ms', 0)))"
  done
done
