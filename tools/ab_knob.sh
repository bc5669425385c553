# same-box A/B of an environment knob on the greedy bench: bash tools/ab_knob.sh VAR "v0 v1 ..." [bench args]
# each value runs twice, interleaved (v0 v1 v0 v1), one short bench line each
var=$1; vals=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for rep in 1 2; do
  for v in $vals; do
    env $var=$v timeout -k 10 300 python -u bench.py --allow-switches --steps 60 --warmup 3 --cpu-baseline 0 --exact 0 --host-inclusive 0 \
      --read-shard 0 "$@" > $O/ab_${var}_${v}_$rep.json 2> $O/ab_${var}_${v}_$rep.err || exit $?
    python3 -c "
import json,sys; d=json.loads(open('$O/ab_${var}_${v}_$rep.json').read().strip().splitlines()[-1])
r=d.get('roofline') or {}
print('$var=$v rep $rep: %.3f ms/step  one call %s  value %.0f  dominant %s %.2f us' % (d['ms_per_step'], (d.get('one_call_in_flight') or {}).get('ms_per_step'), d['value'], r.get('kernel'), 1e3*r.get('avg_launch_ms', 0)))"
  done
done
