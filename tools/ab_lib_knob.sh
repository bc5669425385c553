# same-box A/B over (library, knob value) pairs on the greedy bench:
#   bash tools/ab_lib_knob.sh VAR "lib:val lib:val ..." [bench args]   (tools/_ab/<lib>.so)
var=$1; pairs=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for rep in 1 2; do
  for p in $pairs; do
    lib=${p%%:*}; val=${p#*:}
    env $var=$val NANODEC_AB=1 NANODEC_LIB=$R/tools/_ab/$lib.so timeout -k 10 300 python -u bench.py --allow-switches --steps 40 --warmup 3 \
      --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 --config-legs 0 "$@" > $O/abk_${lib}_${val}_$rep.json \
      2> $O/abk_${lib}_${val}_$rep.err || exit $?
    python3 -c "
import json; d=json.loads(open('$O/abk_${lib}_${val}_$rep.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}
print('$lib $var=$val rep $rep: %.3f ms/step  one call %s  %s %.2f us' % (d['ms_per_step'], (d.get('one_call_in_flight') or {}).get('ms_per_step'), r.get('kernel'), 1e3*r.get('avg_launch_ms', 0)))"
  done
done
