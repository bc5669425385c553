#!/bin/bash
# same-box A/B of several library builds (tools/_ab/NAME.so), interleaved, two reps:
#   bash tools/ab_multi.sh "A B C" [bench args]
vs=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for rep in 1 2; do
  for v in $vs; do
    NANODEC_AB=1 NANODEC_LIB=$R/tools/_ab/$v.so timeout -k 10 300 python -u bench.py --allow-switches --steps 60 --warmup 3 \
      --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 --config-legs 0 "$@" \
      > $O/ab_multi_${v}_$rep.json 2> $O/ab_multi_${v}_$rep.err || exit $?
    python3 -c "
import json; d=json.loads(open('$O/ab_multi_${v}_$rep.json').read().strip().splitlines()[-1])
print('$v rep $rep: %.3f ms/step  one call %s' % (d['ms_per_step'], (d.get('one_call_in_flight') or {}).get('ms_per_step')))"
  done
done
