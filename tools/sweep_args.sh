#!/bin/bash
# same-box sweep of bench.py argument sets on the greedy headline, each run twice, interleaved:
#   bash tools/sweep_args.sh "ARGS1" "ARGS2" ...   (one short bench line per run; prints ms per pooled call)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for rep in 1 2; do
  i=0
  for a in "$@"; do
    i=$((i + 1))
    timeout -k 10 300 python -u bench.py --steps 60 --warmup 3 --cpu-baseline 0 --exact 0 --host-inclusive 0 \
      --read-shard 0 --config-legs 0 $a > $O/sweep_${i}_$rep.json 2> $O/sweep_${i}_$rep.err || exit $?
    python3 -c "
import json; d=json.loads(open('$O/sweep_${i}_$rep.json').read().strip().splitlines()[-1])
print('[$a] rep $rep: %.3f ms/call pooled  one call %s' % (d['ms_per_step'], (d.get('one_call_in_flight') or {}).get('ms_per_step')))"
  done
done
