#!/bin/bash
# bank kernel on fewer workgroups (ND_BANK_GRID): parity at 128, then A/B pooled
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
ND_BANK_GRID=128 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "bank or greedy_config or golden or pool" > $O/t36.log 2>&1; rc=$?; tail -3 $O/t36.log; [ $rc -ne 0 ] && exit $rc
B="--steps 30 --warmup 5 --config-legs 0 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 --allow-switches"
for rep in 1 2; do for g in 0 192 128; do
  ND_BANK_GRID=$g timeout -k 10 300 python -u bench.py $B > $O/b36_$g.json 2> $O/b36_$g.err || exit $?
  python3 -c "
import json; d=json.loads(open('$O/b36_$g.json').read().strip().splitlines()[-1]); r=d['roofline']
print('grid $g: %.3f ms/call  %.3f M   bank alone %.2f us' % (d['ms_per_step'], d['value']/1e6, 1e3*r['avg_launch_ms']))"
done; done
