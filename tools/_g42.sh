#!/bin/bash
# calls in flight with the bank grid: 3 vs 4 lanes (transformer, NanoEncoder)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
B="--steps 30 --warmup 5 --config-legs 0 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 --no-roofline"
for rep in 1 2; do for enc in transformer nano; do for n in 3 4; do
  timeout -k 10 300 python -u bench.py $B --encoder $enc --inflight $n > $O/b42.json 2> $O/b42.err || exit $?
  python3 -c "
import json; d=json.loads(open('$O/b42.json').read().strip().splitlines()[-1])
print('$enc lanes $n: %.3f ms/call  %.3f M' % (d['ms_per_step'], d['value']/1e6))"
done; done; done
