#!/bin/bash
# bank grid sweep in the pool (ND_BANK_GRID), transformer and NanoEncoder
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
B="--steps 30 --warmup 5 --config-legs 0 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 --allow-switches --no-roofline"
for rep in 1 2; do for enc in transformer nano; do for g in 0 64 96 128 160; do
  ND_BANK_GRID=$g timeout -k 10 300 python -u bench.py $B --encoder $enc > $O/b37.json 2> $O/b37.err || exit $?
  python3 -c "
import json; d=json.loads(open('$O/b37.json').read().strip().splitlines()[-1])
print('$enc grid $g: %.3f ms/call  %.3f M' % (d['ms_per_step'], d['value']/1e6))"
done; done; done
