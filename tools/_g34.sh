#!/bin/bash
# three lanes: which lanes stream their bank non-temporally (the rest keep it in the Infinity Cache)
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd $R
for rep in 1 2; do
for nt in 0,1,2 1,2 2; do
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --bank-nt-lanes "$nt" --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 --config-legs 0 > $O/nt3_$nt.json 2> $O/nt3_$nt.err || exit 1
  python3 -c "
import json; d=json.loads(open('$O/nt3_$nt.json').read().strip().splitlines()[-1]); r=d['roofline']
print('nt lanes %-6s: %.3f ms/call  %.3f M samples/s' % ('$nt', d['ms_per_step'], d['value']/1e6))"
done
done
