#!/bin/bash
# self-attention at 8 waves per row for every length (ND_SELF_NW8): parity, then pooled / one call
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
ND_SELF_NW8=1 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "self or golden or greedy_config or pool" > $O/t43.log 2>&1; rc=$?; tail -2 $O/t43.log; [ $rc -ne 0 ] && exit $rc
B="--steps 30 --warmup 5 --config-legs 0 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 --no-roofline --allow-switches"
for rep in 1 2; do for inf in 3 1; do for v in 0 1; do
  ND_SELF_NW8=$v timeout -k 10 300 python -u bench.py $B --inflight $inf > $O/b43.json 2> $O/b43.err || exit $?
  python3 -c "
import json; d=json.loads(open('$O/b43.json').read().strip().splitlines()[-1])
print('inflight $inf nw8=$v: %.3f ms/call  %.3f M' % (d['ms_per_step'], d['value']/1e6))"
done; done; done
