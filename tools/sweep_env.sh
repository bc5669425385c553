#!/bin/bash
# Headline-only bench lines under engine switches (one GPU call; each run time-limited; stops at the first
# failure).   bash tools/sweep_env.sh TAG "ND_X=1 ND_Y=0" "..." ...   -> gpurun_out/TAG_<i>.json
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
tag=$1; shift
B="--config-legs 0 --steps 40 --warmup 5 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 --no-roofline --allow-switches"
i=0
for e in "$@"; do
  env $e timeout -k 10 300 python -u bench.py $B > $O/${tag}_$i.json 2> $O/${tag}_$i.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/${tag}_$i.json').read().strip().splitlines()[-1]); print('$e', '->', d['value'], d['ms_per_step'], 'one call', d.get('one_call_in_flight',{}).get('ms_per_step'), d.get('pool_check',{}).get('result'))"
  i=$((i+1))
done
