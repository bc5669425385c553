#!/bin/bash
# layer-0 table keys: full GPU suite, then bench with and without (A/B)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
B="--steps 20 --warmup 5 --config-legs 0 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0"
bash tools/gpu.sh test && \
timeout -k 10 300 python -u bench.py $B > $O/b16_on.json 2> $O/b16_on.err && \
ND_SELF_TABK=0 timeout -k 10 300 python -u bench.py $B --allow-switches > $O/b16_off.json 2> $O/b16_off.err && \
timeout -k 10 300 python -u bench.py $B --inflight 1 > $O/b16_on1.json 2> $O/b16_on1.err && \
ND_SELF_TABK=0 timeout -k 10 300 python -u bench.py $B --inflight 1 --allow-switches > $O/b16_off1.json 2> $O/b16_off1.err
rc=$?; for f in b16_on b16_off b16_on1 b16_off1; do python3 -c "import json,sys; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'])" 2>/dev/null; done; exit $rc
