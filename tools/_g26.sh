#!/bin/bash
# layer-0 encoder attention in closed form: parity, then A/B (ND_ENC_ATTN0)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "transformer_encoder_vs_oracle or golden or encoder or greedy_config or beam_config or enc_attention" > $O/t26.log 2>&1; rc=$?; tail -3 $O/t26.log; [ $rc -ne 0 ] && exit $rc
B="--steps 30 --warmup 5 --config-legs 0 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0"
for rep in 1 2; do for v in 0 1; do
  ND_ENC_ATTN0=$v timeout -k 10 300 python -u bench.py $B --allow-switches > $O/b26_$v.json 2> $O/b26_$v.err || exit $?
  python3 -c "
import json; d=json.loads(open('$O/b26_$v.json').read().strip().splitlines()[-1]); m=d.get('mfma') or {}
print('attn0=%s: %.3f ms/call  enc %s' % ('$v', d['ms_per_step'], (m.get('encoder_only') or {}).get('ms')))"
done; done
