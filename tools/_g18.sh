#!/bin/bash
# Wo folded into the FFN block: op tests, encoder/golden parity, then A/B (ND_ENC_WO)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
B="--steps 30 --warmup 5 --config-legs 0 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0"
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "enc_ffn or golden or encoder or greedy_config or range_guard" > $O/t18.log 2>&1; rc=$?; tail -2 $O/t18.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do for wo in 1 0; do
  for inf in 1 3; do
    ND_ENC_WO=$wo timeout -k 10 300 python -u bench.py $B --inflight $inf --allow-switches > $O/b18_${wo}_$inf.json 2> $O/b18_${wo}_$inf.err || exit $?
    python3 -c "
import json; d=json.loads(open('$O/b18_${wo}_$inf.json').read().strip().splitlines()[-1]); m=d.get('mfma') or {}
print('wo=%s inflight %d: %.3f ms/call  enc %s' % ('$wo', $inf, d['ms_per_step'], (m.get('encoder_only') or {}).get('ms')))"
  done
done; done
