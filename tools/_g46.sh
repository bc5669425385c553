#!/bin/bash
# barrier-free rank-2 layer-0 attention (ND_ENC_ATTN0=1): parity, pool determinism, co-residency probe, A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
ND_ENC_ATTN0=1 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "encoder or golden or pool or greedy_config" > $O/t46.log 2>&1; rc=$?; tail -2 $O/t46.log; [ $rc -gt 1 ] && exit $rc
ND_ENC_ATTN0=1 PROBE_ROUNDS=6 PROBE_SHORT=1 PROBE_WHERE=1 timeout -k 10 200 python -u tools/rank2_probe.py > $O/r2v2.log 2>&1 || exit $?
grep -v amdgpu.ids $O/r2v2.log | tail -8
B="--steps 30 --warmup 5 --config-legs 0 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 --allow-switches"
for rep in 1 2; do for v in 0 1; do
  ND_ENC_ATTN0=$v timeout -k 10 300 python -u bench.py $B > $O/b46.json 2> $O/b46.err || exit $?
  python3 -c "
import json; d=json.loads(open('$O/b46.json').read().strip().splitlines()[-1]); m=d.get('mfma') or {}
print('attn0=$v: %.3f ms/call  %.3f M  enc %s  one call %s' % (d['ms_per_step'], d['value']/1e6, (m.get('encoder_only') or {}).get('ms'), d['one_call_in_flight']['ms_per_step']))"
done; done
