#!/bin/bash
# bank kernel at 4 waves per chunk (half the LDS): parity, then one-call and pooled A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
B="--steps 30 --warmup 5 --config-legs 0 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0"
NANODEC_LIB=$R/tools/_ab/bank4.so timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "bank or greedy_config or greedy_vs_oracle or golden" > $O/t17.log 2>&1; rc=$?; tail -2 $O/t17.log; [ $rc -ne 0 ] && exit $rc
for v in base bank4 bank4a2 base bank4 bank4a2; do
  L=$R/nanodecoder_amd/libnanodec_hip.so; [ $v != base ] && L=$R/tools/_ab/$v.so
  for inf in 1 3; do
    NANODEC_LIB=$L timeout -k 10 300 python -u bench.py $B --inflight $inf > $O/b17_${v}_$inf.json 2> $O/b17_${v}_$inf.err || exit $?
    python3 -c "
import json; d=json.loads(open('$O/b17_${v}_$inf.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}
print('%-8s inflight %d: %.3f ms/call  bank %.2f us' % ('$v', $inf, d['ms_per_step'], 1e3*r.get('avg_launch_ms', 0)))"
  done
done
