#!/bin/bash
# bank U row-major only (W_vo GEMM reads A row-major): parity, then A/B against base
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "golden or greedy or pool or attn or self or sampl or beam" > $O/t47b.log 2>&1; rc=$?; tail -2 $O/t47b.log; [ $rc -ne 0 ] && exit $rc
B="--steps 30 --warmup 5 --config-legs 0 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0"
for rep in 1 2; do for v in new base; do
  lib=$R/nanodecoder_amd/libnanodec_hip.so; [ $v != new ] && lib=$R/tools/_ab/$v.so
  NANODEC_LIB=$lib timeout -k 10 300 python -u bench.py $B > $O/b47.json 2> $O/b47.err || exit $?
  python3 -c "
import json; d=json.loads(open('$O/b47.json').read().strip().splitlines()[-1]); r=d['roofline']; p=d['roofline_pooled']
print('%-5s %.3f ms/call  %.3f M  bank alone %.2f us  pooled %.2f us  one call %.3f' % ('$v', d['ms_per_step'], d['value']/1e6, 1e3*r['avg_launch_ms'], 1e3*p['avg_launch_ms'], d['one_call_in_flight']['ms_per_step']))"
done; done
