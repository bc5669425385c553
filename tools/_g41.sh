#!/bin/bash
# walking bank kernel: the next chunk's first loads under the merge (new) vs after it (walk_old)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "bank or pool or greedy_config" > $O/t41.log 2>&1; rc=$?; tail -2 $O/t41.log; [ $rc -ne 0 ] && exit $rc
B="--steps 30 --warmup 5 --config-legs 0 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0"
for rep in 1 2; do for v in new walk_old; do
  lib=$R/nanodecoder_amd/libnanodec_hip.so; [ $v != new ] && lib=$R/tools/_ab/$v.so
  NANODEC_LIB=$lib timeout -k 10 300 python -u bench.py $B > $O/b41.json 2> $O/b41.err || exit $?
  python3 -c "
import json; d=json.loads(open('$O/b41.json').read().strip().splitlines()[-1]); p=d['roofline_pooled']
print('%-9s %.3f ms/call  %.3f M  bank pooled %.2f us' % ('$v', d['ms_per_step'], d['value']/1e6, 1e3*p['avg_launch_ms']))"
done; done
