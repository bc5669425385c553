#!/bin/bash
# FFN stagger A/B: op tests on the default (staggered) build, microbench both, bench both
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "enc_ffn or encoder_memory" > $O/t19.log 2>&1; rc=$?; tail -1 $O/t19.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in stag0 base; do
    L=$R/nanodecoder_amd/libnanodec_hip.so; [ $v != base ] && L=$R/tools/_ab/$v.so
    NANODEC_LIB=$L timeout -k 10 120 python -u tools/microbench.py encffn > $O/mb19_$v.log 2>&1 || exit $?
    echo "$v: $(grep enc-ffn $O/mb19_$v.log | tr '\n' ' ')"
  done
done
B="--steps 30 --warmup 5 --config-legs 0 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0"
for v in stag0 base stag0 base; do
  L=$R/nanodecoder_amd/libnanodec_hip.so; [ $v != base ] && L=$R/tools/_ab/$v.so
  NANODEC_LIB=$L timeout -k 10 300 python -u bench.py $B > $O/b19_$v.json 2> $O/b19_$v.err || exit $?
  python3 -c "
import json; d=json.loads(open('$O/b19_$v.json').read().strip().splitlines()[-1]); m=d.get('mfma') or {}
print('%s: %.3f ms/call  enc %s' % ('$v', d['ms_per_step'], (m.get('encoder_only') or {}).get('ms')))"
done
