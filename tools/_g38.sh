#!/bin/bash
# encoder kernels on fewer CUs in the pool (ND_ENC_FFN_GRID / ND_ENC_ATTN_GRID): parity, then A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
ND_ENC_FFN_GRID=7 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "enc_ffn or encoder or golden" > $O/t38.log 2>&1; rc=$?; tail -2 $O/t38.log; [ $rc -ne 0 ] && exit $rc
B="--steps 30 --warmup 5 --config-legs 0 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 --allow-switches --no-roofline"
for rep in 1 2; do for v in "X=0" "ND_ENC_FFN_GRID=224" "ND_ENC_FFN_GRID=192" "ND_ENC_ATTN_GRID=192" "ND_ENC_FFN_GRID=192 ND_ENC_ATTN_GRID=192"; do
  env $v timeout -k 10 300 python -u bench.py $B > $O/b38.json 2> $O/b38.err || exit $?
  python3 -c "
import json; d=json.loads(open('$O/b38.json').read().strip().splitlines()[-1])
print('%-42s %.3f ms/call  %.3f M' % ('$v', d['ms_per_step'], d['value']/1e6))"
done; done
