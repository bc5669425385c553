#!/bin/bash
# next layer's QKV folded into the FFN launch + buffer_load..lds copies: op tests, parity,
# microbench (base / global_load_lds / 3 ahead), bench A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "enc_ffn or golden or encoder or greedy_config or range_guard or beam_config" > $O/t23.log 2>&1; rc=$?; tail -1 $O/t23.log; [ $rc -ne 0 ] && exit $rc
NANODEC_LIB=$R/tools/_ab/ahead3.so timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "enc_ffn" > $O/t23b.log 2>&1; rc=$?; tail -1 $O/t23b.log; [ $rc -ne 0 ] && exit $rc
for v in base glds ahead3 base glds ahead3; do
  L=$R/nanodecoder_amd/libnanodec_hip.so; [ $v != base ] && L=$R/tools/_ab/$v.so
  NANODEC_LIB=$L timeout -k 10 120 python -u tools/microbench.py encffn > $O/mb23_$v.log 2>&1 || exit $?
  echo "$v: $(grep enc-ffn $O/mb23_$v.log | sed 's/ M=131072//' | tr '\n' ' ')"
done
B="--steps 30 --warmup 5 --config-legs 0 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0"
for rep in 1 2; do for v in q0 base ahead3; do
  L=$R/nanodecoder_amd/libnanodec_hip.so; [ $v = ahead3 ] && L=$R/tools/_ab/$v.so
  Q=1; [ $v = q0 ] && Q=0
  ND_ENC_QKV=$Q NANODEC_LIB=$L timeout -k 10 300 python -u bench.py $B --allow-switches > $O/b23_$v.json 2> $O/b23_$v.err || exit $?
  python3 -c "
import json; d=json.loads(open('$O/b23_$v.json').read().strip().splitlines()[-1]); m=d.get('mfma') or {}
print('%s: %.3f ms/call  enc %s' % ('$v', d['ms_per_step'], (m.get('encoder_only') or {}).get('ms')))"
done; done
