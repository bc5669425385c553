#!/bin/bash
# beam context attention at 8 waves per chunk (CTX_NW=8, half the CU) vs 16: parity, then the beam leg pooled / one call
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
NANODEC_LIB=$R/tools/_ab/ctx8.so timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "beam or ctx" > $O/t44.log 2>&1; rc=$?; tail -2 $O/t44.log; [ $rc -ne 0 ] && exit $rc
B="--mode beam --batch 1024 --steps 6 --warmup 3 --config-legs 0 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 --no-roofline"
for rep in 1 2; do for inf in 3 1; do for v in base ctx8; do
  lib=$R/nanodecoder_amd/libnanodec_hip.so; [ $v != base ] && lib=$R/tools/_ab/$v.so
  NANODEC_LIB=$lib timeout -k 10 300 python -u bench.py $B --inflight $inf > $O/b44.json 2> $O/b44.err || exit $?
  python3 -c "
import json; d=json.loads(open('$O/b44.json').read().strip().splitlines()[-1])
print('inflight $inf %-5s: %.3f ms/call  %.3f M' % ('$v', d['ms_per_step'], d['value']/1e6))"
done; done; done
