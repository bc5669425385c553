#!/bin/bash
# 4-wave bank kernel (half the LDS: fits beside a 64 KB GEMM) x bank grid, pooled; parity of the variant first
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
NANODEC_LIB=$R/tools/_ab/bh4.so timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "bank or greedy_config or pool" > $O/t39.log 2>&1; rc=$?; tail -2 $O/t39.log; [ $rc -ne 0 ] && exit $rc
B="--steps 30 --warmup 5 --config-legs 0 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 --no-roofline"
for rep in 1 2; do for v in "default 128" "default 0" "bh4 128" "bh4 0" "bh4 192"; do
  set -- $v; lib=$R/nanodecoder_amd/libnanodec_hip.so; [ $1 != default ] && lib=$R/tools/_ab/$1.so
  NANODEC_LIB=$lib timeout -k 10 300 python -u bench.py $B --bank-grid $2 > $O/b39.json 2> $O/b39.err || exit $?
  python3 -c "
import json; d=json.loads(open('$O/b39.json').read().strip().splitlines()[-1])
print('%-14s %.3f ms/call  %.3f M' % ('$v', d['ms_per_step'], d['value']/1e6))"
done; done
