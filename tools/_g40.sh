#!/bin/bash
# N = 2048 decoder GEMMs on the 2x2 LDS tiles (64 KB) instead of 2x4 (96 KB): pooled and one call
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
ND_P16S_2X4=0 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "golden or gemm_p16" > $O/t40.log 2>&1; rc=$?; tail -2 $O/t40.log; [ $rc -ne 0 ] && exit $rc
B="--steps 30 --warmup 5 --config-legs 0 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 --no-roofline --allow-switches"
for rep in 1 2; do for inf in 3 1; do for v in 1 0; do
  ND_P16S_2X4=$v timeout -k 10 300 python -u bench.py $B --inflight $inf > $O/b40.json 2> $O/b40.err || exit $?
  python3 -c "
import json; d=json.loads(open('$O/b40.json').read().strip().splitlines()[-1])
print('inflight $inf 2x4=$v: %.3f ms/call  %.3f M' % (d['ms_per_step'], d['value']/1e6))"
done; done; done
