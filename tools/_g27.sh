#!/bin/bash
# pool-vs-single determinism A/B: layer-0 closed-form attention off / on
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for v in 1 0; do
  ND_ENC_ATTN0=$v timeout -k 10 200 python -u tools/determinism_probe.py 64 > $O/det27_$v.log 2>&1; rc=$?
  echo "probe attn0=$v rc=$rc"; cat $O/det27_$v.log | tail -12
  [ $rc -ne 0 ] && exit $rc
done
for v in 1 0; do
  ND_ENC_ATTN0=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -q -m gpu --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "pool_matches" > $O/t27_$v.log 2>&1; rc=$?
  echo "attn0=$v rc=$rc"; tail -3 $O/t27_$v.log
  [ $rc -gt 1 ] && exit $rc
done
exit 0
