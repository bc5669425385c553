#!/bin/bash
# rank-2 encoder attention under co-residency: which side is disturbed
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for v in 1 0; do
  ND_ENC_ATTN0=$v timeout -k 10 240 python -u tools/rank2_probe.py > $O/r2p_$v.log 2>&1; rc=$?
  echo "attn0=$v rc=$rc"; grep -v amdgpu.ids $O/r2p_$v.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
