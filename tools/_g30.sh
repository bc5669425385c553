#!/bin/bash
# which decoder GEMM class disturbs which encoder form (tools/rank2_probe2.py)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for v in "ND_ENC_ATTN0=1" "ND_ENC_ATTN0=0" "ND_ENC_FFN=0" "ND_ENC_WO=0" "ND_ENC_QKV=0"; do
  env $v timeout -k 10 200 python -u tools/rank2_probe2.py > $O/r2q.log 2>&1; rc=$?
  echo "$v rc=$rc"; grep -v amdgpu.ids $O/r2q.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
