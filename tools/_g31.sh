#!/bin/bash
# where the co-residency disturbance lands in the memory bank
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for v in "ND_ENC_ATTN0=1" "ND_ENC_FFN=0" "ND_ENC_ATTN_F32=1"; do
  env $v PROBE_ROUNDS=3 PROBE_SHORT=1 PROBE_WHERE=1 timeout -k 10 200 python -u tools/rank2_probe.py > $O/r2w.log 2>&1; rc=$?
  echo "$v rc=$rc"; grep -v amdgpu.ids $O/r2w.log | head -40
  [ $rc -ne 0 ] && exit $rc
done
exit 0
