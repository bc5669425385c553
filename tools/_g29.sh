#!/bin/bash
# rank-2 encoder attention disturbed by which decoder kernel class of the other lane
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for v in default skip_bank skip_self skip_p16; do
  lib=""; [ $v != default ] && lib=$R/tools/_ab/$v.so
  NANODEC_LIB=${lib:-$R/nanodecoder_amd/libnanodec_hip.so} PROBE_ROUNDS=4 PROBE_SHORT=1 \
    timeout -k 10 200 python -u tools/rank2_probe.py > $O/r2v_$v.log 2>&1; rc=$?
  echo "$v rc=$rc"; grep -v amdgpu.ids $O/r2v_$v.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
