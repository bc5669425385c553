#!/bin/bash
# rank-2 kernel LDS rounded to 2 KB (default) vs unrounded with wcnt first (r2_nopad)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for v in default r2_nopad; do
  lib=$R/nanodecoder_amd/libnanodec_hip.so; [ $v != default ] && lib=$R/tools/_ab/$v.so
  NANODEC_LIB=$lib PROBE_ROUNDS=4 PROBE_SHORT=1 PROBE_WHERE=1 timeout -k 10 200 python -u tools/rank2_probe.py > $O/r2pad_$v.log 2>&1; rc=$?
  echo "$v rc=$rc"; grep -v amdgpu.ids $O/r2pad_$v.log | head -30
  [ $rc -ne 0 ] && exit $rc
done
exit 0
