#!/bin/bash
# closed-form layer-0 attention with its arguments from device memory (ND_ENC_ATTN0=2) vs kernarg (=1):
# parity alone, then the co-residency probe
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
ND_ENC_ATTN0=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "encoder or golden" > $O/t50.log 2>&1; rc=$?; tail -2 $O/t50.log; [ $rc -ne 0 ] && exit $rc
for v in 2 1; do
  ND_ENC_ATTN0=$v PROBE_ROUNDS=6 PROBE_SHORT=1 timeout -k 10 200 python -u tools/rank2_probe.py > $O/r2da_$v.log 2>&1 || exit $?
  echo "attn0=$v"; grep -v amdgpu.ids $O/r2da_$v.log | tail -6
done
