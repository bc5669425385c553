#!/bin/bash
# co-residency disturbance vs hardware queues per process (streams sharing a queue?)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q PROBE_ROUNDS=4 PROBE_SHORT=1 timeout -k 10 200 python -u tools/rank2_probe.py > $O/r2hq_$q.log 2>&1; rc=$?
  echo "queues=$q rc=$rc"; grep -v amdgpu.ids $O/r2hq_$q.log | head -30
  [ $rc -ne 0 ] && exit $rc
done
exit 0
