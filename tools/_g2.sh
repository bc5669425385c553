set -u
O=gpurun_out
timeout -k 10 60 ./tools/probe_concurrency 200 > $O/pc_single.log 2>&1 && cat $O/pc_single.log && \
( timeout -k 10 60 ./tools/probe_concurrency 200 > $O/pc_procA.log 2>&1 & timeout -k 10 60 ./tools/probe_concurrency 200 > $O/pc_procB.log 2>&1; wait ) && cat $O/pc_procA.log $O/pc_procB.log
