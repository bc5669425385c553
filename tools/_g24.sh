#!/bin/bash
# round-3 refresh: smoke + every GPU test, the default bench line, a kernel-trace profile
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
bash tools/gpu.sh test || exit $?
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/r03_bench_final.json 2> $O/r03_bench_final.err || exit $?
tail -c 600 $O/r03_bench_final.json
bash tools/gpu.sh prof r03_greedy_final --inflight 1 || exit $?
