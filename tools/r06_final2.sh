#!/bin/bash
# round 6's record on the final tree in two GPU calls (each step time-limited, stops at the first failure):
#   bash tools/r06_final2.sh TAG a   smoke, every GPU test, the bench line
#   bash tools/r06_final2.sh TAG b   kernel traces (one call, three in flight, exact fp32 one call), PMC byte
#                                    passes, MFMA counter passes with the dispatch clock (greedy, nano, beam,
#                                    exact fp32), configs[3]'s beam PMC pass on the bench workload
t=${1:-r06i}; part=${2:-a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export PYTHONUNBUFFERED=1
if [ "$part" = a ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${t}_smoke.log 2>&1 || exit $?
  timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 240 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${t}_gpu_tests.log 2>&1 || exit $?
  timeout -k 10 600 python -u bench.py > gpurun_out/${t}_bench.json 2> gpurun_out/${t}_bench.err || exit $?
else
  bash tools/prof_round.sh $t || exit $?
  ND_GEMM_F32=1 bash tools/gpu.sh prof ${t}_exact_one_call --inflight 1 --allow-switches || exit $?
  ND_GEMM_F32=1 bash tools/gpu.sh mfma ${t}_mfma_exact --inflight 1 --allow-switches || exit $?
  bash tools/pmc_beam.sh $t
fi
