#!/bin/bash
# configs[3]'s context-attention traffic per alive chunk (tools/pmc_beam.py): the alive profile unprofiled,
# then FETCH_SIZE and WRITE_SIZE passes over 1 + 2 plain calls of exactly the bench leg's workload.
#   bash tools/pmc_beam.sh TAG        -> gpurun_out/TAG_pmc_beam.json
t=${1:-r06}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && timeout -k 10 200 python -u tools/pmc_beam.py alive gpurun_out/${t}_beam_alive.json > gpurun_out/${t}_beam_alive.log 2>&1 && \
bash tools/gpu.sh pmcpy ${t}_pmcbF "FETCH_SIZE" $R/tools/pmc_beam.py run 2 && \
bash tools/gpu.sh pmcpy ${t}_pmcbW "WRITE_SIZE" $R/tools/pmc_beam.py run 2 && \
cd $R && python3 tools/pmc_beam.py summary gpurun_out/${t}_beam_alive.json 2 gpurun_out/${t}_pmcbF/run_counter_collection.csv \
  gpurun_out/${t}_pmcbW/run_counter_collection.csv gpurun_out/${t}_pmc_beam.json && \
rm -rf gpurun_out/${t}_pmcbF gpurun_out/${t}_pmcbW
