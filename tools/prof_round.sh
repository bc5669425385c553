#!/bin/bash
# The round's profile set in one GPU call (each step time-limited, stops at the first failure):
# kernel-trace stats one call at a time and three in flight, FETCH_SIZE / WRITE_SIZE passes and the MFMA
# counter passes (greedy, NanoEncoder, beam) one call at a time.  Summaries: tools/pmc_summary.py,
# tools/mfma_summary.py (run by gpu.sh mfma).   bash tools/prof_round.sh TAG   (e.g. r04)
t=${1:-r04}
bash tools/gpu.sh prof ${t}_one_call --inflight 1 && \
bash tools/gpu.sh prof ${t}_pool3 && \
bash tools/gpu.sh pmc ${t}_pmcF "FETCH_SIZE" --inflight 1 && \
bash tools/gpu.sh pmc ${t}_pmcW "WRITE_SIZE" --inflight 1 && \
python3 tools/pmc_summary.py gpurun_out/${t}_pmcF/run_counter_collection.csv gpurun_out/${t}_pmcW/run_counter_collection.csv \
  gpurun_out/${t}_pmc_summary.json && rm -rf gpurun_out/${t}_pmcF gpurun_out/${t}_pmcW && \
bash tools/gpu.sh mfma ${t}_mfma_greedy --inflight 1 && \
bash tools/gpu.sh mfma ${t}_mfma_nano --inflight 1 --encoder nano && \
bash tools/gpu.sh mfma ${t}_mfma_beam --inflight 1 --mode beam --batch 1024
