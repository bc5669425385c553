#!/bin/bash
# PMC breakdown of the fused FFN block (two SQ passes over microbench encffn)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
bash tools/gpu.sh pmcmb ffnpmc1 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU" encffn && \
python3 tools/pmc_kernel.py $O/ffnpmc1/run_counter_collection.csv enc_ffn > $O/ffnpmc1.txt && cat $O/ffnpmc1.txt && \
bash tools/gpu.sh pmcmb ffnpmc2 "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" encffn && \
python3 tools/pmc_kernel.py $O/ffnpmc2/run_counter_collection.csv enc_ffn > $O/ffnpmc2.txt && cat $O/ffnpmc2.txt
