C="SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
bash tools/gpu.sh pmcpy r06h_mfma_sgemm "$C" $GRAFT_REPO_ROOT/tools/probe_sgemm.py && \
python3 tools/mfma_summary.py gpurun_out/r06h_mfma_sgemm/run_counter_collection.csv sgemm gpurun_out/r06h_mfma_sgemm.json > /dev/null && \
bash tools/gpu.sh pmcpy r06h_mfma_f32d "$C" $GRAFT_REPO_ROOT/tools/f32d_check.py $GRAFT_REPO_ROOT/tools/_ab/f32base.so ; \
python3 tools/mfma_summary.py gpurun_out/r06h_mfma_f32d/run_counter_collection.csv f32d gpurun_out/r06h_mfma_f32d.json > /dev/null; rm -rf gpurun_out/r06h_mfma_sgemm gpurun_out/r06h_mfma_f32d
