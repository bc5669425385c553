# PMC counter passes over the split-fp16 encoder FFN1 GEMM (eager launches)
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmcgemm; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export MB_EAGER=1
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR" \
         "TCC_HIT TCC_MISS TCC_BUSY"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $C -d $O/p$i -o run --output-format csv -- python3 $R/tools/microbench.py ffn1s > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $O/p$i.log; exit $rc; fi
done
