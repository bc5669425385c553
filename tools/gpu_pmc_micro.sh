# PMC counter passes over the decoder-step kernel microbench (eager launches)
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmcmicro; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export MB_EAGER=1
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS" \
         "TA_TA_BUSY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ_LATENCY" \
         "TCC_HIT TCC_MISS TCC_BUSY" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C -d $O/p$i -o run --output-format csv -- python3 $R/tools/microbench.py dec256 > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $O/p$i.log; exit $rc; fi
done
