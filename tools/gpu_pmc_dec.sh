set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmcdec; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD --kernel-trace -d $O/a -o run --output-format csv -- python3 $R/tools/microbench.py dec256 > $O/a.log 2>&1
echo "a rc=$?"
timeout -k 10 300 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace -d $O/b -o run --output-format csv -- python3 $R/tools/microbench.py dec256 > $O/b.log 2>&1
echo "b rc=$?"
timeout -k 10 300 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TA_BUSY_avr --kernel-trace -d $O/c -o run --output-format csv -- python3 $R/tools/microbench.py dec256 > $O/c.log 2>&1
echo "c rc=$?"
cd $R && timeout -k 10 120 python3 tools/microbench.py dec256 > $O/plain.log 2>&1; echo "plain rc=$?"
