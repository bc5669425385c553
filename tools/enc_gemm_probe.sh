# encoder FFN: fused block vs the two split GEMMs (microbench timings), parity of the fused op
cd $GRAFT_REPO_ROOT && O=$GRAFT_REPO_ROOT/gpurun_out && \
true
timeout 300 python3 tools/microbench.py encffn > $O/mb_encffn.log 2>&1; rc=$?; cat $O/mb_encffn.log; exit $rc
