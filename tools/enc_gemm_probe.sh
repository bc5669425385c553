# encoder FFN: fused block parity (twice, for an intermittent race) + microbench timing against the two split GEMMs it replaces
cd $GRAFT_REPO_ROOT && O=$GRAFT_REPO_ROOT/gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "enc_ffn or encoder_memory or transformer" > $O/t_ffn.log 2>&1; rc=$?; tail -2 $O/t_ffn.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "enc_ffn" > $O/t_ffn2.log 2>&1; rc=$?; tail -2 $O/t_ffn2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/microbench.py encffn > $O/mb_encffn.log 2>&1; rc=$?; cat $O/mb_encffn.log; exit $rc
