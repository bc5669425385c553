# round 6: beam_size up to 8: op tests (self-attention, context attention, the tail's list-split form), beam 7 / 8
# end to end against the oracle, the beam options and configs[3] tests; then configs[3] A/B of attention.hip
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 400 --timeout-method thread -m gpu -k "beam or ctx_attention or self_attention" > gpurun_out/r06_gpu17_tests.log 2>&1 || exit $?
bash tools/ab_lib.sh att_prev att_b8 --mode beam --batch 1024 --steps 30 > gpurun_out/r06_ab_att_b8.txt 2>&1
