# round 6: the beam self-attention's second slot table only on steps past 256 (LONG): beam / long max_length /
# context tests, then configs[3] A/B against attention.hip before this round's max_length and beam-size changes
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 400 --timeout-method thread -m gpu -k "beam or long_max_length or self_attention" > gpurun_out/r06_gpu18_tests.log 2>&1 || exit $?
bash tools/ab_lib.sh att_r06a att_new --mode beam --batch 1024 --steps 30 > gpurun_out/r06_ab_att_long.txt 2>&1
