# round 6: max_length up to 512 (steps past 256): op and end-to-end tests, the beam configs tests, and the
# configs[3] A/B of the self-attention change (two slot tables) against the previous attention.hip
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 400 --timeout-method thread -m gpu -k "self_attention or long_max_length or beam_config3 or config3" > gpurun_out/r06_gpu12_tests.log 2>&1 || exit $?
bash tools/ab_lib.sh att_prev att_new --mode beam --batch 1024 --steps 30 > gpurun_out/r06_ab_att_beam.txt 2>&1
