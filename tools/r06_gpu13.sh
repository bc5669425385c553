# round 6: the digit bank at chunk lengths below 449 (key blocks per wave = ceil(T / 128)): op tests, then the
# two bank kernels timed at T = 128 .. 512
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu -k "bank_d8 or mem_attention" > gpurun_out/r06_gpu13_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bank_T_probe.py > gpurun_out/r06_bank_T_probe.txt 2>&1
