# round 6, fourth call: the bank kernel's walking form with the next chunk's head prefetched (b8_new) against
# the previous commit's (b8_old), then the bank / pool GPU tests on the new library
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/ab_lib.sh b8_old b8_new > gpurun_out/r06_ab_walk.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 180 --timeout-method thread -m gpu -k "bank_d8 or pool" > gpurun_out/r06_gpu4.log 2>&1 || exit $?
ND_GEMM_F32=1 bash tools/gpu.sh prof r06_exact_pool3 --allow-switches
