set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_asan.py -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_configs.log 2>&1; rc=$?; tail -15 gpurun_out/t_configs.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu.sh bench r03_pool_greedy --steps 20 --warmup 5
