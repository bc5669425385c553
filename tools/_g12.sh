set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -v -m gpu tests/test_gpu_configs.py -k beam1 --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t12.log 2>&1; rc=$?; grep -E "PASSED|FAILED|^E " gpurun_out/t12.log | head; [ $rc -ne 0 ] && exit $rc
bash tools/gpu.sh test && bash tools/gpu.sh bench r03_pool_greedy --steps 20 --warmup 5
