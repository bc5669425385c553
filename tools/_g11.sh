set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu.sh py teardown tools/pool_teardown_probe.py || exit 1
timeout -k 10 900 python -u -X faulthandler -m pytest -v -m gpu tests/test_asan.py tests/test_gpu_configs.py --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t10.log 2>&1; echo rc=$?
grep -E "PASSED|FAILED|ERROR|Segmentation" gpurun_out/t10.log | head -30
