set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -X faulthandler -m pytest -v -m gpu tests/test_asan.py tests/test_bench_launcher.py tests/test_checkpoint_frontend.py tests/test_cli.py tests/test_gpu_configs.py --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t10.log 2>&1; echo rc=$?
grep -E "PASSED|FAILED|ERROR|Segmentation|File \"/tmp" gpurun_out/t10.log | head -30
