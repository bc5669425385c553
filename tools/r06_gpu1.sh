# round 6: the new precision / RCCL tests (no -x: every measurement printed), then the whole GPU suite
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 420 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_rccl.py -v -s --timeout 240 --timeout-method thread -m gpu > gpurun_out/r06_prec1.log 2>&1
rc=$?
echo "precision rc=$rc" >> gpurun_out/r06_prec1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 480 python -u -m pytest tests -x -q --timeout 180 --timeout-method thread -m gpu --deselect tests/test_gpu_precision.py --deselect tests/test_gpu_rccl.py > gpurun_out/r06_gpu1.log 2>&1
