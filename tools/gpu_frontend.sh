# device front end: parity tests, then the GPU suite
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/fe; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "frontend" > $O/t.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" $O/t.log | tail -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; exit $rc
