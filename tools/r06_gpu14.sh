# round 6: the digit bank at every chunk length (T <= 512): the whole GPU suite (the golden fixtures' short
# chunks now take it), then the headline A/B of bank8.hip (the T = 512 path must be unchanged)
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -x -q --timeout 400 --timeout-method thread -m gpu -p no:cacheprovider > gpurun_out/r06_gpu14_tests.log 2>&1 || exit $?
bash tools/ab_lib.sh b8_prev b8_kpw > gpurun_out/r06_ab_b8_kpw.txt 2>&1
