# the DMA-ring fp32 GEMM on 16x16x4 (ND_F32D): bitwise against the register-staged M16 kernel and timed,
# GEMM op tests, then the exact leg A/B
cd $GRAFT_REPO_ROOT && O=$GRAFT_REPO_ROOT/gpurun_out && export PYTHONUNBUFFERED=1
timeout -k 10 240 python -u tools/f32d_check.py tools/_ab/f32dm16_off.so > $O/r06_f32dm16_check.txt 2>&1; rc=$?
cat $O/r06_f32dm16_check.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "test_gemm_vs_fp64" > $O/r06_gpu21_tests.log 2>&1 || { tail -20 $O/r06_gpu21_tests.log; exit 1; }
tail -1 $O/r06_gpu21_tests.log
[ $rc -eq 0 ] || exit 1
bash tools/ab_exact.sh f32dm16_off f32dm16_on
