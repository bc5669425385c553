# fp32 LDS-tiled GEMM on 16x16x4 MFMAs (ND_F32_M16): op tests, encoder-shape microbench, exact-leg A/B
cd $GRAFT_REPO_ROOT && O=$GRAFT_REPO_ROOT/gpurun_out && export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "test_gemm_vs_fp64" > $O/r06_gpu19_tests.log 2>&1 || { tail -30 $O/r06_gpu19_tests.log; exit 1; }
tail -1 $O/r06_gpu19_tests.log
bash tools/ab_f32tile.sh m16off m16on m16off m16on > $O/r06_ab_m16_micro.txt 2>&1 || exit $?
cat $O/r06_ab_m16_micro.txt
bash tools/ab_exact.sh m16off m16on > $O/r06_ab_exact_m16.txt 2>&1 || exit $?
cat $O/r06_ab_exact_m16.txt
