# round 6: the exact leg with the fp32 short-chain GEMM routes (ND_F32_SHORTCHAIN 0 / 1 / 2)
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/ab_exact.sh sc0 sc1 > gpurun_out/r06_ab_exact_sc1.txt 2>&1 || exit $?
bash tools/ab_exact.sh sc0 sc2 > gpurun_out/r06_ab_exact_sc2.txt 2>&1
