# round 6: the fp32 split-K route (exact fp32, pool lanes): its op and precision tests, the exact leg A/B
# (previous gemm.hip vs this one), then the fp32 bank kernel's timing probes
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu -k "splitk or exact_fp32_config1" > gpurun_out/r06_gpu8_tests.log 2>&1 || exit $?
bash tools/ab_exact.sh sk_prev sk_new > gpurun_out/r06_ab_exact_splitk.txt 2>&1 || exit $?
bash tools/mem_probe.sh > gpurun_out/r06_mem_probe.txt 2>&1
