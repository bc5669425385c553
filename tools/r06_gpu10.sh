# round 6: the fp32 bank kernel's walking-form prefetch (exact fp32 pool lanes): op / precision / pooled
# bitwise tests, the kernel alone with and without the prefetch, the exact leg A/B, then calls in flight and
# the bank grid on the exact leg
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 400 --timeout-method thread -m gpu -k "mem_attention or splitk or pool_at_bench or exact_fp32_config1" > gpurun_out/r06_gpu10_tests.log 2>&1 || exit $?
bash tools/mem_probe.sh mb_nopf mb_pf > gpurun_out/r06_mem_prefetch.txt 2>&1 || exit $?
bash tools/ab_exact.sh mb_nopf mb_pf > gpurun_out/r06_ab_exact_prefetch.txt 2>&1 || exit $?
bash tools/sweep_exact.sh "--inflight 3" "--inflight 2" "--inflight 4" "--inflight 3 --bank-grid 192" "--inflight 3 --bank-grid 96" > gpurun_out/r06_sweep_exact.txt 2>&1
