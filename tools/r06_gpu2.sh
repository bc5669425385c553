# round 6, second call: precision / RCCL tests, the whole GPU suite, the bank kernel's probe variants,
# configs[3]'s beam PMC pass on the bench workload, one bench line
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 480 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_rccl.py -v -s --timeout 240 --timeout-method thread -m gpu > gpurun_out/r06_prec2.log 2>&1
rc=$?
echo "precision rc=$rc" >> gpurun_out/r06_prec2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 180 --timeout-method thread -m gpu --deselect tests/test_gpu_precision.py --deselect tests/test_gpu_rccl.py > gpurun_out/r06_gpu2.log 2>&1 || exit $?
bash tools/bank_probe.sh > gpurun_out/r06_bank_probe.txt 2>&1 || exit $?
bash tools/pmc_beam.sh r06 > gpurun_out/r06_pmc_beam.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r06_bench_a.json 2> gpurun_out/r06_bench_a.err
