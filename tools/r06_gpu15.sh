# round 6: short chunks end to end (greedy transformer / NanoEncoder, --fast beam at T = 300) and the fp32 bank
# kernel's 5-7 tile forms
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu -k "short_chunks or mem_attention" > gpurun_out/r06_gpu15_tests.log 2>&1
