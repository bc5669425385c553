# round 6: calls in flight and the bank grid on the exact-fp32 leg
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/sweep_exact.sh "--inflight 3" "--inflight 2" "--inflight 4" "--inflight 3 --bank-grid 192" "--inflight 3 --bank-grid 96" > gpurun_out/r06_sweep_exact.txt 2>&1
