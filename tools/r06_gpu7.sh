cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/sweep_args.sh "--inflight 3" "--inflight 4" "--inflight 3 --bank-grid 96" "--inflight 3 --bank-grid 160" "--inflight 4 --bank-grid 96" > gpurun_out/r06_sweep_pool.txt 2>&1
