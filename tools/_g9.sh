set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu.sh test && bash tools/gpu.sh bench r03_pool_greedy --steps 20 --warmup 5
