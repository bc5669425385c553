# round 6: how busy the GPU is in the pooled headline and the pooled beam leg (kernel-trace unions)
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/gpu.sh busy r06_busy_greedy --steps 30 && bash tools/gpu.sh busy r06_busy_beam --mode beam --batch 1024 --steps 9
