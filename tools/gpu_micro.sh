set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python tools/microbench.py > gpurun_out/micro.log 2>&1
echo "micro rc=$?"
