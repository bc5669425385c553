set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 120 ./tools/graph_latency > gpurun_out/glat.log 2>&1; echo "rc=$?"
