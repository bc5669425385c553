# round 6: the greedy rows' fused output projection (ND_SELF_WO) A/B on the headline bench, then the greedy
# parity tests on the fused default
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/ab_knob.sh ND_SELF_WO "0 1" --config-legs 0 > gpurun_out/r06_ab_self_wo.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 180 --timeout-method thread -m gpu -k "greedy or golden or pool or translator or config or self_attention or exact or outlier or smoke or rccl" > gpurun_out/r06_gpu6.log 2>&1
