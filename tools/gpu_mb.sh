# microbench one section: bash tools/gpu_mb.sh <section> [ENV=VAL ...]
set -u
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
sec=$1; shift
env "$@" timeout -k 10 300 python tools/microbench.py $sec > gpurun_out/mb.log 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/mb.log; exit $rc
