# round 6, third call: the bank kernel's phase stamps, the exact-fp32 one-call kernel trace, the split
# one-call and pooled kernel traces of the current tree
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
NANODEC_AB=1 NANODEC_LIB=$GRAFT_REPO_ROOT/tools/_ab/b8_phases.so timeout -k 10 120 python -u tools/bank_phases.py > gpurun_out/r06_bank_phases.txt 2>&1 || exit $?
ND_GEMM_F32=1 bash tools/gpu.sh prof r06_exact_one_call --inflight 1 --allow-switches || exit $?
bash tools/gpu.sh prof r06a_one_call --inflight 1 || exit $?
bash tools/gpu.sh prof r06a_pool3 || exit $?
