# round 6: beam self-attention variants (SB_DEDUP / SB_LAZY) timed alone at configs[3]'s shape; the fp32 bank's
# walking form (exact fp32, pool lanes) A/B on the all-exact bench
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for v in sb_base sb_dd sb_lazy sb_both; do
    NANODEC_AB=1 NANODEC_LIB=$GRAFT_REPO_ROOT/tools/_ab/$v.so timeout -k 10 120 python -u tools/self_q24_time.py $v > gpurun_out/r06_self_one.txt 2>&1 || exit 1
    grep -v amdgpu.ids gpurun_out/r06_self_one.txt >> gpurun_out/r06_self_ab.txt
  done
done
ND_GEMM_F32=1 bash tools/ab_lib.sh mb_nowalk mb_walk > gpurun_out/r06_ab_exact_walk.txt 2>&1
