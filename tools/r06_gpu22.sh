# DMA-ring fp32 GEMM: ring slots / epilogue passes variants, bitwise check of s3e4 against the register-staged
# kernel, then the exact leg on each (marginal_exact.sh prints exact and headline ms per call)
cd $GRAFT_REPO_ROOT && O=$GRAFT_REPO_ROOT/gpurun_out && export PYTHONUNBUFFERED=1
NANODEC_AB=1 NANODEC_LIB=$GRAFT_REPO_ROOT/tools/_ab/s3e4.so timeout -k 10 240 python -u tools/f32d_check.py tools/_ab/regm16.so > $O/r06_f32d_s3e4_check.txt 2>&1 || { cat $O/r06_f32d_s3e4_check.txt; exit 1; }
cat $O/r06_f32d_s3e4_check.txt
bash tools/marginal_exact.sh regm16 s4e2 s3e4 s4e4
