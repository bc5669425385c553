R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out; export PYTHONPATH=$R
for v in "$@"; do
  NANODEC_AB=1 NANODEC_LIB=$R/tools/_ab/$v.so timeout -k 10 120 python -u tools/ctx_time.py $v 2>&1 | grep -v amdgpu.ids || exit 1
done
