# same-box A/B of library builds on one microbench case:
#   bash tools/ab_micro.sh CASE A B ...   (tools/_ab/<name>.so via NANODEC_LIB, alternated twice)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
case_=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    echo "== $v rep $rep"
    NANODEC_AB=1 NANODEC_LIB=$R/tools/_ab/$v.so timeout -k 10 120 python -u tools/microbench.py $case_ 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
