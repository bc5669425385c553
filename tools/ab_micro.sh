# same-box A/B of library builds on one microbench case:
#   bash tools/ab_micro.sh CASE A B ...   (tools/_ab/<name>.so, alternated twice)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; L=nanodecoder_amd/libnanodec_hip.so; cp $L /tmp/keep.so
case_=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    cp tools/_ab/$v.so $L || exit 1
    echo "== $v rep $rep"; timeout -k 10 120 python -u tools/microbench.py $case_ 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
cp /tmp/keep.so $L
