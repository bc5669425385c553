set -u
cd $GRAFT_REPO_ROOT
for sw in NONE=1 ND_QKV_TABLE=0 ND_HEAD_FUSE=0; do
  env $sw timeout -k 10 120 python -u tools/canary_victim.py 2>&1 | grep spinners || exit 1
done
