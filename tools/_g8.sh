set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/p16s_probe.py 2>&1 | grep -v amdgpu.ids | grep "h3=1 ln=1" || exit 1
timeout -k 10 200 python -u tools/conc_probe.py quick 2>&1 | grep other || exit 1
timeout -k 10 200 python -u tools/canary_victim.py 2>&1 | grep spinners || exit 1
