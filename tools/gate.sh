#!/bin/bash
# One GPU call for a new tree: operand-map probes, the digit-bank op tests, then
# smoke + every -m gpu test and one bench line.  If the digit-bank op tests fail,
# the suite and the bench run on the split-fp16 bank (ND_BANK_D8=0) instead.
#   bash tools/gate.sh TAG [bench args]
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
tag=${1:-gate}; shift
timeout -k 10 120 python -u tools/probe_i8.py > $O/probe_i8.log 2>&1
echo "probe_i8 rc=$?"; grep -v amdgpu.ids $O/probe_i8.log | tail -40
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "bank_d8 or bank_form" > $O/${tag}_d8.log 2>&1
rc=$?; echo "d8 op tests rc=$rc"; tail -15 $O/${tag}_d8.log
case $rc in 0|1) ;; *) exit $rc ;; esac   # a fault, abort or time limit: stop here
extra=""
if [ $rc -ne 0 ]; then export ND_BANK_D8=0; extra="--allow-switches"; echo "== falling back to ND_BANK_D8=0"; fi
bash tools/gpu.sh test; rc=$?; cp $O/tests.log $O/${tag}_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu.sh bench $tag $extra "$@"
