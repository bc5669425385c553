#!/bin/bash
# GPU step for tools/lds_forms_probe.py (build the .so on the CPU first:
#   hipcc --offload-arch=gfx950 -O2 -shared -fPIC -o tools/liblds_forms.so tools/lds_forms_probe.hip)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 240 python -u tools/lds_forms_probe.py > $O/lds_forms.log 2>&1; rc=$?
grep -v amdgpu.ids $O/lds_forms.log | tail -12; exit $rc
