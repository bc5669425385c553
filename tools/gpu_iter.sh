# build-measure iteration: parity tests, bench, kernel profile
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-chunks 2 > gpurun_out/b.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/b.log | cut -c1-400
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/microbench.py dec256 > gpurun_out/micro.log 2>&1
echo "micro rc=$?"; cat gpurun_out/micro.log | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --no-roofline > $R/gpurun_out/prof.log 2>&1
echo "prof rc=$?"
