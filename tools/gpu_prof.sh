set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof1 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 > $R/gpurun_out/prof1.log 2>&1
rc=$?; echo "prof rc=$rc"
if [ $rc -eq 0 ]; then
  timeout -k 10 600 python3 $R/bench.py --mode beam --batch 1024 --steps 2 --warmup 1 --cpu-chunks 2 > $R/gpurun_out/beam1.log 2>&1
  echo "beam rc=$?"
fi
