#!/bin/bash
# One parameterised GPU-box driver (run through gpurun from the repo root).
# Each step runs under its own time limit; the script stops at the first
# failing step (no retries).
#
#   bash tools/gpu.sh test                      smoke() + every -m gpu test
#   bash tools/gpu.sh bench TAG [bench args]    one bench line -> gpurun_out/TAG.json
#   bash tools/gpu.sh prof TAG [bench args]     rocprofv3 --kernel-trace --stats of a short bench
#   bash tools/gpu.sh pmc TAG "CTRS" [args]     one rocprofv3 --pmc pass (one counter group)
#   bash tools/gpu.sh mfma TAG [args]          rocprofv3 MFMA counter pass -> gpurun_out/TAG_mfma.json
#   bash tools/gpu.sh pmcmb TAG "CTRS" CASE   one --pmc pass over a microbench case
#   bash tools/gpu.sh pmcpy TAG "CTRS" tool.py [args]   one --pmc pass over a python tool
#   bash tools/gpu.sh list                      rocprofv3 -L (available counters)
#   bash tools/gpu.sh py TAG script.py [args]   any python tool (probes, microbenches)
# Steps chain with &&:  bash tools/gpu.sh test && bash tools/gpu.sh bench r02_greedy
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
step=$1; shift
SHORT="--config-legs 0 --steps 5 --warmup 2 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 --no-roofline"
case $step in
  test)
    cd $R
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
    rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
    timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
      -p no:cacheprovider > $O/tests.log 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log; exit $rc ;;
  bench)
    tag=$1; shift; cd $R
    timeout -k 10 900 python -u bench.py "$@" > $O/$tag.json 2> $O/$tag.err
    rc=$?; echo "bench $tag rc=$rc"; tail -c 3000 $O/$tag.json; exit $rc ;;
  prof)
    tag=$1; shift
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv -- \
      python3 $R/bench.py $SHORT "$@" > $O/$tag.log 2>&1
    rc=$?; echo "prof $tag rc=$rc"; [ $rc -ne 0 ] && exit $rc
    python3 $R/tools/profsum.py $O/$tag/run_kernel_stats.csv 7 > $O/${tag}_kernel_stats.txt
    # keep the stats, drop the per-dispatch trace (gpurun copies back at most 64 MiB)
    find $O/$tag -name '*.csv' ! -name '*kernel_stats.csv' -delete
    head -30 $O/${tag}_kernel_stats.txt; exit 0 ;;
  steps)
    # kernel trace of a short bench, summarised per launch on the box (tools/trace_steps.py)
    tag=$1; shift
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv -- \
      python3 $R/bench.py $SHORT "$@" > $O/$tag.log 2>&1
    rc=$?; echo "steps $tag rc=$rc"; [ $rc -ne 0 ] && exit $rc
    python3 $R/tools/profsum.py $O/$tag/run_kernel_stats.csv 7 > $O/${tag}_kernel_stats.txt
    python3 $R/tools/trace_steps.py $O/$tag/run_kernel_trace.csv > $O/${tag}_steps.txt
    find $O/$tag -name '*.csv' ! -name '*kernel_stats.csv' -delete
    head -20 $O/${tag}_steps.txt; exit 0 ;;
  busy)
    # kernel trace of a bench run: how busy the GPU is, window by window (tools/trace_busy.py)
    tag=$1; shift
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 600 rocprofv3 --kernel-trace -d $O/$tag -o run --output-format csv -- \
      python3 $R/bench.py $SHORT "$@" > $O/$tag.log 2>&1
    rc=$?; echo "busy $tag rc=$rc"; [ $rc -ne 0 ] && exit $rc
    python3 $R/tools/trace_busy.py $(find $O/$tag -name '*kernel_trace.csv' | head -1) 5 > $O/${tag}_busy.txt
    find $O/$tag -name '*.csv' -delete
    tail -20 $O/${tag}_busy.txt; exit 0 ;;
  pmc)
    tag=$1; ctrs=$2; shift 2
    cd /tmp && export TMPDIR=/tmp
    timeout -s KILL 240 rocprofv3 --pmc $ctrs --kernel-trace -d $O/$tag -o run --output-format csv -- \
      python3 $R/bench.py --config-legs 0 --steps 1 --warmup 1 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 \
      --no-roofline "$@" > $O/$tag.log 2>&1
    rc=$?; echo "pmc $tag rc=$rc"; exit $rc ;;
  mfma)
    # MFMA utilisation counters (one pass: 4 SQ + 1 GRBM), summarised per kernel
    tag=$1; shift
    cd /tmp && export TMPDIR=/tmp
    timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 \
      SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/$tag -o run --output-format csv -- \
      python3 $R/bench.py --config-legs 0 --steps 1 --warmup 1 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 \
      --no-roofline "$@" > $O/$tag.log 2>&1
    rc=$?; echo "mfma $tag rc=$rc"; [ $rc -ne 0 ] && exit $rc
    python3 $R/tools/mfma_summary.py $O/$tag/run_counter_collection.csv $tag $O/${tag}_mfma.json | head -40
    rm -rf $O/$tag; exit 0 ;;
  pmcmb)
    # one --pmc pass over a tools/microbench.py case (plain launches)
    tag=$1; ctrs=$2; shift 2
    cd /tmp && export TMPDIR=/tmp
    MB_EAGER=1 timeout -s KILL 180 rocprofv3 --pmc $ctrs --kernel-trace -d $O/$tag -o run --output-format csv -- \
      python3 $R/tools/microbench.py "$@" > $O/$tag.log 2>&1
    rc=$?; echo "pmcmb $tag rc=$rc"; exit $rc ;;
  pmcpy)
    # one --pmc pass over any python tool (e.g. tools/pmc_beam.py run K)
    tag=$1; ctrs=$2; shift 2
    cd /tmp && export TMPDIR=/tmp
    timeout -s KILL 240 rocprofv3 --pmc $ctrs --kernel-trace -d $O/$tag -o run --output-format csv -- \
      python3 "$@" > $O/$tag.log 2>&1
    rc=$?; echo "pmcpy $tag rc=$rc"; exit $rc ;;
  list)
    cd /tmp && export TMPDIR=/tmp
    timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1
    rc=$?; echo "list rc=$rc"; grep -c . $O/counters.txt; exit $rc ;;
  py)
    tag=$1; shift; cd $R
    timeout -k 10 600 python -u "$@" > $O/$tag.log 2>&1
    rc=$?; echo "py $tag rc=$rc"; tail -20 $O/$tag.log; exit $rc ;;
  ptrace)
    # rocprofv3 --kernel-trace of any python tool (queue ids, start/end per dispatch)
    tag=$1; shift
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace -d $O/$tag -o run --output-format csv -- \
      python3 "$@" > $O/$tag.log 2>&1
    rc=$?; echo "ptrace $tag rc=$rc"; tail -3 $O/$tag.log; exit $rc ;;
  *) echo "unknown step $step"; exit 2 ;;
esac
