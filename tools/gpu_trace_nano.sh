# kernel trace of the NanoEncoder greedy bench (configs[2])
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/tn; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 $R/bench.py --encoder nano --steps 1 --warmup 1 --cpu-baseline 0 --no-roofline > $O/b.json 2> $O/b.err
rc=$?; echo "rc=$rc"; exit $rc
