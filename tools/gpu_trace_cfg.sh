# kernel traces of the beam (configs[3]) and NanoEncoder (configs[2]) benches
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/tc; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/beam -o run --output-format csv -- python3 $R/bench.py --mode beam --batch 1024 --steps 1 --warmup 1 --cpu-baseline 0 --no-roofline > $O/beam.json 2> $O/beam.err
rc=$?; echo "beam rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/nano -o run --output-format csv -- python3 $R/bench.py --encoder nano --steps 2 --warmup 1 --cpu-baseline 0 --no-roofline > $O/nano.json 2> $O/nano.err
rc=$?; echo "nano rc=$rc"; exit $rc
