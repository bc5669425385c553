# HBM traffic per launch for the dominant kernel of every bench line:
# separate --pmc FETCH_SIZE and --pmc WRITE_SIZE passes (one counter group per
# run) over the greedy and the beam bench; tools/pmc_summary.py merges them
# into profiles/pmc_summary.json (FETCH doubled per the gfx950 correction).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmcall; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for mode in greedy beam; do
  if [ $mode = beam ]; then A="--mode beam --batch 1024"; else A=""; fi
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace -d $O/${mode}_$ctr -o run --output-format csv -- python3 $R/bench.py $A --steps 1 --warmup 1 --cpu-baseline 0 --no-roofline > $O/${mode}_$ctr.log 2>&1
    rc=$?; echo "$mode $ctr rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
cd $R
python3 tools/pmc_summary.py $O/greedy_FETCH_SIZE/run_counter_collection.csv $O/greedy_WRITE_SIZE/run_counter_collection.csv $O/greedy.json > /dev/null
python3 tools/pmc_summary.py $O/beam_FETCH_SIZE/run_counter_collection.csv $O/beam_WRITE_SIZE/run_counter_collection.csv $O/beam.json > /dev/null
echo "summaries rc=$?"
