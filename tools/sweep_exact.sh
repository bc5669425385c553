#!/bin/bash
# same-box sweep of bench.py argument sets on the exact-fp32 leg (configs[1]), each run twice, interleaved:
#   bash tools/sweep_exact.sh "ARGS1" "ARGS2" ...   (prints the exact leg's ms per call and the headline's)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for rep in 1 2; do
  i=0
  for a in "$@"; do
    i=$((i + 1))
    timeout -k 10 300 python -u bench.py --steps 160 --warmup 3 --cpu-baseline 0 --exact 1 --host-inclusive 0 \
      --read-shard 0 --config-legs 0 $a > $O/sweepx_${i}_$rep.json 2> $O/sweepx_${i}_$rep.err || exit $?
    python3 -c "
import json; d=json.loads(open('$O/sweepx_${i}_$rep.json').read().strip().splitlines()[-1]); e=d['exact_fp32']
print('[$a] rep $rep: exact %.3f ms/call (frac %.4f)  headline %.3f ms/call' % (e['ms_per_step'], e['roofline']['frac'], d['ms_per_step']))"
  done
done
