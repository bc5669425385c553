#!/bin/bash
# same-box A/B of two library builds on the exact-fp32 leg of the greedy bench (configs[1], 3 calls in flight):
#   bash tools/ab_exact.sh A B [bench args]   (tools/_ab/A.so, tools/_ab/B.so via NANODEC_LIB; A B A B)
a=$1; b=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for rep in 1 2; do
  for v in $a $b; do
    NANODEC_AB=1 NANODEC_LIB=$R/tools/_ab/$v.so timeout -k 10 300 python -u bench.py --allow-switches --steps 160 --warmup 3 \
      --cpu-baseline 0 --exact 1 --host-inclusive 0 --read-shard 0 --config-legs 0 "$@" \
      > $O/ab_exact_${v}_$rep.json 2> $O/ab_exact_${v}_$rep.err || exit $?
    python3 -c "
import json; d=json.loads(open('$O/ab_exact_${v}_$rep.json').read().strip().splitlines()[-1]); e=d['exact_fp32']
print('$v rep $rep: exact %.3f ms/call (frac %.4f)  headline %.3f ms/call' % (e['ms_per_step'], e['roofline']['frac'], d['ms_per_step']))"
  done
done
