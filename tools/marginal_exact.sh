#!/bin/bash
# Marginal cost of each kernel class on the exact-fp32 leg (configs[1], three calls in flight): the bench on
# timing variants of the library whose named kernel returns at once (tools/build_variant.sh -DND_SKIP_*;
# results are garbage, the work of every other kernel is unchanged; greedy decoding runs its 100 steps
# whatever the values).   bash tools/marginal_exact.sh base skip_memattn ...
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for rep in 1 2; do
  for v in "$@"; do
    NANODEC_AB=1 NANODEC_LIB=$R/tools/_ab/$v.so timeout -k 10 300 python -u bench.py --allow-switches --steps 80 --warmup 3 \
      --cpu-baseline 0 --exact 1 --host-inclusive 0 --read-shard 0 --config-legs 0 --no-roofline \
      > $O/margx_${v}_$rep.json 2> $O/margx_${v}_$rep.err || exit $?
    python3 -c "
import json; d=json.loads(open('$O/margx_${v}_$rep.json').read().strip().splitlines()[-1])
print('%-14s rep %d: exact %.3f ms/call  headline %.3f ms/call' % ('$v', $rep, d['exact_fp32']['ms_per_step'], d['ms_per_step']))"
  done
done
