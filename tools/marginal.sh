#!/bin/bash
# Marginal cost of each kernel class, one call vs three calls in flight:
# the greedy bench on timing variants of the library whose named kernel
# returns at once (tools/build_variant.sh -DND_SKIP_*; results are garbage,
# the work of every other kernel is unchanged).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for v in base skip_bank skip_p16 skip_ffn skip_self skip_eattn; do
  for inf in 1 3; do
    NANODEC_AB=1 NANODEC_LIB=$R/tools/_ab/$v.so timeout -k 10 300 python -u bench.py --allow-switches --steps 40 --warmup 3 --inflight $inf \
      --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 --config-legs 0 --no-roofline \
      > $O/marg_${v}_$inf.json 2> $O/marg_${v}_$inf.err || exit $?
    python3 -c "
import json; d=json.loads(open('$O/marg_${v}_$inf.json').read().strip().splitlines()[-1])
print('%-11s inflight %d: %.3f ms/call' % ('$v', $inf, d['ms_per_step']))"
  done
done
