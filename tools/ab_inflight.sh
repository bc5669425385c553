# same-box A/B of the calls in flight (EnginePool lanes) on the greedy bench: bash tools/ab_inflight.sh "3 4" [bench args]
vals=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for rep in 1 2; do
  for v in $vals; do
    timeout -k 10 300 python -u bench.py --inflight $v --steps 40 --warmup 3 --cpu-baseline 0 --exact 0 --host-inclusive 0 \
      --read-shard 0 --config-legs 0 "$@" > $O/abi_${v}_$rep.json 2> $O/abi_${v}_$rep.err || exit $?
    python3 -c "
import json; d=json.loads(open('$O/abi_${v}_$rep.json').read().strip().splitlines()[-1])
print('inflight $v rep $rep: %.3f ms/step  value %.0f' % (d['ms_per_step'], d['value']))"
  done
done
