set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd $R
for rep in 1 2; do
for inf in 2 3 4; do
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --inflight $inf --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 --config-legs 0 > $O/inf_$inf.json 2> $O/inf_$inf.err || exit 1
  python3 -c "
import json; d=json.loads(open('$O/inf_$inf.json').read().strip().splitlines()[-1]); r=d['roofline']
print('inflight %d: %.3f ms/call (%.3f M), bank %.2f us' % ($inf, d['ms_per_step'], d['value']/1e6, 1e3*r['avg_launch_ms']))"
done
done
