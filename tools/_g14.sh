set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd $R
for rep in 1 2; do
for nt in none 1 0,1; do
  a=$nt; [ $nt = none ] && a=""
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --bank-nt-lanes "$a" --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0 --config-legs 0 > $O/nt_$nt.json 2> $O/nt_$nt.err || exit 1
  python3 -c "
import json; d=json.loads(open('$O/nt_$nt.json').read().strip().splitlines()[-1]); r=d['roofline']
print('nt lanes %-5s: %.3f ms/call, bank %.2f us' % ('$nt', d['ms_per_step'], 1e3*r['avg_launch_ms']))"
done
done
