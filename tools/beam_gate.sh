#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "bank_d8" > $O/bb_op.log 2>&1
rc=$?; echo "op rc=$rc"; tail -15 $O/bb_op.log; [ $rc -ne 0 ] && exit $rc
ND_BEAM_BANK=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "beam or classic or pool" > $O/bb_tests.log 2>&1
rc=$?; echo "beam tests rc=$rc"; tail -15 $O/bb_tests.log; [ $rc -ne 0 ] && exit $rc
B="--mode beam --batch 1024 --steps 4 --warmup 2 --config-legs 0 --cpu-baseline 0 --exact 0 --host-inclusive 0 --read-shard 0"
timeout -k 10 300 python -u bench.py $B > $O/bb_bench1.json 2> $O/bb_bench1.err; rc=$?; echo "bench kv (default) rc=$rc"; tail -c 1500 $O/bb_bench1.json; [ $rc -ne 0 ] && exit $rc
ND_BEAM_BANK=1 timeout -k 10 300 python -u bench.py $B --allow-switches > $O/bb_bench0.json 2> $O/bb_bench0.err; rc=$?; echo "bench beam bank rc=$rc"; tail -c 1500 $O/bb_bench0.json; exit $rc
