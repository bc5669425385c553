# beam self-attention change: op + beam parity tests, then the configs[3] bench A/B against tools/_ab/$1.so
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "self_attention or beam or config3 or configs[3] or pool" > $O/sb_tests.log 2>&1
rc=$?; tail -3 $O/sb_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_lib.sh $1 $2 --mode beam --batch 1024 --steps 20 --warmup 2
