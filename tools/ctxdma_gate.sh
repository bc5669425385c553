# context attention change: parity tests (ctx / beam / q24 / the beam pool at the bench's config), timing alone,
# beam bench A/B against a reference library (tools/_ab/$1.so) -- bash tools/ctxdma_gate.sh REF NEW
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export PYTHONPATH=$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "ctx_attention or beam or q24 or configs[3] or config3" > $O/cq_tests.log 2>&1
rc=$?; tail -3 $O/cq_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/ctx_time.py new 2>&1 | grep -v amdgpu.ids || exit 1
bash tools/ab_lib.sh $1 $2 --mode beam --batch 1024 --steps 20 --warmup 2
