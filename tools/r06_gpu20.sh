# encoder FFN block with non-temporal activation rows (FF_NT_ACT): fused-block parity, microbench, headline A/B
cd $GRAFT_REPO_ROOT && O=$GRAFT_REPO_ROOT/gpurun_out && export PYTHONUNBUFFERED=1
for v in ntoff nton ntoff nton; do
  echo "== $v"; NANODEC_AB=1 NANODEC_LIB=$GRAFT_REPO_ROOT/tools/_ab/$v.so timeout -k 10 200 python -u tools/microbench.py encffn > $O/mb_encffn_$v.log 2>&1 || exit $?
  grep enc-ffn $O/mb_encffn_$v.log
done
NANODEC_AB=1 NANODEC_LIB=$GRAFT_REPO_ROOT/tools/_ab/nton.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "enc_ffn" > $O/r06_gpu20_tests.log 2>&1 || { tail -20 $O/r06_gpu20_tests.log; exit 1; }
tail -1 $O/r06_gpu20_tests.log
bash tools/ab_lib.sh ntoff nton
