set -u
mkdir -p gpurun_out
python -c "
import sys; sys.path.insert(0,'.')
from nanodecoder_amd import _lib; L=_lib.lib()
print([l.split()[-1] for l in open('/proc/self/maps') if 'amdhip64' in l][:3])" > gpurun_out/maps.log 2>&1
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -le 1 ]; then
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-chunks 2 > gpurun_out/b1.log 2>&1
  echo "bench rc=$?"
fi
