#!/bin/bash
# Co-residency discriminator for the closed-form layer-0 attention
# (enc_attention_rank2_kernel): parity of the 64 KB layout
# alone, then tools/rank2_probe.py once per LDS layout (engine A encodes beside
# engine B translating; A's memory bank against its serial run):
#   default         65,536 B allocated, every access below 65,536
#   r2_ld17         67,584 B, E[y]/E[r] rows of wave 7 past 65,536 (round 3)
#   r2_pad2k        67,584 B allocated, every access below 65,536
#   r2_pad20k       86,016 B allocated (one workgroup per CU), accesses below 65,536
#   r2_ld17_pad18k  86,016 B allocated, accesses past 65,536
#   r2_front2k      67,584 B, slabs shifted 2 KB: single-address ds_read_b32 / ds_write_b32 past 65,536
#   r2_ld18         69,632 B, [64][18] rows: ds_read2_b64 / ds_write2_b64 past 65,536
# Variants: bash tools/build_variant.sh NAME attention.hip "-DND_R2_EXLD=17 -DND_R2_PAD=..."
#   bash tools/r2_lds.sh [variant ...]   (default: the first five)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
VARIANTS=${*:-default r2_ld17 r2_pad2k r2_pad20k r2_ld17_pad18k}
ND_ENC_ATTN0=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -m gpu --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "encoder or golden" > $O/r2lds_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $O/r2lds_parity.log; [ $rc -ne 0 ] && exit $rc
for v in $VARIANTS; do
  lib=$R/nanodecoder_amd/libnanodec_hip.so
  [ $v != default ] && lib=$R/tools/_ab/$v.so
  NANODEC_AB=1 NANODEC_LIB=$lib ND_ENC_ATTN0=1 PROBE_ROUNDS=4 PROBE_SHORT=1 PROBE_WHERE=1 timeout -k 10 200 \
    python -u tools/rank2_probe.py > $O/r2lds_$v.log 2>&1 || exit $?
  echo "== $v"; grep -v amdgpu.ids $O/r2lds_$v.log | grep -E "round|bad chunks" | tail -6
done
