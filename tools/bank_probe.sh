#!/bin/bash
# The bank kernel's time with parts of its work removed (timing-only variants of bank8.hip, built here with
# tools/build_variant.sh into tools/_ab/): base, no loads (L2-resident data), no score MFMAs, no context
# product, no digit conversion.  Each variant runs twice, alternated.   bash tools/bank_probe.sh [variants]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
vs=${@:-"b8_base b8_noload b8_noscore b8_nou b8_nocvt"}
for rep in 1 2; do
  for v in $vs; do
    NANODEC_AB=1 NANODEC_LIB=$R/tools/_ab/$v.so timeout -k 10 120 python -u tools/bank_probe.py $v 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
