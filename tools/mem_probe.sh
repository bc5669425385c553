#!/bin/bash
# The fp32 bank kernel's time with parts of its work removed (timing-only variants of mem_attention.hip, built
# here with tools/build_variant.sh into tools/_ab/): base, no loads (L2-resident data), no score products, no
# context product.  Each variant runs twice, alternated.   bash tools/mem_probe.sh [variants]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
vs=${@:-"mb_base mb_noload mb_noscore mb_nou"}
for rep in 1 2; do
  for v in $vs; do
    NANODEC_AB=1 NANODEC_LIB=$R/tools/_ab/$v.so timeout -k 10 120 python -u tools/mem_probe.py $v 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
