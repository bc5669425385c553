#!/bin/bash
# Build a timing variant of the library: one csrc file recompiled with extra
# flags, linked with the current objects of the others -> tools/_ab/NAME.so
#   bash tools/build_variant.sh NAME FILE.hip "-DFOO=1 -DBAR=2" [SOURCE]
# (SOURCE: another version of csrc/FILE.hip to compile in its place, e.g. the previous commit's)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; src=$2; flags=$3; alt=${4:-}
python3 -c "import sys; sys.path.insert(0, '$R'); from nanodecoder_amd import build; build.build()" > /dev/null
mkdir -p $R/tools/_ab /tmp/ndvar
objs=""
for o in $R/nanodecoder_amd/_build/*.o; do
  case $(basename $o) in asan_*) continue ;; esac
  if [ "$(basename $o .o).hip" = "$src" ]; then
    /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -I$R/nanodecoder_amd/csrc \
      -I$R/include $flags -c ${alt:-$R/nanodecoder_amd/csrc/$src} -o /tmp/ndvar/$name.o
    objs="$objs /tmp/ndvar/$name.o"
  else
    objs="$objs $o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/tools/_ab/$name.so $objs
echo "tools/_ab/$name.so"
