#!/bin/bash
# A/B variant of libqpb.so with one kernel source replaced and/or built with VFLAGS:
#   VFLAGS=-D... tools/build_variant_any.sh <stem, e.g. qpb_gi_gram> <source> <name>  -> lib/libqpb_<name>.so
set -e
stem=$1; src=$(realpath "$2"); name=$3
cd "$(dirname "$0")/../embedded-qp-solver_amd"
make -s ARCH=gfx950 lib/libqpb.so
cp "$src" csrc/zz_any_$name.hip
/opt/rocm/bin/hipcc -std=c++20 -O3 --offload-arch=gfx950 -fPIC -I../include -I../include/compat -Icsrc \
  -Wno-unused-function ${VFLAGS:-} -c csrc/zz_any_$name.hip -o build/any_$name.o
rm -f csrc/zz_any_$name.hip
objs=$(ls build/qpb_*.o build/compat.o | grep -v "build/$stem.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-Bsymbolic -o lib/libqpb_$name.so build/any_$name.o $objs
echo lib/libqpb_$name.so
