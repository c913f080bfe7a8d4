#!/bin/bash
# A/B variant of libqpb.so whose n<=32 wave kernel comes from another
# qpb_gi_wave.hip source, built with VFLAGS:
#   VFLAGS=-D... tools/build_variant_wave.sh <qpb_gi_wave source> <name>  -> lib/libqpb_<name>.so
set -e
src=$(realpath "$1"); name=$2
cd "$(dirname "$0")/../embedded-qp-solver_amd"
make -s ARCH=gfx950 lib/libqpb.so
cp "$src" csrc/zz_wvariant_$name.hip
/opt/rocm/bin/hipcc -std=c++20 -O3 --offload-arch=gfx950 -fPIC -I../include -I../include/compat -Icsrc \
  -Wno-unused-function ${VFLAGS:-} -c csrc/zz_wvariant_$name.hip -o build/wvariant_$name.o
rm -f csrc/zz_wvariant_$name.hip
objs=$(ls build/qpb_*.o build/compat.o | grep -v "build/qpb_gi_wave.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-Bsymbolic -o lib/libqpb_$name.so build/wvariant_$name.o $objs
echo lib/libqpb_$name.so
