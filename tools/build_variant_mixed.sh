#!/bin/bash
# A/B variant of libqpb.so whose mixed-precision kernel is built with VFLAGS:
#   VFLAGS=-D... tools/build_variant_mixed.sh <name>  -> lib/libqpb_<name>.so
set -e
name=$1
cd "$(dirname "$0")/../embedded-qp-solver_amd"
make -s ARCH=gfx950 lib/libqpb.so
/opt/rocm/bin/hipcc -std=c++20 -O3 --offload-arch=gfx950 -fPIC -I../include -I../include/compat -Icsrc \
  -Wno-unused-function ${VFLAGS:-} -c csrc/qpb_gi_mixed.hip -o build/variant_mx_$name.o
objs=$(ls build/qpb_*.o build/compat.o | grep -v "build/qpb_gi_mixed.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-Bsymbolic -o lib/libqpb_$name.so build/variant_mx_$name.o $objs
echo lib/libqpb_$name.so
