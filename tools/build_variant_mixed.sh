#!/bin/bash
# A/B variant of libqpb.so whose mixed-precision kernel is built with VFLAGS:
#   VFLAGS=-D... tools/build_variant_mixed.sh <name>  -> lib/libqpb_<name>.so
set -e
name=$1
cd "$(dirname "$0")/../embedded-qp-solver_amd"
make -s ARCH=gfx950 lib/libqpb.so
/opt/rocm/bin/hipcc -std=c++20 -O3 --offload-arch=gfx950 -fPIC -I../include -I../include/compat -Icsrc \
  -Wno-unused-function ${VFLAGS:-} -c csrc/qpb_gi_mixed.hip -o build/variant_mx_$name.o
objs="build/qpb_gi_box.o build/qpb_gi.o build/qpb_gi_wave.o build/qpb_gi_block.o build/qpb_gi_gram.o build/qpb_ref.o build/qpb_gen.o build/qpb_api.o build/compat.o build/qpb_wire.o"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-Bsymbolic -o lib/libqpb_$name.so build/variant_mx_$name.o $objs
echo lib/libqpb_$name.so
