#!/bin/bash
# Build an A/B variant of libqpb.so whose n<=16 kernel comes from another
# qpb_gi.hip source:  tools/build_variant.sh <qpb_gi source> <name>
# -> embedded-qp-solver_amd/lib/libqpb_<name>.so (-Bsymbolic: binds to its own
# launchers even when libqpb.so is loaded RTLD_GLOBAL in the same process)
set -e
src=$(realpath "$1"); name=$2
cd "$(dirname "$0")/../embedded-qp-solver_amd"
make -s ARCH=gfx950 lib/libqpb.so
cp "$src" csrc/zz_variant_$name.hip
/opt/rocm/bin/hipcc -std=c++20 -O3 --offload-arch=gfx950 -fPIC -I../include -I../include/compat -Icsrc \
  -Wno-unused-function ${VFLAGS:-} -c csrc/zz_variant_$name.hip -o build/variant_$name.o
rm -f csrc/zz_variant_$name.hip
objs=$(ls build/qpb_*.o build/compat.o | grep -v "build/qpb_gi.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-Bsymbolic -o lib/libqpb_$name.so build/variant_$name.o $objs
echo lib/libqpb_$name.so
