#!/bin/bash
# Build ab_libs/lib<name>.so: the normal objects with csrc/<file>[,<file>...] recompiled under extra
# -D flags.  usage: bash scripts/build_variant.sh <name> <file.hip[,file2.hip]> [-DFOO=1 ...]
set -e
NAME=$1; FILES=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/gemma.ggml_amd
make -s -C $PKG
mkdir -p $ROOT/ab_libs/$NAME
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -mllvm -amdgpu-mfma-vgpr-form=1 -Wno-unused-result"
OBJS=$(ls $PKG/build/*.o)
VOBJS=""
for FILE in ${FILES//,/ }; do
  XL=""; [[ $FILE == *.cpp ]] && XL="-x hip"
  /opt/rocm/bin/hipcc $FLAGS "$@" $XL -c $PKG/csrc/$FILE -o $ROOT/ab_libs/$NAME/$FILE.o &
  OBJS=$(echo "$OBJS" | grep -v "/$FILE.o$")
  VOBJS="$VOBJS $ROOT/ab_libs/$NAME/$FILE.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/ab_libs/lib$NAME.so $OBJS $VOBJS -L/opt/rocm/lib -lrccl -lpthread
echo built ab_libs/lib$NAME.so
