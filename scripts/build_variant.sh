#!/bin/bash
# Build ab_libs/lib<name>.so: the normal objects with csrc/<file> recompiled under extra -D flags.
# usage: bash scripts/build_variant.sh <name> <file.hip> [-DFOO=1 ...]
set -e
NAME=$1; FILE=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/gemma.ggml_amd
make -s -C $PKG
mkdir -p $ROOT/ab_libs/$NAME
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -mllvm -amdgpu-mfma-vgpr-form=1 -Wno-unused-result"
/opt/rocm/bin/hipcc $FLAGS "$@" -c $PKG/csrc/$FILE -o $ROOT/ab_libs/$NAME/$FILE.o
OBJS=$(ls $PKG/build/*.o | grep -v "/$FILE.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/ab_libs/lib$NAME.so $OBJS $ROOT/ab_libs/$NAME/$FILE.o -L/opt/rocm/lib -lrccl -lpthread
echo built ab_libs/lib$NAME.so
