#!/bin/bash
# Build a variant of libpgmi.so with extra compiler flags into pgmi/libpgmi_<name>.so (same-box A/Bs
# via PGMI_LIB_PATH, tools/b8_ab.sh / tools/ab_bench.sh).  usage: bash tools/build_variant.sh <name> "<flags>"
set -e
N=$1; F=$2
C=$(dirname $0)/../multimodal-financial-analysis-tool-using-paligemma_amd/csrc
B=$C/build_$N
mkdir -p $B
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -Wno-unused-function $F"
for f in $C/*.hip; do
  o=$B/$(basename $f .hip).o
  extra=""
  [ "$(basename $f)" = kernels_gemm.hip ] && extra="-mllvm -amdgpu-mfma-vgpr-form"
  if [ ! -f $o ] || [ $f -nt $o ]; then /opt/rocm/bin/hipcc $FLAGS $extra -c $f -o $o & fi
done
wait
/opt/rocm/bin/hipcc $FLAGS -shared $B/*.o -o $C/../pgmi/libpgmi_$N.so -ldl
echo built $C/../pgmi/libpgmi_$N.so
