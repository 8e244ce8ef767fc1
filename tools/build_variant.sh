#!/bin/bash
# Build an A/B variant of the C-ABI library with extra flags for ONE source file (the rest from the
# default build): bash tools/build_variant.sh <name> <source.hip> "<hipcc flags>"
# -> build_ab/<name>.so (git-ignored, travels to the GPU box with gpurun).
set -eu
R="$(cd "$(dirname "$0")/.." && pwd)"
name="$1"; src="$2"; flags="$3"
C="$R/rq-vae-recommender_amd/csrc"
make -C "$C" -j8 >/dev/null
mkdir -p "$R/build_ab"
obj="$R/build_ab/$name.$(basename "$src" .hip).o"
# the Makefile's per-file flags (attention: MFMA accumulators in VGPRs)
if [ "$(basename "$src")" = "attention.hip" ]; then flags="-mllvm -amdgpu-mfma-vgpr-form $flags"; fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function $flags \
  -c "$C/$(basename "$src")" -o "$obj"
objs=""
for o in "$C"/build/*.o; do
  if [ "$(basename "$o" .o)" = "$(basename "$src" .hip)" ]; then objs="$objs $obj"; else objs="$objs $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/build_ab/$name.so" $objs
echo "built build_ab/$name.so ($flags)"
