#!/bin/bash
# Build a variant of libm3d.so with extra compile flags into tools/ab/<name>.so (A/B timing in the
# same gpurun call; tools that take AB_LIB load it).  Usage: [ABX=flags] tools/ab_build.sh NAME [-DFLAG=V ...]
set -eu
name=$1; shift
cd "$(dirname "$0")/../3d-matching_amd/csrc"
out=/tmp/ab_$name; rm -rf $out; mkdir -p $out ../../tools/ab
F="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -I../../include -w $*"
X=${ABX:-"-fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form"}  # ransac/icp flags (ABX overrides)
for f in ransac icp; do /opt/rocm/bin/hipcc $F $X -c $f.hip -o $out/$f.o & done
for f in grid prep feat; do /opt/rocm/bin/hipcc $F -c $f.hip -o $out/$f.o & done
for f in api comm hostio; do /opt/rocm/bin/hipcc $F -x hip -c $f.cpp -o $out/$f.o & done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/ab/$name.so $out/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "tools/ab/$name.so"
