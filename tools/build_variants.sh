#!/usr/bin/env bash
# Build tuning variants of libmyrt.so into build_variants/ (git-ignored; travels with gpurun).
# usage: tools/build_variants.sh NAME "-DFLAG=.." [NAME "-D.." ...]   ->  build_variants/libmyrt_NAME.so
set -eu
cd "$(dirname "$0")/.."
mkdir -p build_variants
C=myraytracer_amd/csrc
while [ $# -ge 2 ]; do
  name="$1"; flags="$2"; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared $flags \
    -o "build_variants/libmyrt_${name}.so" $C/render.hip $C/scene.cpp $C/ply.cpp $C/sceneio.cpp &
done
wait
ls -la build_variants
