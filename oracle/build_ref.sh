#!/usr/bin/env bash
# Compile the REFERENCE's own CPly (miniply + C wrapper) from the sources where they
# lie under /root/reference into oracle/_ref/libcply_ref.so.  Test infrastructure only:
# it produces the PLY golden vectors (tests/golden/make_ply_golden.py) that pin the
# product's fresh PLY reader.  Nothing is copied into the repo; oracle/_ref/ is
# git-ignored.  Sources: Sources/CPly/miniply.cpp, Sources/CPly/wrapper.cpp,
# Sources/CPly/include/{miniply.h,PLYReaderWrapper.h} (Package.swift:11-19).
set -euo pipefail
REF=${REF:-/root/reference}
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
mkdir -p "$HERE/_ref"
g++ -std=c++17 -O2 -fPIC -shared \
    -I "$REF/Sources/CPly/include" \
    "$REF/Sources/CPly/miniply.cpp" "$REF/Sources/CPly/wrapper.cpp" \
    -o "$HERE/_ref/libcply_ref.so"
echo "built $HERE/_ref/libcply_ref.so"
