#!/usr/bin/env bash
# Build everything in-tree (no network, no vendored downloads: HTTP/JSON/ONNX readers are in-tree).
#   ./setup.sh            -> make (host C++ + gfx950 HIP kernels): lib/libdie.so, bin/{worker_node,gateway,loadgen}
#   ./setup.sh cmake      -> the same through CMake/Ninja
set -e
cd "$(dirname "$0")"
if [ "${1:-}" = cmake ]; then
  cmake -S . -B build/cmake -G Ninja && cmake --build build/cmake -j"${JOBS:-8}"
else
  make -j"${JOBS:-8}" ARCH=gfx950
fi
python3 -c 'import die_amd; from die_amd import native; native.lib(); print("die_amd native library OK:", native.lib_path())'
