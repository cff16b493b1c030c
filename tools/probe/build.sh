#!/bin/bash
# Build tools/probe/libprobe.so (timing probes; not part of the product).
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
R=$(cd "$HERE/../.." && pwd)
PKG="$R/leveldb-kv-separation_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-value -Wno-unused-result -shared \
  -I "$R/include" -I "$PKG/csrc" "$HERE/probe.hip" "$PKG/csrc/lvkv_tables.cpp" \
  -L "$PKG" -llvkv_crc32c -Wl,-rpath,'$ORIGIN/../../leveldb-kv-separation_amd' \
  -o "$HERE/libprobe.so"
# Engine probe kernels: an unbundled gfx950 code object for lvkv_engine_load_probe.
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only --no-gpu-bundle-output \
  -I "$R/include" -I "$PKG/csrc" -c "$HERE/engine_probe_kernels.hip" -o "$HERE/engine_probe_kernels.co"
