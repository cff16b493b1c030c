#!/bin/bash
# Builds the CPU SIMT emulation of the device Zstd compressor (debugging aid,
# not part of the product): the kernel source compiled by g++ against
# tools/simt_emu/hip/hip_runtime.h, with AddressSanitizer. Output:
# build/simt_emu/zstdc_emu (see zstdc_emu.cc; tools/simt_emu/zstdc_check.py).
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
REPO=$(cd "$HERE/../.." && pwd)
OUT=$REPO/build/simt_emu
mkdir -p "$OUT"
# the dynamic LDS declaration becomes the emulator's per-workgroup buffer
sed 's/^\(\s*\)extern __shared__ __attribute__((aligned(16))) uint8_t smem\[\];/\1uint8_t* smem = emu::lds_base;/' \
  "$REPO/leveldb-kv-separation_amd/csrc/lvkv_zstd_compress.hip" > "$OUT/lvkv_zstd_compress_emu.cc"
g++ -std=c++20 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -DLVKV_SIMT_EMU \
  -I "$HERE" -I "$REPO/include" -I "$REPO/leveldb-kv-separation_amd/csrc" \
  -include "$HERE/hip/hip_runtime.h" \
  "$OUT/lvkv_zstd_compress_emu.cc" "$HERE/zstdc_emu.cc" -o "$OUT/zstdc_emu" -lpthread
echo "$OUT/zstdc_emu"
