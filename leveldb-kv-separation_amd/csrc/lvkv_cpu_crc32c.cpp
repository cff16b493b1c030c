// Per-call host CRC32C behind the drop-in symbols (leveldb::crc32c::Extend,
// util/crc32c.cc:276; Google crc32c_extend, port/port_stdcxx.h:208-210).
//
// Why this stays on the CPU: every reference call site checksums ONE buffer
// synchronously (<= 32 KiB, table/table_builder.cc:201, db/log_writer.cc:94)
// and a GPU round trip (> 10 us) loses to a ~1 us CPU CRC of 4 KiB. The GPU
// is reached through the batch API in lvkv_capi.cpp instead.
//
// Two implementations, chosen once at load: the SSE4.2 `crc32` instruction
// (which computes exactly the CRC32C register update) and a portable
// slicing-by-8 over tables generated from the GF(2) operators in
// lvkv_tables.cpp. Neither shares code with oracle/.
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <mutex>

#include "lvkv_tables.h"

#if defined(__x86_64__)
#include <cpuid.h>
#endif

namespace lvkv {
namespace {

uint32_t g_slice8[8][256];
std::once_flag g_slice8_once;

void init_slice8() {
  // g_slice8[k][b] = register contribution of byte b followed by k zero bytes.
  for (int k = 0; k < 8; ++k) {
    const Gf2Op z = gf2_zero_advance(static_cast<uint64_t>(k) + 1);
    for (uint32_t b = 0; b < 256; ++b) g_slice8[k][b] = gf2_apply(z, b);
  }
}

uint32_t extend_portable(uint32_t crc, const uint8_t* p, size_t n) {
  std::call_once(g_slice8_once, init_slice8);
  uint32_t reg = crc ^ 0xffffffffu;
  while (n != 0 && (reinterpret_cast<uintptr_t>(p) & 7u) != 0) {
    reg = g_slice8[0][(reg ^ *p++) & 0xffu] ^ (reg >> 8);
    --n;
  }
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= reg;
    reg = g_slice8[7][lo & 0xffu] ^ g_slice8[6][(lo >> 8) & 0xffu] ^
          g_slice8[5][(lo >> 16) & 0xffu] ^ g_slice8[4][lo >> 24] ^
          g_slice8[3][hi & 0xffu] ^ g_slice8[2][(hi >> 8) & 0xffu] ^
          g_slice8[1][(hi >> 16) & 0xffu] ^ g_slice8[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n-- != 0) reg = g_slice8[0][(reg ^ *p++) & 0xffu] ^ (reg >> 8);
  return reg ^ 0xffffffffu;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t extend_sse42(uint32_t crc,
                                                        const uint8_t* p,
                                                        size_t n) {
  uint64_t reg = crc ^ 0xffffffffu;
  while (n != 0 && (reinterpret_cast<uintptr_t>(p) & 7u) != 0) {
    reg = __builtin_ia32_crc32qi(static_cast<uint32_t>(reg), *p++);
    --n;
  }
  // Three independent chains over thirds of the aligned body would need a
  // shift-combine; one chain already runs ~3x the reference portable code.
  while (n >= 8) {
    uint64_t w;
    memcpy(&w, p, 8);
    reg = __builtin_ia32_crc32di(reg, w);
    p += 8;
    n -= 8;
  }
  while (n-- != 0)
    reg = __builtin_ia32_crc32qi(static_cast<uint32_t>(reg), *p++);
  return static_cast<uint32_t>(reg) ^ 0xffffffffu;
}

bool cpu_has_sse42() {
  unsigned eax, ebx, ecx, edx;
  if (!__get_cpuid(1, &eax, &ebx, &ecx, &edx)) return false;
  return (ecx & bit_SSE4_2) != 0;
}
#endif

using ExtendFn = uint32_t (*)(uint32_t, const uint8_t*, size_t);

ExtendFn pick_extend() {
#if defined(__x86_64__)
  if (cpu_has_sse42()) return extend_sse42;
#endif
  return extend_portable;
}

const ExtendFn g_extend = pick_extend();

}  // namespace

uint32_t cpu_crc32c_extend(uint32_t crc, const uint8_t* data, size_t n) {
  return g_extend(crc, data, n);
}

uint32_t cpu_crc32c_extend_portable(uint32_t crc, const uint8_t* data,
                                    size_t n) {
  return extend_portable(crc, data, n);
}

const char* cpu_crc32c_impl_name() {
  return g_extend == extend_portable ? "portable-slice8" : "sse4.2";
}

}  // namespace lvkv

// Test hook (include/lvkv_crc32c_debug.h): the portable slicing-by-8 path,
// whichever implementation the process picked.
extern "C" __attribute__((visibility("default"))) uint32_t lvkv_debug_extend_portable(
    uint32_t crc, const uint8_t* data, size_t n) {
  return lvkv::cpu_crc32c_extend_portable(crc, data, n);
}
