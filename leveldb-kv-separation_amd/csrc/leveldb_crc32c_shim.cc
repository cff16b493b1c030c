// Link-level drop-ins for the reference's CRC32C symbols.
//
// 1. leveldb::crc32c::Extend (util/crc32c.h:17, util/crc32c.cc:276) — the one
//    out-of-line CRC symbol imported by table_builder.cc.o, format.cc.o,
//    log_writer.cc.o and log_reader.cc.o (mangled _ZN7leveldb6crc32c6ExtendEjPKcm).
//    Value/Mask/Unmask stay header inlines in the callers (crc32c.h:20-38).
// 2. The Google crc32c ABI (crc32c_extend / crc32c_value / ::crc32c::Extend)
//    that port::AcceleratedCRC32C binds to when HAVE_CRC32C=1
//    (port/port_stdcxx.h:208-210, CMakeLists.txt:41,281-283).
//
// Both run the per-call host implementation (lvkv_cpu_crc32c.cpp).
#include <stddef.h>
#include <stdint.h>

namespace lvkv {
uint32_t cpu_crc32c_extend(uint32_t crc, const uint8_t* data, size_t n);
}

namespace leveldb {
namespace crc32c {

__attribute__((visibility("default"))) uint32_t Extend(uint32_t init_crc,
                                                       const char* data,
                                                       size_t n) {
  return lvkv::cpu_crc32c_extend(init_crc,
                                 reinterpret_cast<const uint8_t*>(data), n);
}

}  // namespace crc32c
}  // namespace leveldb

namespace crc32c {

__attribute__((visibility("default"))) uint32_t Extend(uint32_t crc,
                                                       const uint8_t* data,
                                                       size_t count) {
  return lvkv::cpu_crc32c_extend(crc, data, count);
}

}  // namespace crc32c

extern "C" {

__attribute__((visibility("default"))) uint32_t crc32c_extend(
    uint32_t crc, const uint8_t* data, size_t count) {
  return lvkv::cpu_crc32c_extend(crc, data, count);
}

__attribute__((visibility("default"))) uint32_t crc32c_value(
    const uint8_t* data, size_t count) {
  return lvkv::cpu_crc32c_extend(0, data, count);
}

}  // extern "C"
