// crc32c/crc32c.h — Google-crc32c-compatible C++ header served by
// liblvkv_crc32c.so. Point the reference's include path here and build it
// with HAVE_CRC32C=1: port::AcceleratedCRC32C (port/port_stdcxx.h:208-210)
// then calls ::crc32c::Extend below, and CanAccelerateCRC32C
// (util/crc32c.cc:267-274) routes every leveldb::crc32c::Extend through it.
#ifndef LVKV_CRC32C_GOOGLE_COMPAT_H_
#define LVKV_CRC32C_GOOGLE_COMPAT_H_

#include <cstddef>
#include <cstdint>
#include <cstring>

#include "../lvkv_google_crc32c.h"

namespace crc32c {

// Extend crc (the CRC32C of some string A) to the CRC32C of A||data.
uint32_t Extend(uint32_t crc, const uint8_t* data, size_t count);

inline uint32_t Crc32c(const uint8_t* data, size_t count) {
  return Extend(0, data, count);
}
inline uint32_t Crc32c(const char* data, size_t count) {
  return Extend(0, reinterpret_cast<const uint8_t*>(data), count);
}

}  // namespace crc32c

#endif  // LVKV_CRC32C_GOOGLE_COMPAT_H_
