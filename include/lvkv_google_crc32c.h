/*
 * lvkv_google_crc32c.h — the Google crc32c library C ABI, served by
 * liblvkv_crc32c.so so that the reference's own accelerator hook can bind to
 * it unchanged.
 *
 * Reference hook: port::AcceleratedCRC32C (port/port_stdcxx.h:208-218) calls
 * ::crc32c::Extend(crc, (const uint8_t*)buf, size) when HAVE_CRC32C is set;
 * CMake sets HAVE_CRC32C when check_library_exists(crc32c crc32c_value) finds
 * the C symbol below (CMakeLists.txt:41, 281-283). The same library also
 * exports the C++ ::crc32c::Extend / ::crc32c::Crc32c overloads. The
 * self-test CanAccelerateCRC32C (util/crc32c.cc:267-274) passes against it.
 */
#ifndef LVKV_GOOGLE_CRC32C_H_
#define LVKV_GOOGLE_CRC32C_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

uint32_t crc32c_extend(uint32_t crc, const uint8_t* data, size_t count);
uint32_t crc32c_value(const uint8_t* data, size_t count);

#ifdef __cplusplus
}
#endif

#endif /* LVKV_GOOGLE_CRC32C_H_ */
