/*
 * lvkv_crc32c_debug.h — test hooks of liblvkv_crc32c.so (not part of the
 * drop-in surface). Used by tests/test_kernel_model.py to check, on the CPU,
 * the GF(2) tables the gfx950 kernel loads into LDS.
 */
#ifndef LVKV_CRC32C_DEBUG_H_
#define LVKV_CRC32C_DEBUG_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* row_tab[1024]: row_tab[t*256 + i] = Z_256(i << 8t);
 * lane_tab[8192]: lane_tab[(k*16 + nib)*64 + s] = Z_{256-4s}(nib << 4k);
 * Z_d = advance the reflected CRC32C register over d zero bytes.
 * Either pointer may be NULL. */
void lvkv_debug_tables(uint32_t* row_tab, uint32_t* lane_tab);

#ifdef __cplusplus
}
#endif

#endif /* LVKV_CRC32C_DEBUG_H_ */
