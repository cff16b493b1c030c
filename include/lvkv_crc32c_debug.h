/*
 * lvkv_crc32c_debug.h — test hooks of liblvkv_crc32c.so (not part of the
 * drop-in surface). Used by tests/test_kernel_model.py to check, on the CPU,
 * the GF(2) tables the gfx950 kernel loads into LDS.
 */
#ifndef LVKV_CRC32C_DEBUG_H_
#define LVKV_CRC32C_DEBUG_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* row_tab[1024]: row_tab[t*256 + i] = Z_256(i << 8t);
 * lane_tab[8192]: lane_tab[(k*16 + nib)*64 + s] = Z_{256-4s}(nib << 4k);
 * Z_d = advance the reflected CRC32C register over d zero bytes.
 * Either pointer may be NULL. */
void lvkv_debug_tables(uint32_t* row_tab, uint32_t* lane_tab);

/* Timing probes (tools/probe.py). Launch a variant of the batch kernel on the
 * uniform layout: variant bit 1 = no table work, 2 = no global loads, 4 = no
 * LDS fill, 8 = shuffle-based wave reduction, 16 = empty kernel, 32 = the
 * uniform end-aligned specialisation (combines with 1, 2, 4), 64 = record
 * per-wave timestamps (see lvkv_debug_set_stamps), 256 = the dedicated
 * uniform kernel (crc32c_uniform.hip; combines with 64, and 128 = row tables
 * before the loads), 512 (with 256) = its one-round small-batch kernel
 * (with 256|512 and variant >= 1 << 16, bits 16..30 are the small kernel's
 * own schedule flags, crc32c_uniform.hip);
 * 0, 8, 32, 96, 256, 320, 384, 448, 768, 832, 896, 960 compute correct CRCs.
 * groups <= 0 uses one workgroup per CU. Returns an LVKV_* code. */
int lvkv_debug_uniform_variant(int variant, int groups, const void* d_base,
                               uint64_t stride, uint32_t length,
                               uint32_t* d_out, size_t nblocks, void* stream);

/* Timestamp buffer for variant bit 64: 8 u64 per wave (grid waves x 8). */
void lvkv_debug_set_stamps(uint64_t* d_stamps);

/* Read `bytes` (multiple of 16) of device memory once, 16 B per lane, grid
 * stride over `groups` x 256 threads (0: 8 per CU; negative: -groups blocks
 * reading 4 B per lane instead): the measured HBM read ceiling. d_scratch
 * receives at most one u32. */
int lvkv_debug_read_bw(const void* d_data, uint64_t bytes, uint32_t* d_scratch,
                       int groups, void* stream);

/* Engine probes (tools/probe). Each waits for outstanding work first. */
struct lvkv_engine;
/* Kernels of overlapped and of ordered dispatches: 0 = 8 waves x 5 chains,
 * one workgroup per CU per dispatch (overlapped default); 1 = 8 x 3, two
 * workgroups per CU (ordered default). */
int lvkv_engine_set_variant(struct lvkv_engine* engine, int variant, int ordered_variant);
/* Ordered (overlapped = 0) or overlapped dispatches run `kernel` (a
 * UniformArgs kernel of the given shape, symbol name with ".kd") from a
 * separate gfx950 code object in memory (tools/probe/build.sh) instead of the
 * engine's own; NULL restores them. */
int lvkv_engine_load_probe(struct lvkv_engine* engine, const void* code_object, size_t size,
                           const char* kernel, uint32_t waves, uint32_t chains, uint32_t per_cu,
                           int overlapped);
/* Dispatch the timestamp build of the current kernel: dispatch k writes 8 u64
 * per wave (s_memrealtime, 100 MHz; slots 0 start, 1 loads issued, 2 image
 * built, 3 walk done, 4 stored) into area k % areas of d_stamps (areas x
 * groups x waves x 8 u64, lvkv_engine_shape). NULL turns it off. */
int lvkv_engine_set_stamps(struct lvkv_engine* engine, uint64_t* d_stamps, uint64_t areas);

#ifdef __cplusplus
}
#endif

#endif /* LVKV_CRC32C_DEBUG_H_ */
