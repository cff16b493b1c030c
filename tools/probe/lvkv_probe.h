/*
 * lvkv_probe.h — entry points of the probe build of the library
 * (tools/probe/liblvkv_probe.so: the product sources compiled with
 * -DLVKV_PROBE_BUILD, which adds the schedule variants, timestamp builds and
 * the read-bandwidth kernel). Timing and A/B parity only; not shipped.
 */
#ifndef LVKV_PROBE_H_
#define LVKV_PROBE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

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

/* WAL verify kernel phase stamps: 8 u64 (s_memrealtime) per workgroup and
 * iteration (16 iterations kept), slots 0 start, 1 placed, 2 next walked,
 * 3 wave 2's records done, 4 all records, 5 long records, 6 merged. */
void lvkv_debug_log_stamps(uint64_t* d_stamps);
void lvkv_debug_zstd_stamps(uint64_t* d_stamps);  /* 8 s_memtime stamps a zstd frame */
/* 16 s_memtime stamps a block of the zstd compressor: 0 start, 1 staged, 2
 * matched, 8 literals counted, 9 tree built, 10 weights coded, 11 streams
 * sized, 3 literals done, 4 sequence tables, 5 sequence bits, 6 end. */
void lvkv_debug_zstdc_stamps(uint64_t* d_stamps);
void lvkv_debug_asm_stamps(uint64_t* d_stamps);
/* Whole-SSTable verify phase stamps: 16 u64 per table (head slots 0-7; the
 * fused form's first CRC workgroup in table 0's slots 8-10). NULL: off. */
void lvkv_debug_sst_stamps(uint64_t* d_stamps);
/* WAL verify kernel ablations (timing only, results wrong): 1 no record CRCs,
 * 4 no placement look-back. */
void lvkv_debug_log_knobs(uint32_t knobs);

#ifdef __cplusplus
}
#endif

#endif  // LVKV_PROBE_H_
