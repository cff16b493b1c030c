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

/* The portable slicing-by-8 per-call path (lvkv_cpu_crc32c.cpp), whatever
 * implementation the per-call entry points picked on this CPU. */
uint32_t lvkv_debug_extend_portable(uint32_t crc, const uint8_t* data, size_t n);

/* Kernel choices of the current device (per device, not process globals;
 * timing and A/B tests): general-layout batches (-1 crc32c_kernel.hip's
 * persistent kernel, 0..31 ragged cfgs), WAL records (ragged cfg), and the
 * whole-SSTable verify form (0 by size, 1 one fused launch, 2 two launches). */
int lvkv_debug_set_general_kernel(int cfg);
int lvkv_debug_set_log_kernel(int cfg);
int lvkv_debug_set_sst_form(int form);

/* lvkv_zstd_uncompress_device with the failure site of each stream
 * (d_detail[i]: 0 none, else the decoder's check that failed; tests). */
int lvkv_debug_zstd_uncompress_device(const void* d_src, const uint64_t* d_src_off,
                                      const uint32_t* d_src_len, void* d_dst,
                                      const uint64_t* d_dst_off, const uint32_t* d_dst_cap,
                                      uint32_t* d_out_len, uint8_t* d_status, uint32_t* d_detail,
                                      size_t nblocks, uint32_t max_ulen, void* stream);

/* The kernel-variant, timestamp and read-bandwidth probes live in the probe
 * build of the library (tools/probe/liblvkv_probe.so, tools/probe/lvkv_probe.h),
 * not in liblvkv_crc32c.so. */

/* Engine probes (tools/probe). Each waits for outstanding work first. */
struct lvkv_engine;
/* Kernels of overlapped and of ordered dispatches: 0 = 8 waves x 5 chains,
 * one workgroup per CU per dispatch (overlapped default); 1 = 8 x 3, two
 * workgroups per CU (ordered default). */
int lvkv_engine_set_variant(struct lvkv_engine* engine, int variant, int ordered_variant);
/* Kernel of LVKV_FLAG_FINAL uniform dispatches (the last before a wait):
 * -1 = as the overlapped ones (default), 0 or 1 as above. */
int lvkv_engine_set_final_variant(struct lvkv_engine* engine, int variant);
/* Ordered (overlapped = 0) or overlapped dispatches run `kernel` (a
 * UniformArgs kernel of the given shape, symbol name with ".kd") from a
 * separate gfx950 code object in memory (tools/probe/build.sh) instead of the
 * engine's own; NULL restores them. */
int lvkv_engine_load_probe(struct lvkv_engine* engine, const void* code_object, size_t size,
                           const char* kernel, uint32_t waves, uint32_t chains, uint32_t per_cu,
                           int overlapped);
/* Memory-fence scopes (0 none, 1 agent, 2 system) of a submission's first
 * dispatch (acquire; default agent) and of the wait's barrier packets
 * (acquire, release; default none, system). Timing probes only. */
int lvkv_engine_set_scopes(struct lvkv_engine* engine, int dispatch_acquire, int fence_acquire,
                           int fence_release);
/* Hardware queue priority of the engine's queues (0 low, 1 normal, 2 high). */
int lvkv_engine_set_priority(struct lvkv_engine* engine, int priority);
/* Dispatch the timestamp build of the current kernel: dispatch k writes 8 u64
 * per wave (s_memrealtime, 100 MHz; slots 0 start, 1 loads issued, 2 image
 * built, 3 walk done, 4 stored) into area k % areas of d_stamps (areas x
 * groups x waves x 8 u64, lvkv_engine_shape). NULL turns it off. */
int lvkv_engine_set_stamps(struct lvkv_engine* engine, uint64_t* d_stamps, uint64_t areas);

/* The no-hang contract under test: stall = 1 blocks every queue of the
 * engine behind a barrier packet that waits on a signal only stall = 0
 * releases (as a faulted or endless dispatch would); every engine wait gives
 * up after stuck_seconds without progress (default 60) and returns
 * LVKV_ERR_HIP, after which the engine refuses work. */
int lvkv_debug_engine_stall(struct lvkv_engine* engine, int stall, double stuck_seconds);
/* The engine's general-layout kernel for every later submit (A/B timing,
 * tools/probe/engine_shapes.py): 2 = persistent 8 x 2 x 24, 3 = persistent
 * 8 x 4 x 8, 4 = one-round 8 x 4 x 17, 5 = one-round 8 x 6 x 8; -1 = chosen by
 * the batch's layout (the default). */
int lvkv_debug_engine_ragged_spec(struct lvkv_engine* engine, int spec);
/* The engine's kernel-argument cache: dispatches whose arguments an earlier
 * dispatch's cached VRAM copy already held (no BAR write, no HDP flush), and
 * those written afresh. */
int lvkv_debug_engine_kernarg_cache(struct lvkv_engine* engine, uint64_t* hits,
                                    uint64_t* misses);

#ifdef __cplusplus
}
#endif

#endif /* LVKV_CRC32C_DEBUG_H_ */
