/*
 * TEST INFRASTRUCTURE ONLY — the CPU oracle for the batched CRC32C engine.
 *
 * This is a from-scratch C restatement of the reference's portable CRC32C
 * (/root/reference/util/crc32c.cc:276-377, header util/crc32c.h:17-38). It is
 * the checker that tests/, __graft_entry__.smoke() and bench.py's
 * `cpu_baseline` leg compare the HIP path against. Nothing in the product
 * library (leveldb-kv-separation_amd/) links or calls it.
 *
 * Parity pin: tests/test_oracle.py checks every function here against
 *   - the RFC 3720 known-answer vectors of util/crc32c_test.cc:12-53,
 *   - the CanAccelerateCRC32C self-test value (util/crc32c.cc:267-274),
 *   - zlib-crc32 fingerprints of the reference's literal tables
 *     (SURVEY.md §8(a) row a4), and
 *   - golden vectors written by oracle/_ref (the reference's own
 *     util/crc32c.cc compiled in place by oracle/Makefile) into tests/golden/.
 */
#ifndef LVKV_ORACLE_CRC32C_ORACLE_H_
#define LVKV_ORACLE_CRC32C_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* leveldb::crc32c::Extend (util/crc32c.cc:276). */
uint32_t oracle_crc32c_extend(uint32_t crc, const uint8_t* data, size_t n);
/* leveldb::crc32c::Value (util/crc32c.h:20). */
uint32_t oracle_crc32c_value(const uint8_t* data, size_t n);
/* leveldb::crc32c::Mask / Unmask (util/crc32c.h:29-38). */
uint32_t oracle_crc32c_mask(uint32_t crc);
uint32_t oracle_crc32c_unmask(uint32_t masked);

/* Copy one of the five generated tables (0 = byte table, 1..4 = stride
 * tables 0..3) into out[256]; used to check fingerprints. Returns 0 on
 * success. */
int oracle_crc32c_table(int which, uint32_t* out);

/* Batch helper: out[i] = Extend(init ? init[i] : 0, base + off[i], len[i]),
 * optionally Mask()ed. Single-threaded loop over the blocks. */
void oracle_crc32c_batch(const uint8_t* base, const uint64_t* offsets,
                         const uint32_t* lengths, const uint32_t* init,
                         uint32_t* out, size_t nblocks, int mask);

/* Same loop split over `threads` POSIX threads (static contiguous partition,
 * SURVEY.md §8(d) CPU-baseline plan). */
void oracle_crc32c_batch_mt(const uint8_t* base, const uint64_t* offsets,
                            const uint32_t* lengths, const uint32_t* init,
                            uint32_t* out, size_t nblocks, int mask,
                            int threads);

/* Uniform-stride batch: block i = base + i*stride, `length` bytes. */
void oracle_crc32c_uniform(const uint8_t* base, uint64_t stride,
                           uint32_t length, uint32_t init, uint32_t* out,
                           size_t nblocks, int mask, int threads);

#ifdef __cplusplus
}
#endif

#endif /* LVKV_ORACLE_CRC32C_ORACLE_H_ */
