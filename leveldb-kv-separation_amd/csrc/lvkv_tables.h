// Host-side GF(2) algebra for CRC32C (reflected Castagnoli, 0x82F63B78).
//
// A linear operator on the 32-bit CRC register is stored as its 32 columns
// (col[b] = image of bit b). Z_d = "advance the register over d zero bytes";
// the reference's tables are special cases of it (util/crc32c.cc:20-243:
// byte table = Z_1 on bytes, stride table K = Z_{13+K}).
#ifndef LVKV_TABLES_H_
#define LVKV_TABLES_H_

#include <stddef.h>
#include <stdint.h>

namespace lvkv {

struct Gf2Op {
  uint32_t col[32];
};

Gf2Op gf2_identity();
// Z_d by repeated squaring of Z_1 (O(log d) compositions).
Gf2Op gf2_zero_advance(uint64_t nbytes);
uint32_t gf2_apply(const Gf2Op& op, uint32_t v);
Gf2Op gf2_compose(const Gf2Op& outer, const Gf2Op& inner);  // outer(inner(v))

// Device tables (see lvkv_kernel_args.h for the LDS layout they feed):
//   row_tab[t*256 + i]              = Z_256(i << 8t)          (1024 dwords)
//   lane_tab[(k*16 + nib)*64 + s]   = Z_{256-4s}(nib << 4k)   (8192 dwords)
void build_row_table(uint32_t* row_tab);
void build_lane_table(uint32_t* lane_tab);
//   lane_cols[(k*64 + s)*4 + j]     = Z_{256-4s}(1 << (4k + j)) (2048 dwords):
//   the columns lane s needs to generate its lane-table entries of nibble k
void build_lane_columns(uint32_t* lane_cols);
//   zpow[j*1024 + t*256 + b]        = Z_{2^j}(b << 8t), j < kZPowCount:
//   Z_n(v) for any n = the product over the set bits j of n
void build_zpow_tables(uint32_t* zpow);
//   zmul[((j - kZMulLog0) * kZMulMaxC + c - 1) * 32 + b] = Z_{c * 2^j}(1 << b),
//   c in [1, kZMulMaxC]: the 32 columns of a constant shift, applied with
//   register xors instead of dependent table lookups (group_crc)
void build_zmul_columns(uint32_t* zmul);


}  // namespace lvkv

#endif  // LVKV_TABLES_H_
