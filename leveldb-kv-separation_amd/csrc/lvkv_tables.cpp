#include "lvkv_tables.h"

#include "lvkv_kernel_args.h"

namespace lvkv {

Gf2Op gf2_identity() {
  Gf2Op op;
  for (int b = 0; b < 32; ++b) op.col[b] = 1u << b;
  return op;
}

uint32_t gf2_apply(const Gf2Op& op, uint32_t v) {
  uint32_t r = 0;
  for (int b = 0; v != 0; ++b, v >>= 1)
    if (v & 1u) r ^= op.col[b];
  return r;
}

Gf2Op gf2_compose(const Gf2Op& outer, const Gf2Op& inner) {
  Gf2Op r;
  for (int b = 0; b < 32; ++b) r.col[b] = gf2_apply(outer, inner.col[b]);
  return r;
}

namespace {

// One zero bit through the reflected register.
uint32_t zero_bit(uint32_t reg) {
  return (reg >> 1) ^ (kCastagnoliReflected & (0u - (reg & 1u)));
}

Gf2Op zero_byte_op() {
  Gf2Op op;
  for (int b = 0; b < 32; ++b) {
    uint32_t v = 1u << b;
    for (int k = 0; k < 8; ++k) v = zero_bit(v);
    op.col[b] = v;
  }
  return op;
}

}  // namespace

Gf2Op gf2_zero_advance(uint64_t nbytes) {
  Gf2Op result = gf2_identity();
  Gf2Op power = zero_byte_op();
  while (nbytes != 0) {
    if (nbytes & 1u) result = gf2_compose(power, result);
    power = gf2_compose(power, power);
    nbytes >>= 1;
  }
  return result;
}

void build_row_table(uint32_t* row_tab) {
  const Gf2Op z = gf2_zero_advance(kRowBytes);
  for (uint32_t t = 0; t < 4; ++t)
    for (uint32_t i = 0; i < 256; ++i)
      row_tab[t * 256 + i] = gf2_apply(z, i << (8 * t));
}

void build_lane_table(uint32_t* lane_tab) {
  for (uint32_t s = 0; s < 64; ++s) {
    const Gf2Op z = gf2_zero_advance(kRowBytes - 4 * s);
    for (uint32_t k = 0; k < 8; ++k)
      for (uint32_t nib = 0; nib < 16; ++nib)
        lane_tab[(k * 16 + nib) * 64 + s] = gf2_apply(z, nib << (4 * k));
  }
}

void build_lane_columns(uint32_t* lane_cols) {
  for (uint32_t s = 0; s < 64; ++s) {
    const Gf2Op z = gf2_zero_advance(kRowBytes - 4 * s);
    for (uint32_t k = 0; k < 8; ++k)
      for (uint32_t j = 0; j < 4; ++j) lane_cols[(k * 64 + s) * 4 + j] = z.col[4 * k + j];
  }
}

void build_zpow_tables(uint32_t* zpow) {
  for (uint32_t j = 0; j < kZPowCount; ++j) {
    const Gf2Op z = gf2_zero_advance(uint64_t{1} << j);
    for (uint32_t t = 0; t < 4; ++t)
      for (uint32_t b = 0; b < 256; ++b) zpow[j * 1024 + t * 256 + b] = gf2_apply(z, b << (8 * t));
  }
}

void build_zmul_columns(uint32_t* zmul) {
  for (uint32_t j = kZMulLog0; j < kZMulLog0 + kZMulLogs; ++j) {
    const Gf2Op z = gf2_zero_advance(uint64_t{1} << j);
    Gf2Op m = z;
    for (uint32_t c = 1; c <= kZMulMaxC; ++c) {
      for (uint32_t b = 0; b < 32; ++b)
        zmul[((j - kZMulLog0) * kZMulMaxC + c - 1) * 32 + b] = m.col[b];
      m = gf2_compose(z, m);
    }
  }
}

}  // namespace lvkv

extern "C" __attribute__((visibility("default"))) void lvkv_debug_tables(
    uint32_t* row_tab, uint32_t* lane_tab) {
  if (row_tab != nullptr) lvkv::build_row_table(row_tab);
  if (lane_tab != nullptr) lvkv::build_lane_table(lane_tab);
}
