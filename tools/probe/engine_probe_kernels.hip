// Probe kernels for the AQL engine (tools/probe/iso_probe.py): schedule and
// shape variants of the uniform kernel, loaded at run time from their own
// code object (lvkv_engine_load_probe) and timed as ordered dispatches.
// Not part of the product.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_burst.h"
#include "lvkv_kernel_args.h"

namespace {
constexpr int kLds = lvkv::kCompactLdsBytes / 4;
}

#define PROBE(NAME, F, W, NCH, OCC)                                       \
  extern "C" __global__ void __launch_bounds__(64 * W, OCC)               \
      NAME(lvkv::UniformArgs a) {                                         \
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLds];           \
    lvkv::burst_kernel_body<F, W, NCH>(a, lds, a.ngroups);                \
  }

using namespace lvkv;
PROBE(pk_pair, 0, 8, 3, 2)
PROBE(pk_pair_bare, kBurstBare, 8, 3, 2)
PROBE(pk_pair_nobuild, kBurstNoBuild, 8, 3, 2)
PROBE(pk_pair_nowalk, kBurstNoWalk, 8, 3, 2)
PROBE(pk_pair_late, kBurstLate, 8, 3, 2)
PROBE(pk_pair_split2, kBurstSplit2, 8, 3, 2)
PROBE(pk_pair_dp, kBurstDefaultPolicy, 8, 3, 2)
PROBE(pk_pair_bare_dp, kBurstBare | kBurstDefaultPolicy, 8, 3, 2)
PROBE(pk_pair_pipe1, kBurstPipe1, 8, 3, 2)
PROBE(pk_pair_pipe2, kBurstPipe2, 8, 3, 2)
PROBE(pk_one_pipe1, kBurstPipe1, 8, 5, 1)
PROBE(pk_one_pipe2, kBurstPipe2, 8, 5, 1)
PROBE(pk_w16_pipe1, kBurstPipe1, 16, 3, 1)
PROBE(pk_pair_pipe1_st, kBurstPipe1 | kBurstStamps, 8, 3, 2)
PROBE(pk_pair_bare_st, kBurstBare | kBurstStamps, 8, 3, 2)
PROBE(pk_pair_st, kBurstStamps, 8, 3, 2)
PROBE(pk_pair_pipe1_s2, kBurstPipe1 | kBurstSplit2, 8, 3, 2)
PROBE(pk_pair_pipe1_s4, kBurstPipe1 | kBurstSplit4, 8, 3, 2)
PROBE(pk_pair_pipe2_s2, kBurstPipe2 | kBurstSplit2, 8, 3, 2)
PROBE(pk_one_pipe2_s2, kBurstPipe2 | kBurstSplit2, 8, 5, 1)
PROBE(pk_w16, 0, 16, 3, 1)
PROBE(pk_w16_bare, kBurstBare, 16, 3, 1)
PROBE(pk_one, 0, 8, 5, 1)
PROBE(pk_one_bare, kBurstBare, 8, 5, 1)
PROBE(pk_w10c2_pipe1, kBurstPipe1, 10, 2, 2)
PROBE(pk_w10c2, 0, 10, 2, 2)
PROBE(pk_w12c2_pipe1, kBurstPipe1, 12, 2, 2)
PROBE(pk_w10c2_pipe1_s2, kBurstPipe1 | kBurstSplit2, 10, 2, 2)
