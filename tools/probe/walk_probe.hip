// WAL header-walk latency probe (not part of the product).
//
// How fast can one wave follow the chain of log record headers of a 32 KiB
// block (db/log_reader.cc:189-271: each header's length locates the next),
// and how does the rate scale when several waves of a CU walk different
// blocks at once? Variants, each timed per wave with s_memtime:
//   0 lds_salu   block in LDS, header dwords read by ds_read2, arithmetic on
//                the scalar unit (readfirstlane) -- the round-2 walk
//   1 lds_valu   block in LDS, address chain in VGPRs, next read issued
//                before the stop test (inline asm) -- the round-3 walk
//   2 glb_salu   block in global memory (L2-warm after a vector sweep),
//                header dwords by s_load_dwordx2, arithmetic on the scalar unit
//   3 glb_vmem   block in global memory (L2-warm), header dwords by a
//                uniform global_load_dwordx2
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe/walk_probe.hip -o build/walk_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

constexpr uint32_t kBlock = 32768;
constexpr uint32_t kHdr = 7;
constexpr int kThreads = 1024;

struct Out {
  unsigned long long cycles, headers;
};

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// variant 0: round-2 form
__device__ uint32_t walk_lds_salu(const uint8_t* blk, uint32_t n) {
  uint32_t p = 0, k = 0;
  while (n - p >= kHdr) {
    const uint32_t x = p + 4;
    const uint32_t* d = reinterpret_cast<const uint32_t*>(blk + (x & ~3u));
    const uint32_t lo = __builtin_amdgcn_readfirstlane(d[0]);
    const uint32_t hi = __builtin_amdgcn_readfirstlane(d[1]);
    const uint32_t w = static_cast<uint32_t>(((static_cast<uint64_t>(hi) << 32) | lo) >> (8u * (x & 3u)));
    const uint32_t length = w & 0xffffu;
    if (kHdr + length > n - p) break;
    if ((w & 0xffffffu) == 0) break;
    ++k;
    p += kHdr + length;
  }
  return k;
}

// variant 1: round-3 form
__device__ uint32_t walk_lds_valu(const uint8_t* blk, uint32_t n) {
  uint32_t p = 0, k = 0;
  if (n < kHdr) return 0;
  const uint32_t base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(blk));
  uint64_t cur, nxt;
  uint32_t bp = base;
  asm volatile("ds_read2_b32 %0, %1 offset0:1 offset1:2" : "=v"(cur) : "v"(base));
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(cur));
  for (;;) {
    const uint32_t w = __builtin_amdgcn_alignbyte(static_cast<uint32_t>(cur >> 32),
                                                  static_cast<uint32_t>(cur), bp & 3u);
    const uint32_t length = w & 0xffffu;
    const uint32_t nbp = bp + kHdr + length;
    asm volatile("ds_read2_b32 %0, %1 offset0:1 offset1:2" : "=v"(nxt) : "v"(nbp & ~3u));
    const uint32_t np = p + kHdr + length;
    __builtin_amdgcn_sched_barrier(0);
    const bool bad = np > n || (w & 0xffffffu) == 0;
    const uint32_t f = __builtin_amdgcn_readfirstlane((bad ? 1u : 0u) | (n - np < kHdr ? 2u : 0u));
    if (f & 1u) break;
    ++k;
    p = np;
    bp = nbp;
    if (f & 2u) break;
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(nxt));
    cur = nxt;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(nxt));
  return k;
}

// variant 4: unaligned ds_read_u16 of the length (+ ds_read_u8 of the type),
// the next header's reads issued before this header's stop test
__device__ uint32_t walk_lds_u16(const uint8_t* blk, uint32_t n) {
  uint32_t k = 0;
  if (n < kHdr) return 0;
  const uint32_t base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(blk));
  const uint32_t end = base + n;
  uint32_t bp = base, len, typ, nlen, ntyp;
  asm volatile("ds_read_u16 %0, %2 offset:4\n\tds_read_u8 %1, %2 offset:6\n\ts_waitcnt lgkmcnt(0)"
               : "=v"(len), "=v"(typ) : "v"(bp));
  for (;;) {
    const uint32_t nbp = bp + kHdr + len;
    asm volatile("ds_read_u16 %0, %2 offset:4\n\tds_read_u8 %1, %2 offset:6"
                 : "=v"(nlen), "=v"(ntyp) : "v"(nbp));
    __builtin_amdgcn_sched_barrier(0);
    const bool bad = nbp > end || (len | typ) == 0;
    if (__builtin_amdgcn_ballot_w64(bad)) break;
    ++k;
    bp = nbp;
    if (__builtin_amdgcn_ballot_w64(end - bp < kHdr)) break;
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(nlen), "+v"(ntyp));
    len = nlen;
    typ = ntyp;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(nlen), "+v"(ntyp));
  return k;
}


// variant 5: the block read from an 8 KiB register window (uniform register
// index + v_readlane), the chain on the scalar unit -- the round-3 walk
typedef uint32_t WinRows __attribute__((ext_vector_type(32)));
__device__ uint32_t walk_regs(const uint8_t* blk, uint32_t n) {
  const uint32_t lane = lane_id();
  const uint32_t* sw = reinterpret_cast<const uint32_t*>(blk);
  uint32_t k = 0, p = 0;
  if (n < kHdr) return 0;
  WinRows win;
  uint32_t wbase = 0;
#pragma unroll
  for (uint32_t r = 0; r < 32; ++r) win[r] = sw[64u * r + lane];
  for (;;) {
    const uint32_t a = __builtin_amdgcn_readfirstlane(p + 4u);
    const uint32_t d = a >> 2;
    if (d + 1u >= wbase + 2048u) {
      wbase = d & ~63u;
#pragma unroll
      for (uint32_t r = 0; r < 32; ++r) win[r] = sw[wbase + 64u * r + lane];
    }
    const uint32_t rel = d - wbase;
    const uint32_t r = rel >> 6, l = rel & 63u;
    const uint32_t lo = __builtin_amdgcn_readlane(win[r], l);
    const uint32_t hi = l == 63u ? __builtin_amdgcn_readlane(win[min(r + 1u, 31u)], 0)
                                 : __builtin_amdgcn_readlane(win[r], l + 1u);
    const uint32_t w = static_cast<uint32_t>(((static_cast<uint64_t>(hi) << 32) | lo) >> (8u * (a & 3u)));
    const uint32_t len = w & 0xffffu;
    const uint32_t np = p + kHdr + len;
    if (np > n || (w & 0xffffffu) == 0) break;
    ++k;
    p = np;
    if (n - p < kHdr) break;
  }
  return k;
}

// variant 2: scalar loads from global memory
__device__ uint32_t walk_glb_salu(const uint8_t* blk, uint32_t n) {
  uint32_t p = 0, k = 0;
  while (n - p >= kHdr) {
    const uint32_t x = p + 4;
    uint64_t v;
    asm volatile("s_load_dwordx2 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)"
                 : "=s"(v)
                 : "s"(blk), "s"(x & ~3u));
    const uint32_t w = static_cast<uint32_t>(v >> (8u * (x & 3u)));
    const uint32_t length = w & 0xffffu;
    if (kHdr + length > n - p) break;
    if ((w & 0xffffffu) == 0) break;
    ++k;
    p += kHdr + length;
  }
  return k;
}

// variant 3: uniform vector loads from global memory
__device__ uint32_t walk_glb_vmem(const uint8_t* blk, uint32_t n) {
  uint32_t p = 0, k = 0;
  while (n - p >= kHdr) {
    const uint32_t x = p + 4;
    const uint2 d = *reinterpret_cast<const uint2*>(blk + (x & ~3u) - ((x & 4u) ? 0u : 0u));
    const uint32_t lo = __builtin_amdgcn_readfirstlane(d.x);
    const uint32_t hi = __builtin_amdgcn_readfirstlane(d.y);
    const uint32_t w = static_cast<uint32_t>(((static_cast<uint64_t>(hi) << 32) | lo) >> (8u * (x & 3u)));
    const uint32_t length = w & 0xffffu;
    if (kHdr + length > n - p) break;
    if ((w & 0xffffffu) == 0) break;
    ++k;
    p += kHdr + length;
  }
  return k;
}

// One workgroup per CU; waves [0, walkers) each walk blocks
// blockIdx.x * walkers + wave + j * gridDim.x * walkers.
template <int V>
__global__ void __launch_bounds__(kThreads, 1)
    walk_kernel(const uint8_t* __restrict__ img, uint32_t nblk, uint32_t walkers, Out* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4][kBlock + 16];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = lane_id();
  if (wave >= walkers) return;
  unsigned long long cyc = 0, hdrs = 0;
  for (uint32_t b = blockIdx.x * walkers + wave; b < nblk; b += gridDim.x * walkers) {
    const uint8_t* src = img + static_cast<uint64_t>(b) * kBlock;
    uint8_t* mine = lds[wave & 3];
    // stage: the block into this wave's LDS area (LDS variants) or just
    // through L2 (global variants)
    uint32_t acc = 0;
    for (uint32_t o = lane * 16; o < kBlock; o += 64 * 16) {
      const uint4 v = *reinterpret_cast<const uint4*>(src + o);
      if (V <= 1 || V >= 4) *reinterpret_cast<uint4*>(mine + o) = v;
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    if (acc == 0x9e3779b9u) out[1023].headers = acc;  // keep the sweep
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    uint32_t k;
    if (V == 0) k = walk_lds_salu(mine, kBlock);
    else if (V == 1) k = walk_lds_valu(mine, kBlock);
    else if (V == 2) k = walk_glb_salu(src, kBlock);
    else if (V == 4) k = walk_lds_u16(mine, kBlock);
    else if (V == 5) k = walk_regs(mine, kBlock);
    else k = walk_glb_vmem(src, kBlock);
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    cyc += c1 - c0;
    hdrs += k;
  }
  if (lane == 0) {
    out[blockIdx.x * 16 + wave].cycles = cyc;
    out[blockIdx.x * 16 + wave].headers = hdrs;
  }
}

static void put_header(std::vector<uint8_t>& img, size_t at, uint32_t len) {
  img[at + 4] = len & 0xff;
  img[at + 5] = (len >> 8) & 0xff;
  img[at + 6] = 1;  // kFullType
  img[at + 0] = 0x5a;
}

int main(int argc, char** argv) {
  const uint32_t nblk = argc > 1 ? atoi(argv[1]) : 2048;
  std::vector<uint8_t> img(static_cast<size_t>(nblk) * kBlock, 0);
  uint64_t s = 0x9e3779b97f4a7c15ull;
  auto rnd = [&]() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  };
  for (uint32_t b = 0; b < nblk; ++b) {
    uint32_t p = 0;
    while (kBlock - p >= kHdr) {
      uint32_t len = static_cast<uint32_t>(rnd() % 2001);
      len = std::min(len, kBlock - p - kHdr);
      put_header(img, static_cast<size_t>(b) * kBlock + p, len);
      for (uint32_t i = 0; i < len; ++i) img[static_cast<size_t>(b) * kBlock + p + kHdr + i] = rnd() | 1;
      p += kHdr + len;
    }
  }
  uint8_t* d_img;
  Out* d_out;
  hipMalloc(&d_img, img.size());
  hipMemcpy(d_img, img.data(), img.size(), hipMemcpyHostToDevice);
  hipMalloc(&d_out, sizeof(Out) * 256 * 16 + 16);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const char* names[] = {"lds_salu", "lds_valu", "glb_salu", "glb_vmem", "lds_u16", "regs"};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int v : {4, 2, 3}) {
    for (uint32_t walkers : {1u, 2u, 4u, 8u}) {
      float best = 1e9f;
      std::vector<Out> h(256 * 16);
      for (int rep = 0; rep < 3; ++rep) {
        hipMemset(d_out, 0, sizeof(Out) * 256 * 16);
        hipEventRecord(e0);
        switch (v) {
          case 0: hipLaunchKernelGGL(walk_kernel<0>, dim3(cus), dim3(kThreads), 0, 0, d_img, nblk, walkers, d_out); break;
          case 1: hipLaunchKernelGGL(walk_kernel<1>, dim3(cus), dim3(kThreads), 0, 0, d_img, nblk, walkers, d_out); break;
          case 2: hipLaunchKernelGGL(walk_kernel<2>, dim3(cus), dim3(kThreads), 0, 0, d_img, nblk, walkers, d_out); break;
          case 3: hipLaunchKernelGGL(walk_kernel<3>, dim3(cus), dim3(kThreads), 0, 0, d_img, nblk, walkers, d_out); break;
          case 5: hipLaunchKernelGGL(walk_kernel<5>, dim3(cus), dim3(kThreads), 0, 0, d_img, nblk, walkers, d_out); break;
          default: hipLaunchKernelGGL(walk_kernel<4>, dim3(cus), dim3(kThreads), 0, 0, d_img, nblk, walkers, d_out); break;
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        best = std::min(best, ms);
        hipMemcpy(h.data(), d_out, sizeof(Out) * 256 * 16, hipMemcpyDeviceToHost);
      }
      unsigned long long c = 0, k = 0;
      for (auto& o : h) {
        c += o.cycles;
        k += o.headers;
      }
      printf("%-9s walkers/CU %2u: %.1f ticks/header (%llu headers), kernel %.1f us for %u blocks, "
             "%.1f ns/header/walker\n",
             names[v], walkers, k ? double(c) / double(k) : 0.0, k, best * 1e3, nblk,
             best * 1e6 / (double(k) / (cus * walkers)));
    }
  }
  return 0;
}
