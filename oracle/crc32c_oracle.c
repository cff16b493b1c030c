/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle (see crc32c_oracle.h for the contract
 * and how it is pinned). Restates the algorithm of the reference's portable
 * CRC32C, /root/reference/util/crc32c.cc:276-377, in plain C:
 *
 *   state  l = crc ^ 0xffffffff                        (crc32c.cc:284)
 *   1. byte steps until the pointer is 4-byte aligned  (crc32c.cc:322-331)
 *   2. if >= 16 bytes remain: seed four interleaved 4-byte streams from one
 *      16-byte swath, the first xored with l            (crc32c.cc:333-338)
 *   3. swath loop: each stream advances 16 bytes       (crc32c.cc:345-347)
 *   4. word loop rotating the streams                  (crc32c.cc:350-358)
 *   5. fold the four streams back through the byte table (STEP4W,
 *      crc32c.cc:300-309, 361-365)
 *   6. byte tail                                       (crc32c.cc:369-371)
 *   return l ^ 0xffffffff                               (crc32c.cc:376)
 *
 * The five 256-entry tables are GENERATED here (the reference ships them as
 * literals, crc32c.cc:20-243): the byte table is one byte of register advance,
 * stride table K advances 13+K zero bytes. Their
 * fingerprints are checked in tests/test_oracle.py.
 */
#include "crc32c_oracle.h"

#include <pthread.h>
#include <string.h>

#define ORACLE_POLY 0x82f63b78u /* reflected Castagnoli polynomial */

static uint32_t g_byte_tab[256];
static uint32_t g_stride_tab[4][256]; /* [K] advances 13+K zero bytes */
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

/* Run the reflected register over `nbytes` zero bytes. */
static uint32_t zero_advance(uint32_t reg, int nbytes) {
  for (int bit = 0; bit < 8 * nbytes; ++bit) {
    reg = (reg >> 1) ^ (ORACLE_POLY & (0u - (reg & 1u)));
  }
  return reg;
}

static void build_tables(void) {
  for (uint32_t v = 0; v < 256; ++v) {
    g_byte_tab[v] = zero_advance(v, 1);
    for (int k = 0; k < 4; ++k) g_stride_tab[k][v] = zero_advance(v, 13 + k);
  }
}

static inline void ensure_tables(void) { pthread_once(&g_once, build_tables); }

/* Little-endian 32-bit load (util/coding.h:82-90 via crc32c.cc:249-251). */
static inline uint32_t load_le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
         ((uint32_t)p[3] << 24);
}

static inline uint32_t byte_step(uint32_t reg, uint8_t b) {
  return g_byte_tab[(reg ^ b) & 0xffu] ^ (reg >> 8);
}

/* One stream advancing by a full 16-byte swath and absorbing the next word
 * of that stream (the reference's STEP4). */
static inline uint32_t stride_step(uint32_t s, const uint8_t* next_word) {
  return load_le32(next_word) ^ g_stride_tab[3][s & 0xffu] ^
         g_stride_tab[2][(s >> 8) & 0xffu] ^
         g_stride_tab[1][(s >> 16) & 0xffu] ^ g_stride_tab[0][s >> 24];
}

/* Feed a finished stream value through four byte steps (STEP4W). */
static inline uint32_t fold_stream(uint32_t reg, uint32_t stream) {
  uint32_t w = stream ^ reg;
  for (int i = 0; i < 4; ++i) w = (w >> 8) ^ g_byte_tab[w & 0xffu];
  return w;
}

uint32_t oracle_crc32c_extend(uint32_t crc, const uint8_t* data, size_t n) {
  ensure_tables();
  const uint8_t* p = data;
  const uint8_t* end = data + n;
  uint32_t reg = crc ^ 0xffffffffu;

  /* 1. head: walk to 4-byte alignment, but only if that point is in range. */
  const uint8_t* aligned =
      (const uint8_t*)(((uintptr_t)p + 3u) & ~(uintptr_t)3u);
  if (aligned <= end) {
    while (p != aligned) reg = byte_step(reg, *p++);
  }

  if (end - p >= 16) {
    /* 2. seed four streams */
    uint32_t s0 = load_le32(p) ^ reg;
    uint32_t s1 = load_le32(p + 4);
    uint32_t s2 = load_le32(p + 8);
    uint32_t s3 = load_le32(p + 12);
    p += 16;
    /* 3. whole swaths */
    while (end - p >= 16) {
      s0 = stride_step(s0, p);
      s1 = stride_step(s1, p + 4);
      s2 = stride_step(s2, p + 8);
      s3 = stride_step(s3, p + 12);
      p += 16;
    }
    /* 4. remaining whole words: advance the lead stream, rotate */
    while (end - p >= 4) {
      uint32_t lead = stride_step(s0, p);
      s0 = s1;
      s1 = s2;
      s2 = s3;
      s3 = lead;
      p += 4;
    }
    /* 5. fold the streams in order */
    reg = 0;
    reg = fold_stream(reg, s0);
    reg = fold_stream(reg, s1);
    reg = fold_stream(reg, s2);
    reg = fold_stream(reg, s3);
  }

  /* 6. tail bytes */
  while (p != end) reg = byte_step(reg, *p++);
  return reg ^ 0xffffffffu;
}

uint32_t oracle_crc32c_value(const uint8_t* data, size_t n) {
  return oracle_crc32c_extend(0, data, n);
}

#define ORACLE_MASK_DELTA 0xa282ead8u /* util/crc32c.h:22 */

uint32_t oracle_crc32c_mask(uint32_t crc) {
  return ((crc >> 15) | (crc << 17)) + ORACLE_MASK_DELTA;
}

uint32_t oracle_crc32c_unmask(uint32_t masked) {
  uint32_t r = masked - ORACLE_MASK_DELTA;
  return (r >> 17) | (r << 15);
}

int oracle_crc32c_table(int which, uint32_t* out) {
  ensure_tables();
  if (which == 0) {
    memcpy(out, g_byte_tab, sizeof(g_byte_tab));
    return 0;
  }
  if (which >= 1 && which <= 4) {
    memcpy(out, g_stride_tab[which - 1], sizeof(g_stride_tab[0]));
    return 0;
  }
  return -1;
}

void oracle_crc32c_batch(const uint8_t* base, const uint64_t* offsets,
                         const uint32_t* lengths, const uint32_t* init,
                         uint32_t* out, size_t nblocks, int mask) {
  for (size_t i = 0; i < nblocks; ++i) {
    uint32_t c = oracle_crc32c_extend(init ? init[i] : 0u, base + offsets[i],
                                      lengths[i]);
    out[i] = mask ? oracle_crc32c_mask(c) : c;
  }
}

typedef struct {
  const uint8_t* base;
  const uint64_t* offsets;
  const uint32_t* lengths;
  const uint32_t* init;
  uint32_t* out;
  size_t begin, end;
  int mask;
  uint64_t stride; /* uniform mode when offsets == NULL */
  uint32_t ulen, uinit;
} oracle_job;

static void* oracle_worker(void* arg) {
  oracle_job* j = (oracle_job*)arg;
  for (size_t i = j->begin; i < j->end; ++i) {
    uint32_t c;
    if (j->offsets) {
      c = oracle_crc32c_extend(j->init ? j->init[i] : 0u,
                               j->base + j->offsets[i], j->lengths[i]);
    } else {
      c = oracle_crc32c_extend(j->uinit, j->base + i * j->stride, j->ulen);
    }
    j->out[i] = j->mask ? oracle_crc32c_mask(c) : c;
  }
  return NULL;
}

static void run_jobs(oracle_job proto, size_t nblocks, int threads) {
  ensure_tables();
  if (threads < 1) threads = 1;
  if ((size_t)threads > nblocks) threads = nblocks ? (int)nblocks : 1;
  pthread_t tid[256];
  oracle_job jobs[256];
  if (threads > 256) threads = 256;
  size_t per = nblocks / (size_t)threads, extra = nblocks % (size_t)threads;
  size_t at = 0;
  for (int t = 0; t < threads; ++t) {
    jobs[t] = proto;
    jobs[t].begin = at;
    at += per + ((size_t)t < extra ? 1 : 0);
    jobs[t].end = at;
  }
  if (threads == 1) {
    oracle_worker(&jobs[0]);
    return;
  }
  for (int t = 0; t < threads; ++t)
    pthread_create(&tid[t], NULL, oracle_worker, &jobs[t]);
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
}

void oracle_crc32c_batch_mt(const uint8_t* base, const uint64_t* offsets,
                            const uint32_t* lengths, const uint32_t* init,
                            uint32_t* out, size_t nblocks, int mask,
                            int threads) {
  oracle_job p;
  memset(&p, 0, sizeof(p));
  p.base = base;
  p.offsets = offsets;
  p.lengths = lengths;
  p.init = init;
  p.out = out;
  p.mask = mask;
  run_jobs(p, nblocks, threads);
}

void oracle_crc32c_uniform(const uint8_t* base, uint64_t stride,
                           uint32_t length, uint32_t init, uint32_t* out,
                           size_t nblocks, int mask, int threads) {
  oracle_job p;
  memset(&p, 0, sizeof(p));
  p.base = base;
  p.out = out;
  p.mask = mask;
  p.stride = stride;
  p.ulen = length;
  p.uinit = init;
  run_jobs(p, nblocks, threads);
}
