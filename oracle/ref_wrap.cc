// TEST INFRASTRUCTURE ONLY — C-ABI wrapper around the reference's own
// leveldb::crc32c::Extend (/root/reference/util/crc32c.cc:276), compiled in
// place from /root/reference by oracle/Makefile into oracle/_ref/ (git-ignored,
// never copied into the repo). Used (a) to pin the C restatement in
// crc32c_oracle.c and (b) as bench.py's cpu_baseline kind "reference".
#include <pthread.h>

#include <cstddef>
#include <cstdint>
#include <vector>

#include "util/crc32c.h"

extern "C" {

uint32_t ref_crc32c_extend(uint32_t crc, const char* data, size_t n) {
  return leveldb::crc32c::Extend(crc, data, n);
}

uint32_t ref_crc32c_mask(uint32_t crc) { return leveldb::crc32c::Mask(crc); }
uint32_t ref_crc32c_unmask(uint32_t c) { return leveldb::crc32c::Unmask(c); }

struct RefJob {
  const char* base;
  uint64_t stride;
  uint32_t length, init;
  uint32_t* out;
  size_t begin, end;
};

static void* ref_worker(void* arg) {
  RefJob* j = static_cast<RefJob*>(arg);
  for (size_t i = j->begin; i < j->end; ++i)
    j->out[i] = leveldb::crc32c::Extend(j->init, j->base + i * j->stride,
                                        j->length);
  return nullptr;
}

// Uniform-stride batch over `threads` POSIX threads, static contiguous
// partition (SURVEY.md §8(d) CPU-baseline plan).
void ref_crc32c_uniform(const char* base, uint64_t stride, uint32_t length,
                        uint32_t init, uint32_t* out, size_t nblocks,
                        int threads) {
  if (threads < 1) threads = 1;
  std::vector<RefJob> jobs(threads);
  std::vector<pthread_t> tids(threads);
  size_t per = nblocks / threads, extra = nblocks % threads, at = 0;
  for (int t = 0; t < threads; ++t) {
    jobs[t] = RefJob{base, stride, length, init, out, at, 0};
    at += per + (static_cast<size_t>(t) < extra ? 1 : 0);
    jobs[t].end = at;
  }
  if (threads == 1) {
    ref_worker(&jobs[0]);
    return;
  }
  for (int t = 0; t < threads; ++t)
    pthread_create(&tids[t], nullptr, ref_worker, &jobs[t]);
  for (int t = 0; t < threads; ++t) pthread_join(tids[t], nullptr);
}

// Ragged batch, 1 thread: block i = base[offsets[i], + lengths[i]).
void ref_crc32c_batch(const char* base, const uint64_t* offsets, const uint32_t* lengths,
                      uint32_t* out, size_t n) {
  for (size_t i = 0; i < n; ++i) out[i] = leveldb::crc32c::Value(base + offsets[i], lengths[i]);
}

}  // extern "C"
