// log::Reader::ReadRecord (db/log_reader.cc:55-176, checksum = true, any
// initial_offset) over a whole WAL / MANIFEST image on the device: the
// logical records the reader returns (FULL, or FIRST MIDDLE* LAST) and every
// Reporter::Corruption call, physical and logical, in the reader's order.
//
// Input: the event stream lvkv_log_verify_blocks_device leaves in the
// library's scratch (lvkv_log_events.h: one packed u32 per candidate record
// and per block). ReadRecord is a state machine over those events with three
// states: idle, inside a fragmented record (with the fragment's start and
// its bytes so far), stopped (kEof). A run of events acts on that state in
// one of two ways: if it holds only MIDDLE records it passes the state
// through (adding their bytes to an open fragment); otherwise its first
// other event resets the state the same way whatever came before, so the run
// ends in a state of its own. That makes runs composable (Summ, compose),
// and so are their record / report counts kept for each state a run may be
// entered in (Agg, agg_compose). One launch, log_asm_onepass: each thread
// summarises a chunk of kChunk items; a workgroup scan gives each chunk's
// start relative to its workgroup's and the workgroup's aggregate; the
// workgroup publishes it and looks back over the workgroups before it (64 at
// a time, one lane each) to the nearest published inclusive prefix, which
// gives its own starting state and output positions; then it writes its
// records (LastRecordOffset from the verify's header offsets, loaded beside
// the events) and reports. (The earlier form, a reduce launch whose last
// workgroup scanned the aggregates and an emit launch redoing the chunks,
// took the same 29 us on the 62k-record log.)
//
// An initial offset (log_reader.cc:29-54, :80-89, :182-187, :261-266) is
// applied to the events as they are loaded: the blocks before the first one
// the reader reads pass nothing on; in that block, records that start before
// the offset become silent kBadRecords (kEvPre) and a physical report whose
// header lies before the offset is dropped; and the reader starts in a
// fourth state, resyncing (MIDDLE and one LAST consumed silently). A
// one-wave launch first finds that block's candidates (log_asm_seek).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "crc32c_device_common.h"
#include "lvkv_crc32c.h"
#include "lvkv_log_events.h"

namespace lvkv {
namespace {


enum : uint32_t { kIdle = 0, kInFrag = 1, kStopped = 2, kUnknown = 3, kResync = 4 };

// A run of events as a transformer of the reader's state.
struct Summ {
  uint32_t pass;     // 1: only MIDDLE records (or no events)
  uint32_t c;        // !pass: the state after the run, whatever came before
  uint64_t len;      // pass: payload bytes of its MIDDLE records
  uint64_t scratch;  // !pass, c == kInFrag: bytes of the open fragment
  uint32_t first;    // !pass, c == kInFrag: its FIRST, candidates from the run's start
  uint32_t nrec;     // candidate records in the run (additive)
  uint32_t stop5;    // c == kStopped because of a header of type 5
};

__device__ __forceinline__ Summ compose(const Summ& x, const Summ& y) {
  Summ r;
  if (!x.pass && x.c == kStopped) {
    r = x;  // the reader stopped: nothing after it counts
  } else if (!y.pass) {
    r = y;
    r.first = y.first + x.nrec;  // y's FIRST, counted from x's start
  } else if (x.pass) {
    r = x;
    r.len = x.len + y.len;
  } else {
    r = x;
    if (x.c == kInFrag) r.scratch += y.len;
  }
  r.nrec = x.nrec + y.nrec;
  return r;
}

// The reader's state while a chunk is replayed.
struct Reader {
  uint32_t st;       // kIdle / kInFrag / kStopped / kResync, or kUnknown (summaries)
  uint32_t first;    // kInFrag: the fragment's FIRST
  uint64_t scratch;  // kInFrag (kUnknown: MIDDLE bytes so far)
  uint32_t stopped;  // a kEof-type header stopped the reader here
  uint64_t first_off;  // kInFrag, emit pass: the FIRST's header offset
};

// Output sinks: pass 2 counts, pass 3 writes.
struct Sink {
  bool write;
  uint32_t nrec, nrep;
  uint64_t bytes;
  lvkv_log_record* recs;
  uint32_t rec_cap;
  lvkv_log_corruption* reps;
  uint32_t rep_cap;

  __device__ __forceinline__ void report(uint64_t bytes_, uint32_t reason, uint32_t type) {
    if (write && nrep < rep_cap) {
      lvkv_log_corruption c;
      c.bytes = bytes_;
      c.reason = reason;
      c.type = type;
      reps[nrep] = c;
    }
    ++nrep;
  }
  __device__ __forceinline__ void record(uint64_t off, uint32_t first, uint32_t nfrags,
                                         uint64_t len) {
    if (write && nrec < rec_cap) {
      lvkv_log_record r;
      r.offset = off;
      r.length = len;
      r.first = first;
      r.nfrags = nfrags;
      recs[nrec] = r;
    }
    ++nrec;
    bytes += len;
  }
};

// One event (item `ev`; for a record its candidate index j and header offset
// hoff) through ReadRecord's switch (log_reader.cc:86-166). kUnknown (the
// summaries) emits nothing: a MIDDLE keeps it, any other event resolves it.
// kResync (:80-89) acts as kIdle except that a MIDDLE is consumed silently
// and a LAST silently ends it.
template <bool kOut>
__device__ __forceinline__ void step(Reader& r, uint32_t ev, uint32_t j, uint64_t hoff,
                                     Sink& out) {
  const uint32_t kind = ev & 15u;
  const uint64_t n = ev >> 16;  // payload bytes / drop bytes
  if (r.st == kStopped || kind == kEvSkip || kind == kEvNone) return;
  const bool in = r.st == kInFrag;
  if (kind != kEvRec) {
    if (kind == kEvEof) {  // kEof: an open fragment is dropped silently (:138-144)
      r.st = kStopped;
      return;
    }
    // kBadRecord; ReadPhysicalRecord reported it first (:221-255); kEvPre /
    // kEvZero: silently
    if (kOut && kind == kEvChecksum) out.report(n, LVKV_LOGR_CHECKSUM, 0);
    if (kOut && kind == kEvBadLength) out.report(n, LVKV_LOGR_BAD_LENGTH, 0);
    if (kOut && in) out.report(r.scratch, LVKV_LOGR_MIDDLE, 0);  // :145-151
    r.st = kIdle;
    return;
  }
  const uint32_t type = (ev >> 8) & 255u;
  switch (type) {
    case 1:  // kFullType (:86-98)
      if (kOut && in && r.scratch != 0) out.report(r.scratch, LVKV_LOGR_PARTIAL_1, 0);
      if (kOut) out.record(hoff, j, 1, n);
      r.st = kIdle;
      break;
    case 2:  // kFirstType (:100-112)
      if (kOut && in && r.scratch != 0) out.report(r.scratch, LVKV_LOGR_PARTIAL_2, 0);
      r.st = kInFrag;
      r.first = j;
      r.first_off = hoff;
      r.scratch = n;
      break;
    case 3:  // kMiddleType (:114-121)
      if (in || r.st == kUnknown) {
        r.scratch += n;
      } else if (kOut && r.st == kIdle) {
        out.report(n, LVKV_LOGR_MISSING_1, 0);
      }
      break;
    case 4:  // kLastType (:123-134)
      if (in) {
        if (kOut) out.record(r.first_off, r.first, j - r.first + 1u, r.scratch + n);
      } else if (kOut && r.st == kIdle) {
        out.report(n, LVKV_LOGR_MISSING_2, 0);
      }
      r.st = kIdle;
      break;
    case 5:  // the header's type byte is kEof: ReadRecord returns false (:136-144)
      r.st = kStopped;
      r.stopped = 1;
      break;
    case 6:  // kBadRecord (:145-151)
      if (kOut && in) out.report(r.scratch, LVKV_LOGR_MIDDLE, 0);
      r.st = kIdle;
      break;
    default:  // zero type with a length, or > kMaxRecordType + 2 (:153-162)
      if (kOut) out.report(n + (in ? r.scratch : 0), LVKV_LOGR_UNKNOWN_TYPE, type);
      r.st = kIdle;
      break;
  }
}

#ifndef LVKV_ASM_CHUNK
#define LVKV_ASM_CHUNK 4
#endif
constexpr uint32_t kChunk = LVKV_ASM_CHUNK;  // items per thread (one 4 kChunk-byte load)
constexpr uint32_t kGT = 256;     // threads per workgroup of the grid launches

__device__ __forceinline__ bool is_candidate(uint32_t ev) {
  const uint32_t kind = ev & 15u;
  return kind == kEvRec || kind == kEvSkip || kind == kEvPre;
}

// Where an initial offset puts the reader (log_asm_seek's result): block b0
// is the first it reads; its candidates are [lo, hi).
struct Seek {
  uint64_t offset;     // initial_offset; 0: no transform
  uint64_t b0;
  uint64_t b0_end;     // file offset of b0's end (the end of its buffer)
  const uint32_t* lohi;
};

// Item k (event ev) as a reader with an initial offset sees it.
__device__ __forceinline__ uint32_t seek_event(const Seek& sk, const uint64_t* hdr_off, uint32_t k,
                                               uint32_t ev) {
  if (sk.offset == 0) return ev;
  const uint32_t kind = ev & 15u;
  const bool cand = kind == kEvRec || kind == kEvSkip;
  const uint64_t lo = sk.lohi[0] + sk.b0, hi = sk.lohi[1] + sk.b0;
  if (k < lo) return cand ? log_event(kEvSkip, 0, 0) : log_event(kEvNone, 0, 0);
  if (k < hi) {  // b0's candidates: those before the offset are skipped silently
    return kind == kEvRec && hdr_off[k - sk.b0] < sk.offset ? log_event(kEvPre, 0, 0) : ev;
  }
  if (k == hi && (kind == kEvChecksum || kind == kEvBadLength) &&
      sk.b0_end - (ev >> 16) < sk.offset)  // ReportDrop's filter: header before the offset
    return log_event(kEvZero, 0, 0);
  return ev;
}

// The chunk's items [k0, k1) into registers (the rest "no event"). k0 is a
// multiple of kChunk and the event array 16-byte aligned.
__device__ __forceinline__ void load_chunk(const uint32_t* events, const uint64_t* hdr_off,
                                           const Seek& sk, uint32_t k0, uint32_t k1,
                                           uint32_t (&ev)[kChunk]) {
  if (kChunk == 4) {
    const uint4 v = k0 < k1 ? reinterpret_cast<const uint4*>(events + k0)[0] : make_uint4(0, 0, 0, 0);
    ev[0] = v.x;
    ev[1 % kChunk] = v.y;
    ev[2 % kChunk] = v.z;
    ev[3 % kChunk] = v.w;
  } else if (kChunk == 2) {
    const uint2 v = k0 < k1 ? reinterpret_cast<const uint2*>(events + k0)[0] : make_uint2(0, 0);
    ev[0] = v.x;
    ev[1 % kChunk] = v.y;
  } else {
    ev[0] = k0 < k1 ? events[k0] : 0u;
  }
#pragma unroll
  for (uint32_t i = 0; i < kChunk; ++i)
    ev[i] = k0 + i >= k1 ? log_event(kEvNone, 0, 0) : seek_event(sk, hdr_off, k0 + i, ev[i]);
}

// v[i] for a run-time i by unrolled selects (no register array in scratch);
// 0 when i >= N.
template <typename T, uint32_t N>
__device__ __forceinline__ T pick(const T (&v)[N], uint32_t i) {
  T r = 0;
#pragma unroll
  for (uint32_t k = 0; k < N; ++k) r = i == k ? v[k] : r;
  return r;
}

// The chunk through step(); hoff[c] = header offset of its c-th candidate.
template <bool kOut>
__device__ __forceinline__ void replay(const uint32_t (&ev)[kChunk], const uint64_t (&hoff)[kChunk],
                                       uint32_t j0, Reader& r, Sink& out) {
  uint32_t c = 0;
#pragma unroll
  for (uint32_t i = 0; i < kChunk; ++i) {
    step<kOut>(r, ev[i], j0 + c, pick(hoff, c), out);
    c += is_candidate(ev[i]) ? 1u : 0u;
  }
}

constexpr Summ kIdentity = {1, kIdle, 0, 0, 0, 0, 0};  // no events

// A starting state as the counts see it: idle, in a fragment with bytes,
// in an empty fragment, resyncing, stopped.
enum : uint32_t { kScIdle = 0, kScFrag = 1, kScEmpty = 2, kScResync = 3, kScStopped = 4 };
constexpr uint32_t kScenarios = 4;  // the ones with counts

__device__ __forceinline__ uint32_t scenario(uint32_t st, uint64_t scratch) {
  return st == kIdle      ? kScIdle
         : st == kStopped ? kScStopped
         : st == kResync  ? kScResync
         : scratch != 0   ? kScFrag
                          : kScEmpty;
}

// A chunk's start given its workgroup's start (scenario sw) and the
// composed summary `x` of the chunks before it in the workgroup.
__device__ __forceinline__ uint32_t chunk_scenario(uint32_t sw, const Summ& x) {
  if (!x.pass) return scenario(x.c, x.scratch);
  if (sw == kScEmpty && x.len != 0) return kScFrag;
  return sw;
}

// One thread's chunk: events, summary and counts from each starting state.
struct Chunk {
  uint32_t ev[kChunk];
  Summ s;
  uint32_t nrec[kScenarios], nrep[kScenarios];
};

// A chunk's counts from starting scenario sc (kScStopped: none).
__device__ __forceinline__ void chunk_counts(const uint32_t (&ev)[kChunk], uint32_t sc,
                                             uint32_t* nrec, uint32_t* nrep) {
  uint64_t hz[kChunk];
#pragma unroll
  for (uint32_t i = 0; i < kChunk; ++i) hz[i] = 0;
  Sink cnt = {false, 0, 0, 0, nullptr, 0, nullptr, 0};
  Reader r = {sc == kScIdle ? kIdle : sc == kScResync ? kResync : sc == kScStopped ? kStopped : kInFrag,
              0, sc == kScFrag ? 1u : 0u, 0, 0};
  replay<true>(ev, hz, 0, r, cnt);
  *nrec = cnt.nrec;
  *nrep = cnt.nrep;
}

// The chunk's events and summary; with kCounts, its counts from every
// starting scenario too.
template <bool kCounts>
__device__ __forceinline__ void chunk_of(const uint32_t* events, const uint64_t* hdr_off,
                                         const Seek& sk, uint32_t K, uint32_t t, Chunk& c) {
  const uint32_t k0 = t * kChunk;
  load_chunk(events, hdr_off, sk, k0, min(K, k0 + kChunk), c.ev);
  uint64_t hz[kChunk];
#pragma unroll
  for (uint32_t i = 0; i < kChunk; ++i) hz[i] = 0;
  Sink none = {false, 0, 0, 0, nullptr, 0, nullptr, 0};
  Reader u = {kUnknown, 0, 0, 0, 0};
  replay<false>(c.ev, hz, 0, u, none);
  c.s.pass = u.st == kUnknown ? 1u : 0u;
  c.s.c = c.s.pass ? kIdle : u.st;
  c.s.len = c.s.pass ? u.scratch : 0;
  c.s.scratch = c.s.pass ? 0 : u.scratch;
  c.s.first = u.first;
  c.s.stop5 = u.stopped;
  uint32_t n = 0;
#pragma unroll
  for (uint32_t i = 0; i < kChunk; ++i) n += is_candidate(c.ev[i]) ? 1u : 0u;
  c.s.nrec = n;
  if (kCounts) {
#pragma unroll
    for (uint32_t sc = 0; sc < kScenarios; ++sc) chunk_counts(c.ev, sc, &c.nrec[sc], &c.nrep[sc]);
  }
}

__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, uint32_t d) {
  const uint32_t lo = __shfl_up(static_cast<uint32_t>(v), d, 64);
  const uint32_t hi = __shfl_up(static_cast<uint32_t>(v >> 32), d, 64);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

__device__ __forceinline__ Summ shfl_up_summ(const Summ& x, uint32_t d) {
  Summ r;
  r.pass = __shfl_up(x.pass, d, 64);
  r.c = __shfl_up(x.c, d, 64);
  r.len = shfl_up64(x.len, d);
  r.scratch = shfl_up64(x.scratch, d);
  r.first = __shfl_up(x.first, d, 64);
  r.nrec = __shfl_up(x.nrec, d, 64);
  r.stop5 = __shfl_up(x.stop5, d, 64);
  return r;
}

// Workgroup-wide exclusive scan of `s` under compose (kT threads): a shuffle
// scan in each wave, then the waves' aggregates through LDS (two barriers);
// *all = the aggregate.
template <uint32_t kT>
__device__ __forceinline__ Summ wg_scan_excl(Summ s, Summ (&wagg)[kT / 64], uint32_t tid,
                                             Summ* all) {
  const uint32_t lane = tid & 63u, w = tid >> 6;
  Summ inc = s;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const Summ o = shfl_up_summ(inc, d);
    if (lane >= d) inc = compose(o, inc);
  }
  Summ ex = shfl_up_summ(inc, 1);
  if (lane == 0) ex = kIdentity;
  if (lane == 63) wagg[w] = inc;
  __syncthreads();
  Summ pre = kIdentity, tot = kIdentity;
  for (uint32_t v = 0; v < kT / 64; ++v) {
    if (v == w) pre = tot;
    tot = compose(tot, wagg[v]);
  }
  *all = tot;
  __syncthreads();  // wagg is reused
  return compose(pre, ex);
}

// Workgroup-wide exclusive sums of N counters per thread (kT threads), the
// same way; tot[i] = the totals.
template <uint32_t kT, uint32_t N>
__device__ __forceinline__ void wg_sum_excl(uint32_t (&v)[N], uint32_t (&wsum)[kT / 64][N],
                                            uint32_t tid, uint32_t (&tot)[N]) {
  const uint32_t lane = tid & 63u, w = tid >> 6;
  uint32_t inc[N];
#pragma unroll
  for (uint32_t i = 0; i < N; ++i) inc[i] = v[i];
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
#pragma unroll
    for (uint32_t i = 0; i < N; ++i) {
      const uint32_t o = __shfl_up(inc[i], d, 64);
      if (lane >= d) inc[i] += o;
    }
  }
  if (lane == 63) {
#pragma unroll
    for (uint32_t i = 0; i < N; ++i) wsum[w][i] = inc[i];
  }
  __syncthreads();
#pragma unroll
  for (uint32_t i = 0; i < N; ++i) {
    uint32_t pre = 0, all = 0;
    for (uint32_t u = 0; u < kT / 64; ++u) {
      if (u < w) pre += wsum[u][i];
      all += wsum[u][i];
    }
    v[i] = pre + inc[i] - v[i];
    tot[i] = all;
  }
  __syncthreads();  // wsum is reused
}

// A run of events (a chunk, a workgroup, a run of workgroups) as a map of
// the reader's state: its composed summary and its record / report counts
// for each state the reader may enter it in. Runs of them compose
// associatively (agg_compose), which is what the look-back needs.
struct Agg {
  Summ s;
  uint32_t nrec[kScenarios], nrep[kScenarios];
};

// A workgroup's look-back slot: its aggregate, then its inclusive prefix (the
// composition of every workgroup up to it), each published by a release of
// `flag` = call tag << 2 | 1 or 2.
struct AsmSlot {
  uint32_t flag, pad_[3];
  Agg agg, incl;
};

struct AsmArgs {
  const uint32_t* events;
  const uint64_t* hdr_off;
  const lvkv_log_report* phys;
  uint32_t nblocks;
  uint32_t rec_cap, rep_cap;
  uint32_t groups;  // workgroups of the grid launches
  uint32_t init_st; // the reader's first state: kIdle, or kResync with an offset
  Seek seek;
  uint32_t* lohi;   // log_asm_seek's output (seek.lohi)
  uint32_t tag;     // this call's look-back tag (never 0, < 2^30)
  uint32_t* done;   // workgroups finished (left at 0 by the last one)
  unsigned long long* bytes;  // the records' bytes, summed (left at 0 by the last one)
  lvkv_log_record* recs;
  lvkv_log_corruption* reps;
  lvkv_log_read_report* out;
  AsmSlot* slots;
};

// Items on the device: candidate records the verify placed, plus blocks.
__device__ __forceinline__ uint32_t asm_items(const AsmArgs& a) {
  return a.phys->status == LVKV_OK ? a.phys->count_ + a.nblocks : 0u;
}

// lower_bound(hdr_off[0, n), key) by one wave: a 64-way search, one round of
// loads per factor of 64.
__device__ uint32_t wave_lower_bound(const uint64_t* hdr_off, uint32_t n, uint64_t key,
                                     uint32_t lane) {
  uint32_t lo = 0, len = n;
  while (len > 64) {
    const uint32_t s = (len + 63) / 64;
    const uint32_t idx = lo + (lane + 1) * s - 1;
    const bool below = idx < lo + len && hdr_off[idx] < key;
    const uint32_t c = __popcll(__ballot(below));  // segments wholly below: a prefix
    const uint32_t nlo = lo + c * s;
    len = nlo >= lo + len ? 0u : min(s, lo + len - nlo);
    lo = nlo;
  }
  const bool below = lane < len && hdr_off[lo + lane] < key;
  return lo + static_cast<uint32_t>(__popcll(__ballot(below)));
}

// The first block the reader reads (b0, log_reader.cc:33-54): its candidates
// [lo, hi) among the verify's, which are in file order.
__global__ void __launch_bounds__(64) log_asm_seek(AsmArgs a) {
  const uint32_t lane = threadIdx.x;
  const uint32_t n = a.phys->status == LVKV_OK ? a.phys->count_ : 0u;
  const uint32_t lo = wave_lower_bound(a.hdr_off, n, a.seek.b0 * 32768ull, lane);
  const uint32_t hi = wave_lower_bound(a.hdr_off, n, (a.seek.b0 + 1) * 32768ull, lane);
  if (lane == 0) {
    a.lohi[0] = lo;
    a.lohi[1] = hi;
  }
}

// Y after X: the summary composed; for each entering scenario, X's counts
// and Y's from the state X leaves it in (none once X has stopped the reader).
__device__ __forceinline__ Agg agg_compose(const Agg& x, const Agg& y) {
  Agg r;
  r.s = compose(x.s, y.s);
#pragma unroll
  for (uint32_t sc = 0; sc < kScenarios; ++sc) {
    const uint32_t after = chunk_scenario(sc, x.s);  // kScStopped: pick gives 0
    r.nrec[sc] = x.nrec[sc] + pick(y.nrec, after);
    r.nrep[sc] = x.nrep[sc] + pick(y.nrep, after);
  }
  return r;
}

constexpr Agg kAggIdentity = {kIdentity, {0, 0, 0, 0}, {0, 0, 0, 0}};

__device__ __forceinline__ Agg shfl_agg(const Agg& v, uint32_t src) {
  Agg r;
  r.s.pass = __shfl(v.s.pass, src, 64);
  r.s.c = __shfl(v.s.c, src, 64);
  r.s.len = __shfl(static_cast<unsigned long long>(v.s.len), src, 64);
  r.s.scratch = __shfl(static_cast<unsigned long long>(v.s.scratch), src, 64);
  r.s.first = __shfl(v.s.first, src, 64);
  r.s.nrec = __shfl(v.s.nrec, src, 64);
  r.s.stop5 = __shfl(v.s.stop5, src, 64);
#pragma unroll
  for (uint32_t i = 0; i < kScenarios; ++i) {
    r.nrec[i] = __shfl(v.nrec[i], src, 64);
    r.nrep[i] = __shfl(v.nrep[i], src, 64);
  }
  return r;
}

// Slot words move as agent-scope relaxed atomics (sc1: through to the
// coherent level, no L1/L2 maintenance). The publisher's stores are waited
// for (vmcnt) before its flag store, and a reader reads the words only after
// seeing the flag: an acquire per wait would invalidate the XCD's L2 each
// time (a first form with acquire spins took 678 us a call).
template <typename T>
__device__ __forceinline__ T sc1_ld(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void sc1_st(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ Agg load_agg(const Agg* p) {
  Agg r;
  r.s.pass = sc1_ld(&p->s.pass);
  r.s.c = sc1_ld(&p->s.c);
  r.s.len = sc1_ld(&p->s.len);
  r.s.scratch = sc1_ld(&p->s.scratch);
  r.s.first = sc1_ld(&p->s.first);
  r.s.nrec = sc1_ld(&p->s.nrec);
  r.s.stop5 = sc1_ld(&p->s.stop5);
#pragma unroll
  for (uint32_t i = 0; i < kScenarios; ++i) {
    r.nrec[i] = sc1_ld(&p->nrec[i]);
    r.nrep[i] = sc1_ld(&p->nrep[i]);
  }
  return r;
}

__device__ __forceinline__ void store_agg(Agg* p, const Agg& v) {
  sc1_st(&p->s.pass, v.s.pass);
  sc1_st(&p->s.c, v.s.c);
  sc1_st(&p->s.len, v.s.len);
  sc1_st(&p->s.scratch, v.s.scratch);
  sc1_st(&p->s.first, v.s.first);
  sc1_st(&p->s.nrec, v.s.nrec);
  sc1_st(&p->s.stop5, v.s.stop5);
#pragma unroll
  for (uint32_t i = 0; i < kScenarios; ++i) {
    sc1_st(&p->nrec[i], v.nrec[i]);
    sc1_st(&p->nrep[i], v.nrep[i]);
  }
}

// ReadRecord over every event in ONE launch (reduce, look-back, emit):
// workgroup g's chunks are summarised and scanned (each chunk's start
// relative to the workgroup's; the workgroup's aggregate with its counts for
// each entering state); wave 0 publishes the aggregate, then looks back over
// the slots of the workgroups before it, 64 at a time (one lane each, all
// loads at once), composing aggregates back to the nearest published
// inclusive prefix (a shuffle tree: the composition is associative), and
// publishes its own prefix. Lower workgroups were dispatched first and
// publish their aggregates without waiting on anyone, so every wait ends.
// Then the workgroup's records and reports are written from the known start
// state and output positions. The last workgroup to finish (a completion
// counter it leaves at 0) writes the report.
__global__ void __launch_bounds__(kGT) log_asm_onepass(AsmArgs a) {
  __shared__ Summ wagg[kGT / 64];
  __shared__ uint32_t wsum[kGT / 64][2 * kScenarios];
  __shared__ Agg start_s;
  __shared__ uint32_t last_s;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u;
  const uint32_t K = asm_items(a);
  // workgroups with items (at least one, which writes the report)
  const uint32_t G = max(1u, min(a.groups, (K + kGT * kChunk - 1) / (kGT * kChunk)));
  const uint32_t g = blockIdx.x;
  if (g >= G) return;  // the whole workgroup; nothing waits on it
  Chunk c;
  chunk_of<true>(a.events, a.hdr_off, a.seek, K, g * kGT + tid, c);
  Agg agg;
  const Summ x = wg_scan_excl<kGT>(c.s, wagg, tid, &agg.s);
  {
    uint32_t v[2 * kScenarios], tot[2 * kScenarios];
#pragma unroll
    for (uint32_t sw = 0; sw < kScenarios; ++sw) {
      const uint32_t sc = chunk_scenario(sw, x);
      v[2 * sw] = pick(c.nrec, sc);  // 0 when stopped
      v[2 * sw + 1] = pick(c.nrep, sc);
    }
    wg_sum_excl<kGT>(v, wsum, tid, tot);
#pragma unroll
    for (uint32_t sw = 0; sw < kScenarios; ++sw) {
      agg.nrec[sw] = tot[2 * sw];
      agg.nrep[sw] = tot[2 * sw + 1];
    }
  }
  // ---- look-back (wave 0) ----
  if (tid < 64) {
    AsmSlot* me = a.slots + g;
    if (lane == 0) {
      store_agg(&me->agg, agg);
      __hip_atomic_store(&me->flag, (a.tag << 2) | 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    Agg before = kAggIdentity;  // every workgroup before g, composed
    for (int32_t hi = static_cast<int32_t>(g) - 1; hi >= 0; hi -= 64) {
      // lane l: workgroup hi - 63 + l (lanes below 0: the identity)
      const int32_t w = hi - 63 + static_cast<int32_t>(lane);
      uint32_t f = 0;
      if (w >= 0) {
        while (((f = __hip_atomic_load(&a.slots[w].flag, __ATOMIC_ACQUIRE,
                                       __HIP_MEMORY_SCOPE_AGENT)) >> 2) != a.tag)
          __builtin_amdgcn_s_sleep(1);
        f &= 3u;
      }
      // the nearest inclusive prefix: the window starts there
      const uint64_t pm = __ballot(f == 2u);
      const uint32_t from = pm ? 63u - static_cast<uint32_t>(__builtin_clzll(pm)) : 0u;
      Agg v = kAggIdentity;
      if (w >= 0 && lane >= from) v = load_agg(lane == from && pm ? &a.slots[w].incl : &a.slots[w].agg);
      // fold the window in lane order (a shuffle tree: lane 63 ends with all)
#pragma unroll
      for (uint32_t d = 1; d < 64; d <<= 1) {
        const Agg o = shfl_agg(v, (lane >= d ? lane - d : lane));
        if (lane >= d) v = agg_compose(o, v);
      }
      const Agg win = shfl_agg(v, 63);
      before = agg_compose(win, before);
      if (pm) break;
    }
    if (lane == 0) {
      store_agg(&me->incl, agg_compose(before, agg));
      __hip_atomic_store(&me->flag, (a.tag << 2) | 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      start_s = before;
    }
  }
  __syncthreads();
  // ---- emit from the workgroup's start ----
  const Agg p = start_s;
  const uint32_t in_st = p.s.pass ? a.init_st : p.s.c;
  const uint64_t in_scratch = p.s.pass ? 0 : p.s.scratch;
  const uint32_t init_sc = scenario(a.init_st, 0);
  const uint32_t rec_base = pick(p.nrec, init_sc), rep_base = pick(p.nrep, init_sc);
  const uint32_t j_base = p.s.nrec;
  Reader r = {in_st, p.s.first, in_scratch, 0, 0};
  if (!x.pass) {
    r.st = x.c;
    r.first = j_base + x.first;
    r.scratch = x.scratch;
  } else if (r.st == kInFrag) {
    r.scratch += x.len;
  }
  const uint32_t sw = scenario(in_st, in_scratch);
  const uint32_t sc = chunk_scenario(sw, x);
  uint32_t v[2], t[2];  // this chunk's counts from its known start (0 when stopped)
  chunk_counts(c.ev, sc, &v[0], &v[1]);
  {
    uint32_t (&ws2)[kGT / 64][2] = *reinterpret_cast<uint32_t (*)[kGT / 64][2]>(&wsum[0][0]);
    wg_sum_excl<kGT>(v, ws2, tid, t);
  }
  const uint32_t rb = v[0] + rec_base, pb = v[1] + rep_base;
  const uint32_t j0 = j_base + x.nrec;
  uint64_t hoff[kChunk];
#pragma unroll
  for (uint32_t i = 0; i < kChunk; ++i) hoff[i] = i < c.s.nrec ? a.hdr_off[j0 + i] : 0;
  if (r.st == kInFrag) r.first_off = a.hdr_off[r.first];
  Sink out = {true, 0, 0, 0, a.recs + rb, a.rec_cap > rb ? a.rec_cap - rb : 0u, a.reps + pb,
              a.rep_cap > pb ? a.rep_cap - pb : 0u};
  replay<true>(c.ev, hoff, j0, r, out);
  // the records' bytes: one atomic per wave
  unsigned long long bytes = out.bytes;
  for (int d = 32; d >= 1; d >>= 1) bytes += __shfl_xor(bytes, d, 64);
  if (lane == 0 && bytes) atomicAdd(a.bytes, bytes);
  // ---- the last workgroup to finish writes the report ----
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_s_waitcnt(0);  // this workgroup's byte atomics have landed
    const uint32_t n = __hip_atomic_fetch_add(a.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_s = n == G - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (!last_s || tid != 0) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const Agg tot = load_agg(&a.slots[G - 1].incl);  // published before its arrival
  const uint32_t r0 = pick(tot.nrec, init_sc), r1 = pick(tot.nrep, init_sc);
  lvkv_log_read_report o;
  o.status = (a.phys->status != LVKV_OK || r0 > a.rec_cap || r1 > a.rep_cap) ? LVKV_LOG_CAPACITY
                                                                              : LVKV_OK;
  o.nrecords = r0;
  o.nreports = r1;
  o.stopped = (!tot.s.pass && tot.s.c == kStopped) ? tot.s.stop5 : 0u;
  o.bytes = __hip_atomic_load(a.bytes, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  *a.out = o;
  // the next call with this scratch reuses the counters
  __hip_atomic_store(a.bytes, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(a.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- the records' bytes ---------------------------------------------------
//
// ReadRecord hands back each record as one buffer (scratch->assign/append,
// *record = Slice(*scratch), db/log_reader.cc:92-137). Here every record is
// written end to end into one output: physical candidate j belongs to a
// returned record iff the last record whose first fragment is <= j also
// spans j (records are in order and their fragments disjoint, a binary
// search over their `first`); its payload goes to dest[j] = the payloads of
// the returned fragments before it (a scan over candidates), so record i
// starts at dest[first_i]. Two launches: the places (1024 candidates a
// workgroup, the scan across workgroups by decoupled look-back: each
// workgroup publishes its aggregate, then its inclusive prefix, under the
// call's tag, and waits only on lower workgroups, dispatched before it),
// then the copies, one wave per candidate.

constexpr uint32_t kGatherT = 256, kGatherItems = 4, kGatherPer = kGatherT * kGatherItems;

// A workgroup's look-back slot: its aggregate, then its inclusive prefix,
// each published by a release of `tag` = call tag << 2 | 1 or 2.
struct LookSlot {
  unsigned long long agg, incl;
  uint32_t tag, pad_[3];
};

struct GatherArgs {
  const uint8_t* file;
  const uint64_t* hdr_off;
  const lvkv_log_report* phys;
  const lvkv_log_record* recs;
  const lvkv_log_read_report* read;
  uint32_t rec_cap;
  uint32_t tag;           // the call's look-back tag (never 0)
  uint8_t* out;
  uint64_t out_cap;
  uint64_t* rec_pos;      // nullable
  struct LookSlot* look;  // per workgroup
  ulonglong2* dst;  // per candidate: {its payload's place in `out` (~0: not returned),
                   //  payload file offset | length << 48}
};

// The u16 at p (any alignment) from the aligned dword(s) holding it: no
// misaligned sub-dword global load.
__device__ __forceinline__ uint32_t ld_u16_any(const uint8_t* p) {
  const uint64_t x = reinterpret_cast<uint64_t>(p);
  const uint32_t* d = reinterpret_cast<const uint32_t*>(x & ~uint64_t{3});
  const uint32_t sh = static_cast<uint32_t>(x & 3u);
  const uint32_t lo = d[0];
  const uint32_t hi = sh == 3u ? d[1] : 0u;
  return __builtin_amdgcn_alignbyte(hi, lo, sh) & 0xffffu;
}

// Index of the last record whose first fragment is <= j (or -1).
__device__ __forceinline__ int32_t owner_of(const lvkv_log_record* recs, uint32_t n, uint32_t j) {
  uint32_t lo = 0, hi = n;  // first record with first > j
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (recs[mid].first <= j) lo = mid + 1; else hi = mid;
  }
  return static_cast<int32_t>(lo) - 1;
}

__global__ void __launch_bounds__(kGatherT) log_gather_kernel(GatherArgs a) {
  __shared__ unsigned long long wsum[kGatherT / 64];
  __shared__ unsigned long long base_s;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u, wave = tid >> 6;
  const uint32_t N = a.phys->status == LVKV_OK ? a.phys->count_ : 0u;
  const uint32_t R = a.phys->status == LVKV_OK ? min(a.read->nrecords, a.rec_cap) : 0u;
  const uint32_t g = blockIdx.x;
  if (g * kGatherPer >= N) return;  // the whole workgroup; nothing waits on it
  // this thread's candidates: owned payload lengths
  const uint32_t j0 = g * kGatherPer + tid * kGatherItems;
  uint32_t len[kGatherItems];
  int32_t own[kGatherItems];
  uint64_t mine = 0;
#pragma unroll
  for (uint32_t t = 0; t < kGatherItems; ++t) {
    const uint32_t j = j0 + t;
    len[t] = 0;
    own[t] = -1;
    if (j < N && R != 0) {
      const int32_t i = owner_of(a.recs, R, j);
      if (i >= 0 && j < a.recs[i].first + a.recs[i].nfrags) {
        len[t] = ld_u16_any(a.file + a.hdr_off[j] + 4);
        own[t] = i;
      }
    }
    mine += len[t];
  }
  // workgroup scan
  uint64_t inc = mine;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t o = __shfl_up(static_cast<unsigned long long>(inc), d, 64);
    if (lane >= d) inc += o;
  }
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  uint64_t pre = 0, agg = 0;
#pragma unroll
  for (uint32_t w = 0; w < kGatherT / 64; ++w) {
    if (w < wave) pre += wsum[w];
    agg += wsum[w];
  }
  // look-back (thread 0): publish the aggregate, sum predecessors, publish
  // the inclusive prefix
  if (tid == 0) {
    LookSlot* me = a.look + g;
    uint64_t before = 0;
    if (g != 0) {
      __hip_atomic_store(&me->agg, static_cast<unsigned long long>(agg), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&me->tag, (a.tag << 2) | 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      for (int32_t p = static_cast<int32_t>(g) - 1; p >= 0; --p) {
        LookSlot* q = a.look + p;
        uint32_t tw;
        while (((tw = __hip_atomic_load(&q->tag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) >> 2) !=
               a.tag)
          __builtin_amdgcn_s_sleep(1);
        // an inclusive prefix ends the walk; an aggregate adds and goes on
        const bool incl = (tw & 3u) == 2u;
        before += __hip_atomic_load(incl ? &q->incl : &q->agg, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
        if (incl) break;
      }
    }
    __hip_atomic_store(&me->incl, static_cast<unsigned long long>(before + agg), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&me->tag, (a.tag << 2) | 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    base_s = before;
  }
  __syncthreads();
  uint64_t dst = base_s + pre + inc - mine;
#pragma unroll
  for (uint32_t t = 0; t < kGatherItems; ++t) {
    const uint32_t j = j0 + t;
    if (j < N) {
      if (own[t] >= 0 && a.rec_pos != nullptr && a.recs[own[t]].first == j) a.rec_pos[own[t]] = dst;
      // the copy's whole descriptor in one 16-byte entry: place, and the
      // payload's file offset with its length in the top 16 bits
      a.dst[j] = own[t] >= 0 ? make_ulonglong2(dst, (a.hdr_off[j] + 7) | (uint64_t{len[t]} << 48))
                             : make_ulonglong2(~0ull, 0);
    }
    dst += len[t];
  }
}

// The owned fragments' payloads to their places, one wave per candidate (a
// grid of N waves: the copies are latency-bound, so as many as the chip
// holds are in flight; with the copy inside the scan's 61 workgroups it
// took 680 us for a 66 MB log). Each output word is rebuilt from two aligned
// source dwords (a buffer resource over the payload's aligned dwords: a
// dword past them reads as 0; one partly past a range's end would read as 0
// whole); the 0-3 bytes before the output's first 4-byte boundary and after
// its last go bytewise.
__global__ void __launch_bounds__(256) log_gather_copy_kernel(GatherArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t j = blockIdx.x * 4u + (threadIdx.x >> 6);
  const uint32_t N = a.phys->status == LVKV_OK ? a.phys->count_ : 0u;
  if (j >= N) return;
  const ulonglong2 de = a.dst[j];
  const uint64_t d = de.x;
  if (d == ~0ull) return;
  const uint8_t* src = a.file + (de.y & ((uint64_t{1} << 48) - 1));
  const uint32_t l = static_cast<uint32_t>(de.y >> 48);
  if (d + l > a.out_cap) return;
  const uint32_t hb = min(l, (4u - static_cast<uint32_t>(d & 3u)) & 3u);
  if (lane < hb) a.out[d + lane] = src[lane];
  const uint64_t s0 = reinterpret_cast<uint64_t>(src);
  const uint64_t sa = s0 & ~uint64_t{3};
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(sa), 0, static_cast<int>((s0 + l - sa + 3u) & ~uint64_t{3}),
      kBufferDword3);
  const uint32_t nw = (l - hb) >> 2;
  uint32_t* dw = reinterpret_cast<uint32_t*>(a.out + d + hb);
  const uint32_t sb = static_cast<uint32_t>(s0 - sa) + hb;
  // four words a lane in flight per round
  for (uint32_t w0 = 0; w0 < nw; w0 += 256) {
    uint32_t lo[4], hi[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
      const uint32_t so = sb + 4u * (w0 + 64u * u + lane);
      lo[u] = __builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>(so & ~3u), 0, 0);
      hi[u] = __builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>((so & ~3u) + 4u), 0, 0);
    }
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
      const uint32_t w = w0 + 64u * u + lane;
      if (w < nw) dw[w] = __builtin_amdgcn_alignbyte(hi[u], lo[u], sb & 3u);
    }
  }
  const uint32_t tb = (l - hb) & 3u;
  if (lane < tb) a.out[d + hb + 4u * nw + lane] = src[hb + 4u * nw + lane];
}

}  // namespace

size_t log_asm_scratch_bytes(size_t max_items) {
  const size_t groups = (max_items + kGT * kChunk - 1) / (kGT * kChunk);
  return groups * sizeof(AsmSlot) + 16;  // + log_asm_seek's two words
}

// `scratch`: log_asm_scratch_bytes(capacity + nblocks) bytes, 16-byte aligned
// (any contents: slots of other tags are ignored); `done` and `bytes`: a u32
// and a u64 that are 0 (zeroed once; every call leaves them at 0), used by
// one call at a time; `tag`: this call's, never 0, below 2^30.
hipError_t launch_log_assemble(const uint32_t* events, const uint64_t* hdr_off,
                               const lvkv_log_report* phys, uint64_t size, uint32_t capacity,
                               uint64_t initial_offset, lvkv_log_record* recs, uint32_t rec_cap,
                               lvkv_log_corruption* reps, uint32_t rep_cap,
                               lvkv_log_read_report* out, void* scratch, uint32_t* done,
                               unsigned long long* bytes, uint32_t tag, hipStream_t stream) {
  AsmArgs a;
  a.events = events;
  a.hdr_off = hdr_off;
  a.phys = phys;
  a.nblocks = static_cast<uint32_t>((size + 32767) / 32768);
  a.rec_cap = rec_cap;
  a.rep_cap = rep_cap;
  const uint64_t items = uint64_t{capacity} + a.nblocks;
  a.groups = static_cast<uint32_t>((items + kGT * kChunk - 1) / (kGT * kChunk));
  a.recs = recs;
  a.reps = reps;
  a.out = out;
  a.slots = static_cast<AsmSlot*>(scratch);
  a.lohi = reinterpret_cast<uint32_t*>(a.slots + a.groups);
  a.tag = tag;
  a.done = done;
  a.bytes = bytes;
  a.init_st = initial_offset ? kResync : kIdle;
  a.seek.offset = initial_offset;
  // SkipToInitialBlock (log_reader.cc:33-54): the block holding the offset,
  // or the next one when the offset lies in the last 5 bytes (the trailer)
  const uint64_t in_block = initial_offset % 32768;
  a.seek.b0 = (initial_offset - in_block) / 32768 + (in_block > 32768 - 6 ? 1 : 0);
  a.seek.b0_end = std::min<uint64_t>(size, (a.seek.b0 + 1) * 32768);
  a.seek.lohi = a.lohi;
  hipError_t e;
  if (initial_offset) {
    hipLaunchKernelGGL(log_asm_seek, dim3(1), dim3(64), 0, stream, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  hipLaunchKernelGGL(log_asm_onepass, dim3(a.groups), dim3(kGT), 0, stream, a);
  return hipGetLastError();
}

// lvkv_log_gather_device: two launches; `look`: 32 bytes per workgroup of
// ceil(capacity / 1024) (any contents: slots of other tags are ignored), then
// 16 bytes per candidate.
size_t log_gather_scratch_bytes(size_t capacity) {
  return ((capacity + kGatherPer - 1) / kGatherPer) * sizeof(LookSlot) + capacity * 16;
}

hipError_t launch_log_gather(const uint8_t* file, const uint64_t* hdr_off, size_t capacity,
                             const lvkv_log_report* phys, const lvkv_log_record* recs,
                             uint32_t rec_cap, const lvkv_log_read_report* read, uint8_t* out,
                             uint64_t out_cap, uint64_t* rec_pos, void* look, uint32_t tag,
                             hipStream_t stream) {
  GatherArgs a;
  a.file = file;
  a.hdr_off = hdr_off;
  a.phys = phys;
  a.recs = recs;
  a.read = read;
  a.rec_cap = rec_cap;
  a.tag = tag;
  a.out = out;
  a.out_cap = out_cap;
  a.rec_pos = rec_pos;
  a.look = static_cast<LookSlot*>(look);
  const uint32_t groups = static_cast<uint32_t>((capacity + kGatherPer - 1) / kGatherPer);
  a.dst = reinterpret_cast<ulonglong2*>(a.look + groups);
  hipLaunchKernelGGL(log_gather_kernel, dim3(groups), dim3(kGatherT), 0, stream, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(log_gather_copy_kernel, dim3(static_cast<uint32_t>((capacity + 3) / 4)),
                     dim3(256), 0, stream, a);
  return hipGetLastError();
}

}  // namespace lvkv
