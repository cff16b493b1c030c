// log::Reader::ReadRecord (db/log_reader.cc:55-176, checksum = true,
// initial_offset = 0) over a whole WAL / MANIFEST image on the device: the
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
// and one workgroup does it in three passes over contiguous chunks:
//
//   1. each thread summarises its chunk (Summ); a scan of the summaries gives
//      every chunk the reader's state at its start;
//   2. each thread replays its chunk from that state, counting records,
//      reports and bytes; a scan gives output positions;
//   3. each thread replays it again and writes records and reports; then the
//      records' LastRecordOffset values are filled in parallel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device_common.h"
#include "lvkv_crc32c.h"
#include "lvkv_log_events.h"

namespace lvkv {
namespace {

constexpr uint32_t kAT = 1024;  // threads of the one workgroup

enum : uint32_t { kIdle = 0, kInFrag = 1, kStopped = 2, kUnknown = 3 };

// A run of events as a transformer of the reader's state.
struct Summ {
  uint32_t pass;     // 1: only MIDDLE records (or no events)
  uint32_t c;        // !pass: the state after the run, whatever came before
  uint64_t len;      // pass: payload bytes of its MIDDLE records
  uint64_t scratch;  // !pass, c == kInFrag: bytes of the open fragment
  uint32_t first;    // !pass, c == kInFrag: its FIRST, candidates from the run's start
  uint32_t nrec;     // candidate records in the run (additive)
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
  uint32_t st;       // kIdle / kInFrag / kStopped, or kUnknown (pass 1)
  uint32_t first;    // kInFrag: the fragment's FIRST
  uint64_t scratch;  // kInFrag (kUnknown: MIDDLE bytes so far)
  uint32_t stopped;  // a kEof-type header stopped the reader here
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
  __device__ __forceinline__ void record(uint32_t first, uint32_t nfrags, uint64_t len) {
    if (write && nrec < rec_cap) {
      lvkv_log_record r;
      r.offset = 0;  // LastRecordOffset: filled in after the pass
      r.length = len;
      r.first = first;
      r.nfrags = nfrags;
      recs[nrec] = r;
    }
    ++nrec;
    bytes += len;
  }
};

// One event (item `ev`, candidate index j for a record) through ReadRecord's
// switch (log_reader.cc:86-166). kUnknown (pass 1) emits nothing: a MIDDLE
// keeps it, any other event resolves it.
template <bool kOut>
__device__ __forceinline__ void step(Reader& r, uint32_t ev, uint32_t j, Sink& out) {
  const uint32_t kind = ev & 15u;
  const uint64_t n = ev >> 16;  // payload bytes / drop bytes
  if (r.st == kStopped || kind == kEvSkip || kind == kEvNone) return;
  const bool in = r.st == kInFrag;
  if (kind != kEvRec) {
    if (kind == kEvEof) {  // kEof: an open fragment is dropped silently (:138-144)
      r.st = kStopped;
      return;
    }
    // kBadRecord; ReadPhysicalRecord reported it first (:221-255)
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
      if (kOut) out.record(j, 1, n);
      r.st = kIdle;
      break;
    case 2:  // kFirstType (:100-112)
      if (kOut && in && r.scratch != 0) out.report(r.scratch, LVKV_LOGR_PARTIAL_2, 0);
      r.st = kInFrag;
      r.first = j;
      r.scratch = n;
      break;
    case 3:  // kMiddleType (:114-121)
      if (in || r.st == kUnknown) {
        r.scratch += n;
      } else if (kOut) {
        out.report(n, LVKV_LOGR_MISSING_1, 0);
      }
      break;
    case 4:  // kLastType (:123-134)
      if (in) {
        if (kOut) out.record(r.first, j - r.first + 1u, r.scratch + n);
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

// Replays items [k0, k1) (candidate records from j0 on) from `r`, eight
// event loads in flight at a time.
template <bool kOut>
__device__ __forceinline__ uint32_t replay(const uint32_t* events, uint32_t k0, uint32_t k1,
                                           uint32_t j0, Reader& r, Sink& out) {
  uint32_t j = j0;
  for (uint32_t k = k0; k < k1; k += 8) {
    uint32_t ev[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      ev[i] = k + i < k1 ? events[k + i] : log_event(kEvNone, 0, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      step<kOut>(r, ev[i], j, out);
      const uint32_t kind = ev[i] & 15u;
      j += (kind == kEvRec || kind == kEvSkip) ? 1u : 0u;
    }
  }
  return j;
}

struct AsmArgs {
  const uint32_t* events;
  const uint64_t* hdr_off;
  const lvkv_log_report* phys;
  uint64_t size;
  uint32_t nblocks;
  uint32_t rec_cap, rep_cap;
  lvkv_log_record* recs;
  lvkv_log_corruption* reps;
  lvkv_log_read_report* out;
};

__global__ void __launch_bounds__(kAT, 1) log_assemble_kernel(AsmArgs a) {
  __shared__ Summ sm[2][kAT];
  __shared__ uint32_t cnt[2][kAT][2];
  __shared__ unsigned long long byt[2][kAT];
  __shared__ uint32_t stop_any;
  const uint32_t tid = threadIdx.x;
  const bool ok = a.phys->status == LVKV_OK;
  // candidate records the verify placed (0 when they did not fit)
  const uint32_t nrec = ok ? a.phys->count_ : 0u;
  const uint32_t K = ok ? nrec + a.nblocks : 0u;
  const uint32_t k0 = static_cast<uint32_t>(static_cast<uint64_t>(tid) * K / kAT);
  const uint32_t k1 = static_cast<uint32_t>(static_cast<uint64_t>(tid + 1) * K / kAT);
  if (tid == 0) stop_any = 0;

  // 1. the chunk's summary, then an inclusive scan of the summaries
  Sink none = {false, 0, 0, 0, nullptr, 0, nullptr, 0};
  Reader u = {kUnknown, 0, 0, 0};
  const uint32_t jend = replay<false>(a.events, k0, k1, 0, u, none);
  Summ s;
  s.pass = u.st == kUnknown ? 1u : 0u;
  s.c = u.st;
  s.len = s.pass ? u.scratch : 0;
  s.scratch = u.scratch;
  s.first = u.first;
  s.nrec = jend;
  uint32_t cur = 0;
  sm[cur][tid] = s;
  __syncthreads();
  for (uint32_t d = 1; d < kAT; d <<= 1) {
    if (tid >= d) s = compose(sm[cur][tid - d], s);
    sm[cur ^ 1u][tid] = s;
    cur ^= 1u;
    __syncthreads();
  }
  // the reader's state at the chunk's start: the log starts idle
  Reader r = {kIdle, 0, 0, 0};
  uint32_t j0 = 0;
  if (tid > 0) {
    const Summ p = sm[cur][tid - 1];
    j0 = p.nrec;
    if (!p.pass) {
      r.st = p.c;
      r.first = p.first;
      r.scratch = p.scratch;
    }
  }

  // 2. counts from that state, exclusive scans of them
  Sink cnt_sink = {false, 0, 0, 0, nullptr, 0, nullptr, 0};
  {
    Reader rr = r;
    replay<true>(a.events, k0, k1, j0, rr, cnt_sink);
    if (rr.stopped) atomicOr(&stop_any, 1u);
  }
  uint32_t c0 = cnt_sink.nrec, c1 = cnt_sink.nrep;
  unsigned long long bb = cnt_sink.bytes;
  cur = 0;
  cnt[cur][tid][0] = c0;
  cnt[cur][tid][1] = c1;
  byt[cur][tid] = bb;
  __syncthreads();
  for (uint32_t d = 1; d < kAT; d <<= 1) {
    if (tid >= d) {
      c0 += cnt[cur][tid - d][0];
      c1 += cnt[cur][tid - d][1];
      bb += byt[cur][tid - d];
    }
    cnt[cur ^ 1u][tid][0] = c0;
    cnt[cur ^ 1u][tid][1] = c1;
    byt[cur ^ 1u][tid] = bb;
    cur ^= 1u;
    __syncthreads();
  }
  const uint32_t rec_base = c0 - cnt_sink.nrec, rep_base = c1 - cnt_sink.nrep;
  const uint32_t nrec_total = cnt[cur][kAT - 1][0], nrep_total = cnt[cur][kAT - 1][1];

  // 3. write them
  Sink w = {true, 0, 0, 0, a.recs + rec_base,
            a.rec_cap > rec_base ? a.rec_cap - rec_base : 0u, a.reps + rep_base,
            a.rep_cap > rep_base ? a.rep_cap - rep_base : 0u};
  replay<true>(a.events, k0, k1, j0, r, w);
  __syncthreads();
  const uint32_t nr = min(nrec_total, a.rec_cap);
  for (uint32_t i = tid; i < nr; i += kAT) a.recs[i].offset = a.hdr_off[a.recs[i].first];
  if (tid == 0) {
    lvkv_log_read_report o;
    o.status = (!ok || nrec_total > a.rec_cap || nrep_total > a.rep_cap) ? LVKV_LOG_CAPACITY
                                                                          : LVKV_OK;
    o.nrecords = nrec_total;
    o.nreports = nrep_total;
    o.stopped = stop_any;
    o.bytes = byt[cur][kAT - 1];
    *a.out = o;
  }
}

}  // namespace

hipError_t launch_log_assemble(const uint32_t* events, const uint64_t* hdr_off,
                               const lvkv_log_report* phys, uint64_t size,
                               lvkv_log_record* recs, uint32_t rec_cap,
                               lvkv_log_corruption* reps, uint32_t rep_cap,
                               lvkv_log_read_report* out, hipStream_t stream) {
  AsmArgs a;
  a.events = events;
  a.hdr_off = hdr_off;
  a.phys = phys;
  a.size = size;
  a.nblocks = static_cast<uint32_t>((size + 32767) / 32768);
  a.rec_cap = rec_cap;
  a.rep_cap = rep_cap;
  a.recs = recs;
  a.reps = reps;
  a.out = out;
  hipLaunchKernelGGL(log_assemble_kernel, dim3(1), dim3(kAT), 0, stream, a);
  return hipGetLastError();
}

}  // namespace lvkv
