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
// entered in (Agg, agg_compose). Two launches, one item per thread, each
// item's summary and its counts for each entering state computed
// straight-line: log_asm_reduce scans each workgroup's items and writes the
// workgroup's aggregate; log_asm_emit composes the summaries of the
// aggregates before its workgroup (64 per wave step, by ballots and wave
// sums: window_summ) into its starting state, counts them for that one state
// (window_counts_sc), rescans its items and puts each through step() once,
// writing records (LastRecordOffset from the header offsets carried with the
// events and in the summaries) and reports. Round 3 measured the alternatives on the
// 62k-record log: chunks of four items replayed through step() five times
// in one launch with a decoupled look-back, 29.7 us; one item per thread
// with the look-back, 34 us (release / acquire flags) and 41 us (flags and
// payloads as device-scope atomics, which contend): the look-back's waits,
// not the arithmetic, were the cost. A kernel boundary is the cheaper
// cross-XCD exchange.
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
  uint64_t first_off;  // !pass, c == kInFrag: its FIRST's header offset
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

// The reader's state before an item.
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

constexpr uint32_t kGT = 256;  // threads (= items) per workgroup of the grid launch

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

// Item k (event ev, header offset off) as a reader with an initial offset
// sees it.
__device__ __forceinline__ uint32_t seek_event(const Seek& sk, uint64_t off, uint32_t k,
                                               uint32_t ev) {
  if (sk.offset == 0) return ev;
  const uint32_t kind = ev & 15u;
  const bool cand = kind == kEvRec || kind == kEvSkip;
  const uint64_t lo = sk.lohi[0] + sk.b0, hi = sk.lohi[1] + sk.b0;
  if (k < lo) return cand ? log_event(kEvSkip, 0, 0) : log_event(kEvNone, 0, 0);
  if (k < hi) {  // b0's candidates: those before the offset are skipped silently
    return kind == kEvRec && off < sk.offset ? log_event(kEvPre, 0, 0) : ev;
  }
  if (k == hi && (kind == kEvChecksum || kind == kEvBadLength) &&
      sk.b0_end - (ev >> 16) < sk.offset)  // ReportDrop's filter: header before the offset
    return log_event(kEvZero, 0, 0);
  return ev;
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

constexpr Summ kIdentity = {1, kIdle, 0, 0, 0, 0, 0, 0};  // no events

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

// An item's start given its run's start (scenario sw) and the composed
// summary `x` of the items before it in the run.
__device__ __forceinline__ uint32_t chunk_scenario(uint32_t sw, const Summ& x) {
  if (sw == kScStopped) return kScStopped;  // nothing after a stop counts
  if (!x.pass) return scenario(x.c, x.scratch);
  if (sw == kScEmpty && x.len != 0) return kScFrag;
  return sw;
}

// One event (its header at `off`) as a run: the state it leaves the reader
// in (step() from an unknown state, straight-line).
__device__ __forceinline__ Summ event_summ(uint32_t ev, uint64_t off) {
  const uint32_t kind = ev & 15u, type = (ev >> 8) & 255u, n = ev >> 16;
  Summ s = kIdentity;
  s.nrec = is_candidate(ev) ? 1u : 0u;
  const bool rec = kind == kEvRec;
  if (kind == kEvSkip || kind == kEvNone) return s;
  if (rec && type == 3) {  // MIDDLE: passes the state through
    s.len = n;
    return s;
  }
  s.pass = 0;
  const bool stop = kind == kEvEof || (rec && type == 5);
  const bool first = rec && type == 2;
  s.c = stop ? kStopped : first ? kInFrag : kIdle;
  s.stop5 = rec && type == 5 ? 1u : 0u;
  s.scratch = first ? n : 0u;
  s.first_off = first ? off : 0u;
  return s;
}

// One event's record / report counts for each entering scenario, packed
// rec | rep << 16 (step()'s outputs, straight-line).
__device__ __forceinline__ void event_counts(uint32_t ev, uint32_t (&cnt)[kScenarios]) {
  const uint32_t kind = ev & 15u, type = (ev >> 8) & 255u;
  const bool rec = kind == kEvRec;
  const bool nop = kind == kEvSkip || kind == kEvNone || kind == kEvEof;
  const uint32_t phys = (kind == kEvChecksum || kind == kEvBadLength) ? 1u : 0u;
#pragma unroll
  for (uint32_t sc = 0; sc < kScenarios; ++sc) {
    const uint32_t idle = sc == kScIdle, frag = sc == kScFrag;
    const uint32_t in = sc == kScFrag || sc == kScEmpty;
    uint32_t nrec = 0, nrep = 0;
    if (rec) {
      nrec = (type == 1 || (type == 4 && in)) ? 1u : 0u;
      nrep = (type == 1 || type == 2) ? frag
             : (type == 3 || type == 4) ? idle
             : type == 5              ? 0u
             : type == 6              ? in
                                      : 1u;
    } else if (!nop) {
      nrep = phys + in;
    }
    cnt[sc] = nrec | (nrep << 16);
  }
}

// One event's returned bytes for each entering scenario (step()'s records):
// a FULL record its payload in any live state, a LAST its payload plus the
// open fragment's bytes (`uses`) when the reader is in a fragment.
__device__ __forceinline__ void event_bytes(uint32_t ev, uint32_t (&eb)[kScenarios],
                                            uint32_t (&eu)[kScenarios]) {
  const uint32_t kind = ev & 15u, type = (ev >> 8) & 255u, n = ev >> 16;
  const bool rec = kind == kEvRec;
#pragma unroll
  for (uint32_t sc = 0; sc < kScenarios; ++sc) {
    const bool in = sc == kScFrag || sc == kScEmpty;
    const bool full = rec && type == 1, last = rec && type == 4 && in;
    eb[sc] = (full || last) ? n : 0u;
    eu[sc] = last ? 1u : 0u;
  }
}

// A run of events (a chunk, a workgroup, a run of workgroups) as a map of
// the reader's state: its composed summary and its record / report counts
// for each state the reader may enter it in. Runs of them compose
// associatively (agg_compose), which is what the look-back needs.
struct Agg {
  Summ s;
  uint32_t nrec[kScenarios], nrep[kScenarios];
  // bytes of the records the run returns, entered in each scenario with an
  // empty fragment; uses[sc]: a LAST before the run's first reset also
  // returns the entering fragment's bytes (add them when they are not 0)
  unsigned long long nbytes[kScenarios];
  uint32_t uses[kScenarios];
};

struct AsmArgs {
  const uint32_t* events;
  const uint64_t* item_off;  // each item's header offset (lvkv_log_events.h)
  const uint64_t* hdr_off;
  const lvkv_log_report* phys;
  uint32_t nblocks;
  uint32_t rec_cap, rep_cap;
  uint32_t groups;  // workgroups of the grid launches
  uint32_t init_st; // the reader's first state: kIdle, or kResync with an offset
  Seek seek;
  uint32_t* lohi;   // log_asm_seek's output (seek.lohi)
  lvkv_log_record* recs;
  lvkv_log_corruption* reps;
  lvkv_log_read_report* out;
  Agg* aggs;        // per workgroup (log_asm_reduce)
  Agg* pref;        // many workgroups: per 64-workgroup window, the windows
                    // before it composed (log_asm_scan); else nullptr
  uint64_t* stamps;  // probe build only: 8 u64 per workgroup
};

// Phase stamps of log_asm_emit (probe build): 0 start, 1 shares and items
// summarised, 2 past barrier 1, 3 counted (past barrier 2), 5 items written.
__device__ __forceinline__ void asm_stamp(const AsmArgs& a, uint32_t slot) {
#ifdef LVKV_PROBE_BUILD
  if (a.stamps != nullptr) a.stamps[blockIdx.x * 8u + slot] = __builtin_amdgcn_s_memrealtime();
#endif
}

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
  // the fragment bytes y is entered with, beyond x's entering ones
  const uint64_t carried = x.s.pass ? x.s.len : (x.s.c == kInFrag ? x.s.scratch : 0u);
#pragma unroll
  for (uint32_t sc = 0; sc < kScenarios; ++sc) {
    const uint32_t after = chunk_scenario(sc, x.s);  // kScStopped: pick gives 0
    r.nrec[sc] = x.nrec[sc] + pick(y.nrec, after);
    r.nrep[sc] = x.nrep[sc] + pick(y.nrep, after);
    const uint32_t yu = pick(y.uses, after);
    r.nbytes[sc] = x.nbytes[sc] + pick(y.nbytes, after) + (yu ? carried : 0u);
    r.uses[sc] = x.uses[sc] | (x.s.pass ? yu : 0u);
  }
  return r;
}

constexpr Agg kAggIdentity = {kIdentity, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};

// (every lane active; DPP, crc32c_device_common.h)
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) { return wave_sum_dpp<uint64_t>(v); }

// The 64 lanes' summaries composed in lane order (a window of aggregates;
// all lanes active), by ballots and sums instead of a tree of compose: the
// state the window's last reset lane leaves (plus the MIDDLE bytes after
// it), or stopped from its first stop lane on.
__device__ __forceinline__ Summ window_summ(const Summ& s, uint32_t lane) {
  const uint64_t Rm = __ballot(!s.pass);
  const uint64_t Sm = __ballot(!s.pass && s.c == kStopped);
  Summ r = kIdentity;
  r.nrec = wave_sum_dpp<uint32_t>(s.nrec);
  if (Sm) {
    r.pass = 0;
    r.c = kStopped;
    r.stop5 = lane_u32(s.stop5, static_cast<uint32_t>(__builtin_ctzll(Sm)));
  } else if (Rm) {
    const uint32_t r0 = 63u - static_cast<uint32_t>(__builtin_clzll(Rm));
    const uint32_t c = lane_u32(s.c, r0);
    const uint64_t tail = wave_sum64(lane > r0 ? s.len : 0u);
    r.pass = 0;
    r.c = c;
    r.scratch = lane_u64(s.scratch, r0) + (c == kInFrag ? tail : 0u);
    r.first = lane_u32(s.first, r0) + wave_sum_dpp<uint32_t>(lane < r0 ? s.nrec : 0u);
    r.first_off = lane_u64(s.first_off, r0);
  } else {
    r.len = wave_sum64(s.len);
  }
  return r;
}

// Lane l of a window is entered in the state of the last reset lane below it
// (rb != 0: scenario `fixed`, whatever the window's), else in the window's own
// entering state (an empty fragment turning non-empty when MIDDLE bytes lie
// below: len_below); `carried`: the fragment bytes it is entered with beyond
// the window's own.
struct WinLane {
  uint64_t rb;
  uint32_t fixed;
  bool len_below;
  uint64_t carried;
};

__device__ __forceinline__ WinLane window_lane(const Summ& s, uint32_t lane) {
  const uint64_t Rm = __ballot(!s.pass);
  const uint64_t Sm = __ballot(!s.pass && s.c == kStopped);
  const uint64_t Lm = __ballot(s.pass && s.len != 0);
  const uint64_t below = (uint64_t{1} << lane) - 1u;
  WinLane L;
  L.rb = Rm & below;
  const uint32_t rl = L.rb ? 63u - static_cast<uint32_t>(__builtin_clzll(L.rb)) : 0u;
  const uint32_t rc = __shfl(s.c, rl, 64);
  const uint64_t rs = __shfl(static_cast<unsigned long long>(s.scratch), rl, 64);
  const uint64_t between = Lm & below & ~((uint64_t{2} << rl) - 1u);  // lanes in (rl, l)
  L.fixed = (Sm & below) ? kScStopped : scenario(rc, rs | (between ? 1u : 0u));
  L.len_below = (Lm & below) != 0;
  // MIDDLE bytes of the lanes below l (exclusive scan), and those after the
  // last reset below l
  const uint64_t incl = wave_scan_dpp<uint64_t>(s.pass ? s.len : 0u, lane);
  const uint64_t excl = incl - (s.pass ? s.len : 0u);
  const uint64_t at_r = __shfl(static_cast<unsigned long long>(incl), rl, 64);
  L.carried = L.rb ? (rc == kInFrag ? rs + (excl - at_r) : 0u) : excl;
  return L;
}

__device__ __forceinline__ uint32_t window_lane_sc(const WinLane& L, uint32_t sw) {
  return L.rb ? L.fixed : (sw == kScEmpty && L.len_below ? kScFrag : sw);
}

// A run's returned records, reports and bytes from one entering scenario.
struct Counts {
  uint32_t nrec, nrep;
  uint64_t nbytes;  // entered with an empty fragment; add its bytes when `uses`
  uint32_t uses;
};

__device__ __forceinline__ Counts window_counts_sc(const Agg& A, const WinLane& L, uint32_t sw) {
  const uint32_t sc = window_lane_sc(L, sw);
  const uint64_t t = wave_sum64(pick(A.nrec, sc) | (uint64_t{pick(A.nrep, sc)} << 32));
  const uint32_t u = pick(A.uses, sc);
  Counts c;
  c.nrec = static_cast<uint32_t>(t);
  c.nrep = static_cast<uint32_t>(t >> 32);
  c.nbytes = wave_sum64(pick(A.nbytes, sc) + (u ? L.carried : 0u));
  c.uses = __ballot(!L.rb && u) ? 1u : 0u;
  return c;
}

// The 64 lanes' aggregates composed in lane order, for every entering
// scenario (log_asm_scan).
__device__ __forceinline__ Agg window_fold(const Agg& A, uint32_t lane) {
  Agg r;
  r.s = window_summ(A.s, lane);
  const WinLane L = window_lane(A.s, lane);
#pragma unroll
  for (uint32_t sw = 0; sw < kScenarios; ++sw) {
    const Counts c = window_counts_sc(A, L, sw);
    r.nrec[sw] = c.nrec;
    r.nrep[sw] = c.nrep;
    r.nbytes[sw] = c.nbytes;
    r.uses[sw] = c.uses;
  }
  return r;
}

// The items of workgroup g: the event of each thread's item, its counts
// for each entering scenario, its summary's exclusive scan in the workgroup
// (x), its exclusive output positions for each scenario the workgroup may be
// entered in (v: rec | rep << 16, at most 256 records and 512 reports), and
// the workgroup's aggregate.
struct Items {
  uint32_t ev;
  uint64_t off;  // the item's header offset (a candidate's)
  Summ x;
  uint32_t v[kScenarios];
  Agg agg;
};

// The composition of the lanes in `below` (a prefix of the wave) as one
// summary, from ballots: the state its last reset lane leaves (plus the
// MIDDLE bytes after it), or stopped from its first stop lane. C / R / S:
// the candidate / reset / stop lanes; P: MIDDLE bytes of the lanes in
// `below`; r: the last reset lane in `below` and its state (c_r, sc_r) and
// inclusive MIDDLE bytes p_r and header offset off_r; stop5_0: the first
// stop lane's stop5.
__device__ __forceinline__ Summ prefix_summ(uint64_t below, uint64_t C, uint64_t R, uint64_t S,
                                            uint32_t P, uint32_t r, uint32_t c_r, uint32_t sc_r,
                                            uint32_t p_r, uint64_t off_r, uint32_t stop5_0) {
  Summ x = kIdentity;
  x.nrec = static_cast<uint32_t>(__popcll(C & below));
  if (S & below) {
    x.pass = 0;
    x.c = kStopped;
    x.stop5 = stop5_0;
  } else if (R & below) {
    x.pass = 0;
    x.c = c_r;
    x.scratch = sc_r + (c_r == kInFrag ? P - p_r : 0u);
    x.first = static_cast<uint32_t>(__popcll(C & ((uint64_t{1} << r) - 1u)));
    x.first_off = off_r;
  } else {
    x.len = P;
  }
  return x;
}

// Item k's event and header offset as loaded (issued before anything that
// waits, so their latency overlaps the emit's fold).
struct ItemIn {
  uint32_t ev;
  uint64_t off;
};
__device__ __forceinline__ ItemIn load_item(const AsmArgs& a, uint32_t K, uint32_t k) {
  ItemIn in;
  in.ev = k < K ? a.events[k] : log_event(kEvNone, 0, 0);
  in.off = k < K ? a.item_off[k] : 0u;
  return in;
}

// The wave's share of workgroup g's items, before the workgroup's barrier:
// each item's event (seek applied) and summary, its exclusive summary within
// the wave (it.x), and the wave's total into wagg[w].
__device__ __forceinline__ void wave_items(const AsmArgs& a, uint32_t g, uint32_t tid,
                                           const ItemIn& in, Summ (&wagg)[kGT / 64], Items& it) {
  const uint32_t lane = tid & 63u, w = tid >> 6;
  const uint32_t k = g * kGT + tid;
  it.ev = seek_event(a.seek, in.off, k, in.ev);
  it.off = in.off;
  const Summ e = event_summ(it.ev, it.off);
  // the wave's exclusive scan of summaries, from ballots
  const uint64_t below = (uint64_t{1} << lane) - 1u;
  const uint64_t C = __ballot(e.nrec != 0);
  const uint64_t R = __ballot(!e.pass);
  const uint64_t S = __ballot(!e.pass && e.c == kStopped);
  const uint32_t len = e.pass ? static_cast<uint32_t>(e.len) : 0u;  // < 2^16 an item
  const uint32_t inc = wave_scan_dpp<uint32_t>(len, lane);
  const uint64_t rb = R & below;
  const uint32_t r = rb ? 63u - static_cast<uint32_t>(__builtin_clzll(rb)) : 0u;
  const uint32_t sc = static_cast<uint32_t>(e.scratch);
  const uint32_t stop5_0 = lane_u32(e.stop5, S ? static_cast<uint32_t>(__builtin_ctzll(S)) : 0u);
  const Summ xw = prefix_summ(below, C, R, S, inc - len, r, __shfl(e.c, r, 64), __shfl(sc, r, 64),
                              __shfl(inc, r, 64),
                              __shfl(static_cast<unsigned long long>(it.off), r, 64), stop5_0);
  // the wave's total (shuffles on every lane, then lane 0 writes it)
  const uint32_t rt = R ? 63u - static_cast<uint32_t>(__builtin_clzll(R)) : 0u;
  const uint32_t p_all = lane_u32(inc, 63), c_rt = lane_u32(e.c, rt);
  const uint32_t sc_rt = lane_u32(sc, rt), p_rt = lane_u32(inc, rt);
  const uint64_t off_rt = lane_u64(it.off, rt);
  if (lane == 0)
    wagg[w] = prefix_summ(~uint64_t{0}, C, R, S, p_all, rt, c_rt, sc_rt, p_rt, off_rt, stop5_0);
  it.x = xw;
}

// After the barrier: the waves before this one composed into it.x, and the
// workgroup's summary (it.agg.s).
__device__ __forceinline__ void items_compose(const Summ (&wagg)[kGT / 64], uint32_t w, Items& it) {
  Summ pre = kIdentity, tot = kIdentity;
#pragma unroll
  for (uint32_t v = 0; v < kGT / 64; ++v) {
    if (v == w) pre = tot;
    tot = compose(tot, wagg[v]);
  }
  it.agg.s = tot;
  it.x = compose(pre, it.x);
}

// The reduce's items: summaries, then the positions and counts for every
// scenario the workgroup may be entered in.
__device__ __forceinline__ void wg_items(const AsmArgs& a, uint32_t g, uint32_t tid,
                                         const ItemIn& in, Summ (&wagg)[kGT / 64],
                                         uint32_t (&wsum)[kGT / 64][kScenarios], Items& it) {
  const uint32_t lane = tid & 63u, w = tid >> 6;
  const uint64_t below = (uint64_t{1} << lane) - 1u;
  wave_items(a, g, tid, in, wagg, it);
  __syncthreads();
  items_compose(wagg, w, it);
  // output positions for each entering scenario: per item at most one
  // record and two reports, so the wave's prefix counts are ballots; and the
  // returned bytes (Agg::nbytes / uses)
  __shared__ unsigned long long wbytes[kGT / 64][kScenarios];
  __shared__ uint32_t wuses[kGT / 64][kScenarios];
  uint32_t cnt[kScenarios], eb[kScenarios], eu[kScenarios];
  event_counts(it.ev, cnt);
  event_bytes(it.ev, eb, eu);
  const uint64_t carried = it.x.pass ? it.x.len : (it.x.c == kInFrag ? it.x.scratch : 0u);
#pragma unroll
  for (uint32_t sw = 0; sw < kScenarios; ++sw) {
    const uint32_t isc = chunk_scenario(sw, it.x);
    const uint32_t c = pick(cnt, isc);
    const uint64_t br = __ballot(c & 1u), b0 = __ballot((c >> 16) & 1u), b1 = __ballot((c >> 17) & 1u);
    it.v[sw] = static_cast<uint32_t>(__popcll(br & below)) |
               static_cast<uint32_t>(__popcll(b0 & below) + 2 * __popcll(b1 & below)) << 16;
    const uint32_t u = pick(eu, isc);
    const uint64_t nb = wave_sum64(pick(eb, isc) + (u ? carried : 0u));
    const uint64_t bu = __ballot(it.x.pass && u);
    if (lane == 0) {
      wsum[w][sw] = static_cast<uint32_t>(__popcll(br)) |
                    static_cast<uint32_t>(__popcll(b0) + 2 * __popcll(b1)) << 16;
      wbytes[w][sw] = nb;
      wuses[w][sw] = bu ? 1u : 0u;
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t sw = 0; sw < kScenarios; ++sw) {
    uint32_t before = 0, all = 0, uses = 0;
    unsigned long long bytes = 0;
#pragma unroll
    for (uint32_t v = 0; v < kGT / 64; ++v) {
      before += v < w ? wsum[v][sw] : 0u;
      all += wsum[v][sw];
      bytes += wbytes[v][sw];
      uses |= wuses[v][sw];
    }
    it.v[sw] += before;
    it.agg.nrec[sw] = all & 0xffffu;
    it.agg.nrep[sw] = all >> 16;
    it.agg.nbytes[sw] = bytes;
    it.agg.uses[sw] = uses;
  }
}

// Workgroups with items (at least one, which writes the report).
__device__ __forceinline__ uint32_t asm_groups(const AsmArgs& a, uint32_t K) {
  return max(1u, min(a.groups, (K + kGT - 1) / kGT));
}

// ReadRecord, launch 1 of 2: each workgroup's aggregate.
__global__ void __launch_bounds__(kGT) log_asm_reduce(AsmArgs a) {
  __shared__ Summ wagg[kGT / 64];
  __shared__ uint32_t wsum[kGT / 64][kScenarios];
  const uint32_t K = asm_items(a);
  if (blockIdx.x >= asm_groups(a, K)) return;
  const ItemIn in = load_item(a, K, blockIdx.x * kGT + threadIdx.x);
  Items it;
  wg_items(a, blockIdx.x, threadIdx.x, in, wagg, wsum, it);
  if (threadIdx.x == 0) a.aggs[blockIdx.x] = it.agg;
}

// Past this many workgroups the emit no longer folds every aggregate before
// its own (a quadratic total): log_asm_scan composes the 64-workgroup
// windows' prefixes first, and each emit workgroup folds one window. (The
// scan is launched when the host's bound, from the capacity, passes it, and
// does nothing when the items on the device do not.)
constexpr uint32_t kAsmFoldMax = 1024;

// ReadRecord, between the two launches when there are many workgroups: the
// exclusive prefix of every 64-workgroup window (pref[k] = windows 0..k-1
// composed). One workgroup; each wave folds a contiguous share of the windows
// (window_fold), the shares' totals are composed in LDS, and each wave walks
// its share again writing the running prefix. Linear in the workgroups.
__global__ void __launch_bounds__(kGT) log_asm_scan(AsmArgs a) {
  __shared__ Agg wtot[kGT / 64];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u, w = tid >> 6;
  const uint32_t G = asm_groups(a, asm_items(a));
  if (G <= kAsmFoldMax) return;  // the emit folds (the host knew only a bound)
  const uint32_t nwin = (G + 63) / 64;
  const uint32_t k0 = w * nwin / (kGT / 64), k1 = (w + 1) * nwin / (kGT / 64);
  Agg part = kAggIdentity;
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t idx = k * 64 + lane;
    part = agg_compose(part, window_fold(idx < G ? a.aggs[idx] : kAggIdentity, lane));
  }
  if (lane == 0) wtot[w] = part;
  __syncthreads();
  Agg run = kAggIdentity;
  for (uint32_t v = 0; v < w; ++v) run = agg_compose(run, wtot[v]);
  for (uint32_t k = k0; k < k1; ++k) {
    if (lane == 0) a.pref[k] = run;
    const uint32_t idx = k * 64 + lane;
    run = agg_compose(run, window_fold(idx < G ? a.aggs[idx] : kAggIdentity, lane));
  }
}

// The reader entering a run: its state (kIdle, kInFrag, kStopped, kResync)
// and the open fragment's bytes.
struct Entry {
  uint32_t st;
  uint64_t scratch;
};

__device__ __forceinline__ Entry entry_after(Entry e, const Summ& y) {
  if (e.st == kStopped) return e;
  if (!y.pass) return Entry{y.c, y.c == kInFrag ? y.scratch : 0u};
  if (e.st == kInFrag) e.scratch += y.len;
  return e;
}

__device__ __forceinline__ uint32_t entry_sc(const Entry& e) { return scenario(e.st, e.scratch); }

// ReadRecord, launch 2 of 2. Wave w takes a contiguous share of the windows
// of earlier workgroups' aggregates (with the windows' prefixes scanned,
// a.pref: wave 0 takes g's window prefix and the workgroups of g's own window
// before it) and composes their summaries while the items are scanned; after
// one barrier every wave knows the state its share is entered in, so it counts
// that share's records, reports and bytes for that one scenario (not all four)
// and the items their positions for the workgroup's; after a second barrier
// each item goes through step() once. Workgroup G - 1 writes the report; no
// workgroup waits for or counts the others (round 3's completion counter, one
// device-scope atomic per workgroup on one address, cost ~5 us). Instruction
// issue is the bound here (one wave per SIMD, every step a latency chain), so
// the single scenario is the saving: round 4 measured 12.2 us folding and
// counting all four.
__global__ void __launch_bounds__(kGT) log_asm_emit(AsmArgs a) {
  constexpr uint32_t kW = kGT / 64;
  constexpr uint32_t kMaxWin = kAsmFoldMax / 64;
  __shared__ Summ wagg[kW];      // the waves' items
  __shared__ Summ share_s[kW];   // the waves' shares of the earlier workgroups
  __shared__ Summ win_s[kMaxWin];  // each window of them (window 0: a.pref's form)
  __shared__ uint32_t srec[kW], srep[kW], own_v[kW], own_u[kW];
  __shared__ unsigned long long sbytes[kW], own_b[kW];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u, w = tid >> 6;
  const uint32_t K = asm_items(a);
  const uint32_t G = asm_groups(a, K);
  const uint32_t g = blockIdx.x;
  if (g >= G) return;  // the whole workgroup
  if (tid == 0) asm_stamp(a, 0);
  const ItemIn in = load_item(a, K, g * kGT + tid);
  // 1. this wave's share: its summary, each window's kept for step 3
  const bool scanned = a.pref != nullptr && G > kAsmFoldMax;
  uint32_t wi0 = 0, wi1 = 0;
  if (!scanned) {
    const uint32_t nwin = (g + 63) / 64;
    wi0 = w * nwin / kW;
    wi1 = (w + 1) * nwin / kW;
  } else if (w == 0) {
    wi0 = g >> 6;
    wi1 = wi0 + 1;
  }
  Summ sh = kIdentity;
  if (scanned && w == 0) sh = a.pref[g >> 6].s;
  // the share's first window whole (step 3 counts it from registers; a wave
  // has one window below 256 workgroups), the others' summaries
  const Agg A0 = wi0 < wi1 && wi0 * 64 + lane < g ? a.aggs[wi0 * 64 + lane] : kAggIdentity;
  for (uint32_t wi = wi0; wi < wi1; ++wi) {
    const uint32_t idx = wi * 64 + lane;
    const Summ ws = window_summ(wi == wi0 ? A0.s : idx < g ? a.aggs[idx].s : kIdentity, lane);
    if (lane == 0) win_s[scanned ? 0u : wi] = ws;
    sh = compose(sh, ws);
  }
  if (lane == 0) share_s[w] = sh;
  Items it;
  wave_items(a, g, tid, in, wagg, it);
  if (tid == 0) asm_stamp(a, 1);
  __syncthreads();
  if (tid == 0) asm_stamp(a, 2);
  items_compose(wagg, w, it);
  // 2. the state each share is entered in (e_w), the workgroup's (e), and the
  // earlier workgroups' summary (P)
  Entry e = {a.init_st, 0}, e_w = e;
  Summ P = kIdentity;
#pragma unroll
  for (uint32_t v = 0; v < kW; ++v) {
    if (v == w) e_w = e;
    const Summ sv = share_s[v];
    e = entry_after(e, sv);
    P = compose(P, sv);
  }
  // 3. this wave's share counted from e_w
  uint32_t crec = 0, crep = 0;
  uint64_t cby = 0;
  if (scanned && w == 0) {
    const Agg& pf = a.pref[g >> 6];
    const uint32_t sc = entry_sc(e_w);
    crec = pick(pf.nrec, sc);
    crep = pick(pf.nrep, sc);
    cby = pick(pf.nbytes, sc) + (pick(pf.uses, sc) ? e_w.scratch : 0u);
    e_w = entry_after(e_w, pf.s);
  }
  for (uint32_t wi = wi0; wi < wi1 && e_w.st != kStopped; ++wi) {
    const uint32_t idx = wi * 64 + lane;
    const Agg A = wi == wi0 ? A0 : idx < g ? a.aggs[idx] : kAggIdentity;
    const Counts c = window_counts_sc(A, window_lane(A.s, lane), entry_sc(e_w));
    crec += c.nrec;
    crep += c.nrep;
    cby += c.nbytes + (c.uses ? e_w.scratch : 0u);
    e_w = entry_after(e_w, win_s[scanned ? 0u : wi]);
  }
  // the items' positions for the workgroup's entering scenario (per item at
  // most one record and two reports: ballots), and for the report the
  // returned bytes
  const uint64_t below = (uint64_t{1} << lane) - 1u;
  const uint32_t isc = chunk_scenario(entry_sc(e), it.x);
  uint32_t cnt[kScenarios];
  event_counts(it.ev, cnt);
  const uint32_t c1 = pick(cnt, isc);
  const uint64_t br = __ballot(c1 & 1u), b0 = __ballot((c1 >> 16) & 1u), b1 = __ballot((c1 >> 17) & 1u);
  const uint32_t vpos = static_cast<uint32_t>(__popcll(br & below)) |
                        static_cast<uint32_t>(__popcll(b0 & below) + 2 * __popcll(b1 & below)) << 16;
  const bool last = g == G - 1;
  uint64_t ob = 0;
  uint32_t ou = 0;
  if (last) {
    uint32_t eb[kScenarios], eu[kScenarios];
    event_bytes(it.ev, eb, eu);
    const uint64_t carried = it.x.pass ? it.x.len : (it.x.c == kInFrag ? it.x.scratch : 0u);
    const uint32_t u = pick(eu, isc);
    ob = wave_sum64(pick(eb, isc) + (u ? carried : 0u));
    ou = __ballot(it.x.pass && u) ? 1u : 0u;
  }
  if (lane == 0) {
    srec[w] = crec;
    srep[w] = crep;
    sbytes[w] = cby;
    own_v[w] = static_cast<uint32_t>(__popcll(br)) |
               static_cast<uint32_t>(__popcll(b0) + 2 * __popcll(b1)) << 16;
    own_b[w] = ob;
    own_u[w] = ou;
  }
  __syncthreads();
  if (tid == 0) asm_stamp(a, 3);
  uint32_t base_rec = 0, base_rep = 0, before = 0, all = 0, ouses = 0;
  uint64_t by = 0;
#pragma unroll
  for (uint32_t v = 0; v < kW; ++v) {
    base_rec += srec[v];
    base_rep += srep[v];
    by += sbytes[v] + own_b[v];
    before += v < w ? own_v[v] : 0u;
    all += own_v[v];
    ouses |= own_u[v];
  }
  const Summ& x = it.x;
  const uint32_t ev = it.ev;
  const uint32_t pos = before + vpos;
  const uint32_t rb = base_rec + (pos & 0xffffu);
  const uint32_t pb = base_rep + (pos >> 16);
  const uint32_t j = P.nrec + x.nrec;  // the item's candidate index
  Reader r = {e.st, P.first, e.scratch, 0, P.first_off};
  if (e.st == kStopped) {
    // a stop before this workgroup: nothing after it is read
  } else if (!x.pass) {
    r.st = x.c;
    r.first = P.nrec + x.first;
    r.scratch = x.scratch;
    r.first_off = x.first_off;
  } else if (r.st == kInFrag) {
    r.scratch += x.len;
  }
  // a FULL record's offset is its own header's, a LAST's its FIRST's (carried
  // in the summaries): no load waits on the shares or the scan
  Sink out = {true, 0, 0, 0, a.recs + rb, a.rec_cap > rb ? a.rec_cap - rb : 0u, a.reps + pb,
              a.rep_cap > pb ? a.rep_cap - pb : 0u};
  step<true>(r, ev, j, it.off, out);
  // the report: the earlier workgroups' counts and this one's, from the
  // reader's first state
  if (last && tid == 0) {
    const Summ ts = compose(P, it.agg.s);
    const uint32_t r0 = base_rec + (all & 0xffffu), r1 = base_rep + (all >> 16);
    a.out->status = (a.phys->status != LVKV_OK || r0 > a.rec_cap || r1 > a.rep_cap)
                        ? LVKV_LOG_CAPACITY
                        : LVKV_OK;
    a.out->nrecords = r0;
    a.out->nreports = r1;
    a.out->stopped = (!ts.pass && ts.c == kStopped) ? ts.stop5 : 0u;
    a.out->bytes = by + (ouses ? e.scratch : 0u);
  }
  if (tid == 0) asm_stamp(a, 5);
}

// ---- the records' bytes ---------------------------------------------------
//
// ReadRecord hands back each record as one buffer (scratch->assign/append,
// *record = Slice(*scratch), db/log_reader.cc:92-137). Here every record is
// written end to end into one output: physical candidate j belongs to
// returned record i iff first_i <= j < first_i + nfrags_i (records are in
// order and their fragments disjoint); its payload goes to dest[j] = the
// payloads of the returned fragments before it (a scan over candidates), so
// record i starts at dest[first_i]. Four launches: each record marks its
// fragments with its index (tagged with the call, so nothing is cleared);
// each candidate's owner and length (1024 candidates a workgroup) with the
// workgroup's sum; the places (each workgroup folds the sums before it, 64
// per wave step, and scans its own); the copies. (A binary search over the
// records' `first` per thread, the round-3 owner launch, took 12.7 us on
// the 62k-record log: 16 dependent loads a thread. With the scan across
// workgroups as a decoupled look-back in one launch, the first two took
// 22-28 us: waits on other XCDs' flags.)

constexpr uint32_t kGatherT = 256, kGatherItems = 4, kGatherPer = kGatherT * kGatherItems;

// A workgroup's payload bytes (log_gather_own_kernel).
struct LookSlot {
  unsigned long long sum, pad_;
};

struct GatherArgs {
  const uint8_t* file;
  const uint64_t* hdr_off;
  const lvkv_log_report* phys;
  const lvkv_log_record* recs;
  const lvkv_log_read_report* read;
  uint32_t rec_cap;
  uint32_t cap;           // candidates the scratch holds (the read call's capacity)
  uint8_t* out;
  uint64_t out_cap;
  uint64_t* rec_pos;      // nullable
  struct LookSlot* look;  // per workgroup
  ulonglong2* dst;  // per candidate: .x = {the marking record, tagged (launch 1); its owner
                    //  (launch 2), then its payload's place in `out` (launch 3); ~0: not
                    //  returned}, .y = payload file offset | length << 48
  uint32_t tag;     // this call's mark tag: bit 31 set, bit 30 clear (never ~0's high
                    //  word nor a place's, < 2^14)
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

// Launch 1: record i marks its fragments' entries with (tag << 32) | i.
__global__ void __launch_bounds__(256) log_gather_mark_kernel(GatherArgs a) {
  const uint32_t N = a.phys->status == LVKV_OK ? min(a.phys->count_, a.cap) : 0u;
  const uint32_t R = a.phys->status == LVKV_OK ? min(a.read->nrecords, a.rec_cap) : 0u;
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= R) return;
  const lvkv_log_record r = a.recs[i];
  const unsigned long long m = (static_cast<unsigned long long>(a.tag) << 32) | i;
  const uint32_t end = static_cast<uint32_t>(min<uint64_t>(N, uint64_t{r.first} + r.nfrags));
  for (uint32_t f = r.first; f < end; ++f) a.dst[f].x = m;
}

// Launch 2: each candidate's owner record (its mark, if this call's) and
// payload length into dst, and the workgroup's sum of owned lengths.
__global__ void __launch_bounds__(kGatherT) log_gather_own_kernel(GatherArgs a) {
  __shared__ unsigned long long wsum[kGatherT / 64];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u, wave = tid >> 6;
  const uint32_t N = a.phys->status == LVKV_OK ? min(a.phys->count_, a.cap) : 0u;
  const uint32_t g = blockIdx.x;
  if (g * kGatherPer >= N) return;
  const uint32_t j0 = g * kGatherPer + tid * kGatherItems;
  uint64_t mine = 0;
  unsigned long long mk[kGatherItems];
  uint64_t ho[kGatherItems];
#pragma unroll
  for (uint32_t t = 0; t < kGatherItems; ++t) {
    const uint32_t j = j0 + t;
    mk[t] = j < N ? a.dst[j].x : ~0ull;
    ho[t] = j < N ? a.hdr_off[j] : 0;
  }
  const uint32_t R = a.phys->status == LVKV_OK ? min(a.read->nrecords, a.rec_cap) : 0u;
#pragma unroll
  for (uint32_t t = 0; t < kGatherItems; ++t) {
    const uint32_t j = j0 + t;
    if (j >= N) break;
    // this call's mark, naming a record that spans j: the tag alone could be
    // matched by stale scratch bytes (the buffer is pooled with other
    // calls'), the span check cannot (fragments of returned records are
    // disjoint, and every fragment of one was marked by it)
    const uint32_t i = static_cast<uint32_t>(mk[t]);
    bool owned = static_cast<uint32_t>(mk[t] >> 32) == a.tag && i < R;
    if (owned) {
      const lvkv_log_record r = a.recs[i];
      owned = r.first <= j && j - r.first < r.nfrags;
    }
    const uint32_t len = owned ? ld_u16_any(a.file + ho[t] + 4) : 0u;
    a.dst[j] = make_ulonglong2(owned ? (mk[t] & 0xffffffffull) : ~0ull,
                               (ho[t] + 7) | (uint64_t{len} << 48));
    mine += len;
  }
  const uint64_t w = wave_sum64(mine);
  if (lane == 0) wsum[wave] = w;
  __syncthreads();
  if (tid == 0) {
    uint64_t agg = 0;
#pragma unroll
    for (uint32_t v = 0; v < kGatherT / 64; ++v) agg += wsum[v];
    a.look[g].sum = agg;
  }
}

// Launch 3: the places. Wave 0 sums the workgroups before this one while
// every thread reads its candidates' lengths; a workgroup scan; dst[j].x
// becomes the payload's place (~0: not returned), and each record's first
// fragment gives its position.
__global__ void __launch_bounds__(kGatherT) log_gather_kernel(GatherArgs a) {
  __shared__ unsigned long long wsum[kGatherT / 64];
  __shared__ unsigned long long base_s;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u, wave = tid >> 6;
  const uint32_t N = a.phys->status == LVKV_OK ? min(a.phys->count_, a.cap) : 0u;
  const uint32_t g = blockIdx.x;
  if (g * kGatherPer >= N) return;
  const uint32_t j0 = g * kGatherPer + tid * kGatherItems;
  ulonglong2 de[kGatherItems];
  uint64_t mine = 0;
#pragma unroll
  for (uint32_t t = 0; t < kGatherItems; ++t) {
    de[t] = j0 + t < N ? a.dst[j0 + t] : make_ulonglong2(~0ull, 0);
    mine += de[t].y >> 48;
  }
  if (tid < 64) {
    uint64_t before = 0;
    for (uint32_t b = 0; b < g; b += 64) before += wave_sum64(b + lane < g ? a.look[b + lane].sum : 0u);
    if (lane == 0) base_s = before;
  }
  const uint64_t inc = wave_scan_dpp<uint64_t>(mine, lane);
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  uint64_t pre = 0;
#pragma unroll
  for (uint32_t w = 0; w < kGatherT / 64; ++w)
    if (w < wave) pre += wsum[w];
  uint64_t dst = base_s + pre + inc - mine;
#pragma unroll
  for (uint32_t t = 0; t < kGatherItems; ++t) {
    const uint32_t j = j0 + t;
    if (j < N) {
      const bool owned = de[t].x != ~0ull;
      if (owned && a.rec_pos != nullptr && a.recs[de[t].x].first == j) a.rec_pos[de[t].x] = dst;
      a.dst[j].x = owned ? dst : ~0ull;
    }
    dst += de[t].y >> 48;
  }
}

// The owned fragments' payloads to their places. A bounded grid (a few
// workgroups per CU, whatever the capacity); wave v takes candidates v, v + W,
// ... and walks them as a stream of 1 KiB units (candidate, round): the next
// unit's loads are issued before the current unit's stores, and each
// candidate's place is fetched one candidate ahead, so two units of every wave
// are in flight. A lane moves 16 consecutive output bytes a round, each word
// rebuilt from two aligned source dwords (one 16-byte and one 4-byte buffer
// load over the payload's aligned dwords: a dword past them reads as 0, one
// partly past a range's end would read as 0 whole; eight 4-byte loads and
// four 4-byte stores a lane, this round's first form, took 35 us on the
// 62k-record log); the 0-3 bytes before the
// output's first 4-byte boundary and after its last go bytewise. (One wave per candidate over a grid of N waves: 50 us for the
// 62k-record log, and a grid sized by the capacity that passed 2^32
// work-items above ~470 MB images.)
struct CopyJob {
  const uint8_t* src;  // payload start
  uint8_t* dst;        // its place
  uint32_t l;          // bytes (0: nothing to copy)
  uint32_t rounds;     // 1 KiB rounds of whole output words (at least 1)
};

__device__ __forceinline__ CopyJob copy_job(const GatherArgs& a, ulonglong2 de) {
  CopyJob c;
  const uint64_t d = de.x;
  c.l = static_cast<uint32_t>(de.y >> 48);
  c.src = a.file + (de.y & ((uint64_t{1} << 48) - 1));
  if (d == ~0ull || d + c.l > a.out_cap) c.l = 0;
  c.dst = a.out + (c.l ? d : 0);
  const uint32_t hb = min(c.l, (4u - static_cast<uint32_t>(reinterpret_cast<uint64_t>(c.dst) & 3u)) & 3u);
  const uint32_t nw = (c.l - hb) >> 2;
  c.rounds = max(1u, (nw + 255u) >> 8);
  return c;
}

typedef uint32_t CopyV4 __attribute__((ext_vector_type(4)));

// A lane's part of a round: output words w0 .. w0 + 3 (w0 = 256 r + 4 lane)
// from the five aligned source dwords holding them.
struct CopyRegs {
  CopyV4 d;    // source dwords k0 .. k0 + 3
  uint32_t e;  // source dword k0 + 4
};

// Loads of round r of job c: one 16-byte and one 4-byte buffer load a lane.
__device__ __forceinline__ CopyRegs copy_load(const CopyJob& c, uint32_t r, uint32_t lane) {
  CopyRegs x;
  const uint64_t s0 = reinterpret_cast<uint64_t>(c.src);
  const uint64_t sa = s0 & ~uint64_t{3};
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(sa), 0, static_cast<int>((s0 + c.l - sa + 3u) & ~uint64_t{3}),
      kBufferDword3);
  const uint32_t hb = min(c.l, (4u - static_cast<uint32_t>(reinterpret_cast<uint64_t>(c.dst) & 3u)) & 3u);
  const uint32_t sb = static_cast<uint32_t>(s0 - sa) + hb;
  const int off = static_cast<int>((sb & ~3u) + 4u * (256u * r + 4u * lane));
  x.d = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
  x.e = __builtin_amdgcn_raw_buffer_load_b32(rs, off + 16, 0, 0);
  return x;
}

// Stores of round r of job c (the head and tail bytes with round 0): one
// 16-byte store a lane where its four words are all inside the payload.
__device__ __forceinline__ void copy_store(const CopyJob& c, uint32_t r, uint32_t lane,
                                           const CopyRegs& x) {
  if (c.l == 0) return;
  const uint32_t hb = min(c.l, (4u - static_cast<uint32_t>(reinterpret_cast<uint64_t>(c.dst) & 3u)) & 3u);
  const uint32_t nw = (c.l - hb) >> 2;
  const uint32_t sh = static_cast<uint32_t>(reinterpret_cast<uint64_t>(c.src) + hb) & 3u;
  uint32_t* dw = reinterpret_cast<uint32_t*>(c.dst + hb);
  const uint32_t w0 = 256u * r + 4u * lane;
  CopyV4 o;
  o.x = __builtin_amdgcn_alignbyte(x.d.y, x.d.x, sh);
  o.y = __builtin_amdgcn_alignbyte(x.d.z, x.d.y, sh);
  o.z = __builtin_amdgcn_alignbyte(x.d.w, x.d.z, sh);
  o.w = __builtin_amdgcn_alignbyte(x.e, x.d.w, sh);
  if (w0 + 4u <= nw) {
    __builtin_memcpy(dw + w0, &o, 16);  // (4-byte aligned: one dwordx4 store on gfx950)
  } else {
    if (w0 < nw) dw[w0] = o.x;
    if (w0 + 1u < nw) dw[w0 + 1u] = o.y;
    if (w0 + 2u < nw) dw[w0 + 2u] = o.z;
  }
  if (r == 0) {
    if (lane < hb) c.dst[lane] = c.src[lane];
    const uint32_t tb = (c.l - hb) & 3u;
    if (lane < tb) c.dst[hb + 4u * nw + lane] = c.src[hb + 4u * nw + lane];
  }
}

__global__ void __launch_bounds__(256) log_gather_copy_kernel(GatherArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t W = gridDim.x * 4u;
  const uint32_t N = a.phys->status == LVKV_OK ? min(a.phys->count_, a.cap) : 0u;
  uint32_t j = blockIdx.x * 4u + wave;
  if (j >= N) return;
  CopyJob c = copy_job(a, a.dst[j]);
  ulonglong2 de_next = j + W < N ? a.dst[j + W] : make_ulonglong2(~0ull, 0);
  uint32_t r = 0;
  CopyRegs x = copy_load(c, 0, lane);
  for (;;) {
    // the next unit: the job's next round, or the next candidate's round 0
    CopyJob cn = c;
    uint32_t rn = r + 1;
    uint32_t jn = j;
    if (rn == c.rounds) {
      jn = j + W;
      rn = 0;
      if (jn < N) {
        cn = copy_job(a, de_next);
        de_next = jn + W < N ? a.dst[jn + W] : make_ulonglong2(~0ull, 0);
      }
    }
    const bool more = jn < N;
    CopyRegs xn;
    if (more) xn = copy_load(cn, rn, lane);
    copy_store(c, r, lane, x);
    if (!more) break;
    c = cn;
    r = rn;
    j = jn;
    x = xn;
  }
}

}  // namespace

#ifdef LVKV_PROBE_BUILD
uint64_t* g_asm_stamps = nullptr;  // lvkv_debug_asm_stamps
#endif

size_t log_asm_scratch_bytes(size_t max_items) {
  const size_t groups = (max_items + kGT - 1) / kGT;
  // the aggregates, the window prefixes, log_asm_seek's two words
  return (groups + (groups + 63) / 64) * sizeof(Agg) + 16;
}

// `scratch`: log_asm_scratch_bytes(capacity + nblocks) bytes, 16-byte aligned
// (any contents); `events` / `item_off`: the verify's event stream and the
// items' header offsets (lvkv_log_events.h); `hdr_off`: the candidates'
// (log_asm_seek's search).
hipError_t launch_log_assemble(const uint32_t* events, const uint64_t* item_off,
                               const uint64_t* hdr_off, const lvkv_log_report* phys,
                               uint64_t size, uint32_t capacity, uint64_t initial_offset,
                               lvkv_log_record* recs, uint32_t rec_cap,
                               lvkv_log_corruption* reps, uint32_t rep_cap,
                               lvkv_log_read_report* out, void* scratch, hipStream_t stream) {
  AsmArgs a;
  a.events = events;
  a.item_off = item_off;
  a.hdr_off = hdr_off;
  a.phys = phys;
  a.nblocks = static_cast<uint32_t>((size + 32767) / 32768);
  a.rec_cap = rec_cap;
  a.rep_cap = rep_cap;
  const uint64_t items = uint64_t{capacity} + a.nblocks;
  a.groups = static_cast<uint32_t>((items + kGT - 1) / kGT);
  a.recs = recs;
  a.reps = reps;
  a.out = out;
  a.aggs = static_cast<Agg*>(scratch);
#ifdef LVKV_PROBE_BUILD
  a.stamps = g_asm_stamps;
#else
  a.stamps = nullptr;
#endif
  const uint32_t nwin = (a.groups + 63) / 64;
  a.pref = a.groups > kAsmFoldMax ? a.aggs + a.groups : nullptr;
  a.lohi = reinterpret_cast<uint32_t*>(a.aggs + a.groups + nwin);
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
  hipLaunchKernelGGL(log_asm_reduce, dim3(a.groups), dim3(kGT), 0, stream, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (a.pref != nullptr) {
    hipLaunchKernelGGL(log_asm_scan, dim3(1), dim3(kGT), 0, stream, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  hipLaunchKernelGGL(log_asm_emit, dim3(a.groups), dim3(kGT), 0, stream, a);
  return hipGetLastError();
}

// lvkv_log_gather_device: four launches; `look`: 16 bytes per workgroup of
// ceil(capacity / 1024), then 16 bytes per candidate (any contents: the
// marks carry `tag`, a per-call value, so stale entries are never taken for
// this call's).
size_t log_gather_scratch_bytes(size_t capacity) {
  return ((capacity + kGatherPer - 1) / kGatherPer) * sizeof(LookSlot) + capacity * 16;
}

hipError_t launch_log_gather(const uint8_t* file, const uint64_t* hdr_off, size_t capacity,
                             const lvkv_log_report* phys, const lvkv_log_record* recs,
                             uint32_t rec_cap, const lvkv_log_read_report* read, uint8_t* out,
                             uint64_t out_cap, uint64_t* rec_pos, void* look, uint32_t tag,
                             int cus, hipStream_t stream) {
  GatherArgs a;
  a.file = file;
  a.hdr_off = hdr_off;
  a.phys = phys;
  a.recs = recs;
  a.read = read;
  a.rec_cap = rec_cap;
  a.cap = static_cast<uint32_t>(capacity);
  a.out = out;
  a.out_cap = out_cap;
  a.rec_pos = rec_pos;
  a.look = static_cast<LookSlot*>(look);
  a.tag = (tag & 0x3fffffffu) | 0x80000000u;
  const uint32_t groups = static_cast<uint32_t>((capacity + kGatherPer - 1) / kGatherPer);
  a.dst = reinterpret_cast<ulonglong2*>(a.look + groups);
  hipLaunchKernelGGL(log_gather_mark_kernel, dim3(std::max(1u, (rec_cap + 255u) / 256u)),
                     dim3(256), 0, stream, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(log_gather_own_kernel, dim3(groups), dim3(kGatherT), 0, stream, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(log_gather_kernel, dim3(groups), dim3(kGatherT), 0, stream, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // the copy: a bounded grid (8 workgroups of 4 waves per CU), grid-stride
  // over the candidates the device counted
  const uint32_t copy_groups = static_cast<uint32_t>(
      std::min<uint64_t>((capacity + 3) / 4, uint64_t{8} * static_cast<uint64_t>(cus)));
  hipLaunchKernelGGL(log_gather_copy_kernel, dim3(std::max(1u, copy_groups)), dim3(256), 0,
                     stream, a);
  return hipGetLastError();
}

}  // namespace lvkv
