// The event stream log::Reader::ReadRecord consumes (db/log_reader.cc:55-176),
// one packed u32 per item, as lvkv_log_verify_blocks_device leaves it for
// the logical-record kernel (lvkv_log_assemble.hip): item order is block by
// block, each block's candidate physical records in file order, then the
// block's own event. Candidate record g of block b is item g + b; block b's
// event is item (records in blocks 0..b) + b. Beside it, one u64 per item:
// a candidate's header offset in the file (hdr_off of its record), so the
// logical layer reads an item's offset with its event instead of after
// counting the candidates before it.
//
//   bits 0-3   kind (kEv*)
//   bits 8-15  kEvRec: the header's type byte
//   bits 16-31 kEvRec: payload length; block events: reported drop bytes
#ifndef LVKV_LOG_EVENTS_H_
#define LVKV_LOG_EVENTS_H_

#include <stdint.h>

#include "lvkv_crc32c.h"

namespace lvkv {

enum : uint32_t {
  kEvRec = 0,       // a record ReadPhysicalRecord returns (checksum passed)
  kEvSkip = 1,      // a candidate that is not returned (mismatch, dropped)
  kEvNone = 2,      // a block that ends without an error
  kEvChecksum = 3,  // kBadRecord, "checksum mismatch" reported (:243-255)
  kEvBadLength = 4, // kBadRecord, "bad record length" reported (:221-232)
  kEvZero = 5,      // kBadRecord, silent (zero-type zero-length, :234-240)
  kEvEof = 6,       // kEof: truncated record or header at the end (:206-213, :228)
  // Written by the logical layer only, for a reader with an initial offset:
  kEvPre = 7,       // a candidate that started before initial_offset: a silent
                    // kBadRecord (:261-266)
};

__host__ __device__ inline uint32_t log_event(uint32_t kind, uint32_t type, uint32_t len) {
  return kind | (type << 8) | (len << 16);
}

// Block b's event from its LVKV_LOGBLK_* verdict and drop bytes.
__host__ __device__ inline uint32_t log_block_event(uint32_t status, uint32_t drop) {
  switch (status) {
    case LVKV_LOGBLK_CHECKSUM: return log_event(kEvChecksum, 0, drop);
    case LVKV_LOGBLK_BAD_LENGTH: return log_event(kEvBadLength, 0, drop);
    case LVKV_LOGBLK_ZERO: return log_event(kEvZero, 0, 0);
    case LVKV_LOGBLK_EOF: return log_event(kEvEof, 0, 0);
    default: return log_event(kEvNone, 0, 0);
  }
}

}  // namespace lvkv

#endif  // LVKV_LOG_EVENTS_H_
