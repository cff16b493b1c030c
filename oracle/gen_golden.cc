// TEST INFRASTRUCTURE ONLY — golden-fixture generator.
//
// Built by `make -C oracle golden` against the reference sources where they
// lie under /root/reference (never copied). It runs the reference's own code
// to produce the data files committed under tests/golden/:
//
//   kat.json            util/crc32c_test.cc:12-53 vectors + self-test values,
//                       recomputed by the reference Extend/Value/Mask/Unmask
//   corpus.json         length x misalignment x init corpus
//   blocks1000_crc.bin  1000 x 4096 B splitmix64 blocks, u32 LE CRCs (item 3)
//   table.sst           an SST written by leveldb::TableBuilder, kNoCompression,
//                       block_size 4096, bloom filter (item 4)
//   table_blocks.json   every block handle + trailer of table.sst, each
//                       re-verified through leveldb::ReadBlock(verify_checksums)
//   wal.log             a log written by leveldb::log::Writer with FULL, FIRST,
//                       MIDDLE, LAST and zero-length records (item 5)
//   wal_records.json    every physical record of wal.log; the whole log is
//                       re-read through leveldb::log::Reader(checksum=true)
//
// Data bytes come from splitmix64 (Steele et al.; state += 0x9E3779B97F4A7C15,
// two xor-shift-multiply rounds), 8 little-endian bytes per output, so tests
// regenerate the same bytes in numpy instead of storing them.
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "db/log_format.h"
#include "db/log_reader.h"
#include "db/log_writer.h"
#include "leveldb/env.h"
#include "leveldb/filter_policy.h"
#include "leveldb/options.h"
#include "leveldb/table_builder.h"
#include "table/format.h"
#include "util/coding.h"
#include "util/crc32c.h"

namespace {

using leveldb::Slice;
using leveldb::Status;

uint64_t splitmix_next(uint64_t* state) {
  uint64_t z = (*state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

std::vector<uint8_t> splitmix_bytes(uint64_t seed, size_t n) {
  std::vector<uint8_t> out((n + 7) & ~size_t{7});
  uint64_t st = seed;
  for (size_t i = 0; i < out.size(); i += 8) {
    uint64_t v = splitmix_next(&st);
    for (int b = 0; b < 8; ++b) out[i + b] = static_cast<uint8_t>(v >> (8 * b));
  }
  out.resize(n);
  return out;
}

std::string hex(const uint8_t* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s;
  for (size_t i = 0; i < n; ++i) {
    s.push_back(d[p[i] >> 4]);
    s.push_back(d[p[i] & 15]);
  }
  return s;
}

FILE* open_out(const std::string& dir, const char* name, const char* mode) {
  std::string path = dir + "/" + name;
  FILE* f = std::fopen(path.c_str(), mode);
  if (!f) {
    std::perror(path.c_str());
    std::exit(1);
  }
  return f;
}

// In-memory WritableFile (the pattern of db/log_test.cc StringDest).
class StringSink : public leveldb::WritableFile {
 public:
  std::string contents;
  Status Append(const Slice& s) override {
    contents.append(s.data(), s.size());
    return Status::OK();
  }
  Status Close() override { return Status::OK(); }
  Status Flush() override { return Status::OK(); }
  Status Sync() override { return Status::OK(); }
};

// Records the sequence of Append sizes so block handles can be recovered:
// TableBuilder::WriteRawBlock appends contents then the 5-byte trailer
// (table/table_builder.cc:192-209); Finish() ends with the 48-byte footer.
class RecordingSink : public StringSink {
 public:
  std::vector<size_t> appends;
  Status Append(const Slice& s) override {
    appends.push_back(s.size());
    return StringSink::Append(s);
  }
};

class StringRandomAccess : public leveldb::RandomAccessFile {
 public:
  explicit StringRandomAccess(const std::string* s) : s_(s) {}
  Status Read(uint64_t offset, size_t n, Slice* result,
              char* scratch) const override {
    if (offset > s_->size()) return Status::InvalidArgument("offset");
    size_t avail = s_->size() - offset;
    if (n > avail) n = avail;
    std::memcpy(scratch, s_->data() + offset, n);
    *result = Slice(scratch, n);
    return Status::OK();
  }

 private:
  const std::string* s_;
};

class StringSequential : public leveldb::SequentialFile {
 public:
  explicit StringSequential(const std::string* s) : s_(s) {}
  Status Read(size_t n, Slice* result, char* scratch) override {
    size_t avail = s_->size() - pos_;
    if (n > avail) n = avail;
    std::memcpy(scratch, s_->data() + pos_, n);
    pos_ += n;
    *result = Slice(scratch, n);
    return Status::OK();
  }
  Status Skip(uint64_t n) override {
    pos_ += n;
    if (pos_ > s_->size()) pos_ = s_->size();
    return Status::OK();
  }

 private:
  const std::string* s_;
  size_t pos_ = 0;
};

class CountingReporter : public leveldb::log::Reader::Reporter {
 public:
  size_t dropped = 0;
  void Corruption(size_t bytes, const Status&) override { dropped += bytes; }
};

void write_kat(const std::string& dir) {
  using namespace leveldb::crc32c;
  FILE* f = open_out(dir, "kat.json", "w");
  std::fprintf(f, "{\n  \"generator\": \"oracle/gen_golden.cc (reference util/crc32c.cc)\",\n");
  std::fprintf(f, "  \"vectors\": [\n");
  struct V {
    std::string name;
    std::vector<uint8_t> data;
    uint32_t init;
  };
  std::vector<V> vs;
  vs.push_back({"rfc3720_zeros32", std::vector<uint8_t>(32, 0x00), 0});
  vs.push_back({"rfc3720_ones32", std::vector<uint8_t>(32, 0xff), 0});
  {
    std::vector<uint8_t> a(32), b(32);
    for (int i = 0; i < 32; ++i) {
      a[i] = static_cast<uint8_t>(i);
      b[i] = static_cast<uint8_t>(31 - i);
    }
    vs.push_back({"rfc3720_incr32", a, 0});
    vs.push_back({"rfc3720_decr32", b, 0});
  }
  {
    const uint8_t pdu[48] = {
        0x01, 0xc0, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
        0x00, 0x00, 0x00, 0x00, 0x14, 0x00, 0x00, 0x00, 0x00, 0x00, 0x04, 0x00,
        0x00, 0x00, 0x00, 0x14, 0x00, 0x00, 0x00, 0x18, 0x28, 0x00, 0x00, 0x00,
        0x00, 0x00, 0x00, 0x00, 0x02, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00};
    vs.push_back({"rfc3720_iscsi_pdu48", std::vector<uint8_t>(pdu, pdu + 48), 0});
  }
  auto str = [](const char* s) {
    return std::vector<uint8_t>(s, s + std::strlen(s));
  };
  vs.push_back({"self_test_TestCRCBuffer", str("TestCRCBuffer"), 0});
  vs.push_back({"check_123456789", str("123456789"), 0});
  vs.push_back({"a", str("a"), 0});
  vs.push_back({"foo", str("foo"), 0});
  vs.push_back({"hello_world", str("hello world"), 0});
  vs.push_back({"extend_world_after_hello_", str("world"),
                Value("hello ", 6)});
  vs.push_back({"empty", {}, 0});
  vs.push_back({"empty_init", {}, 0x12345678u});
  for (size_t i = 0; i < vs.size(); ++i) {
    const V& v = vs[i];
    uint32_t c = Extend(v.init, reinterpret_cast<const char*>(v.data.data()),
                        v.data.size());
    std::fprintf(f,
                 "    {\"name\": \"%s\", \"hex\": \"%s\", \"init\": %" PRIu32
                 ", \"crc\": %" PRIu32 ", \"masked\": %" PRIu32 "}%s\n",
                 v.name.c_str(), hex(v.data.data(), v.data.size()).c_str(),
                 v.init, c, Mask(c), i + 1 < vs.size() ? "," : "");
  }
  std::fprintf(f, "  ],\n");
  uint32_t foo = Value("foo", 3);
  std::fprintf(f,
               "  \"mask\": {\"crc\": %" PRIu32 ", \"mask1\": %" PRIu32
               ", \"mask2\": %" PRIu32 ", \"unmask_of_crc\": %" PRIu32 "},\n",
               foo, Mask(foo), Mask(Mask(foo)), Unmask(foo));
  std::fprintf(f, "  \"mask_delta\": %" PRIu32 "\n}\n", kMaskDelta);
  std::fclose(f);
}

void write_corpus(const std::string& dir) {
  const uint64_t seed = 0x1EDC6F41ull;
  const size_t nbuf = 40 * 1024;
  std::vector<uint8_t> buf = splitmix_bytes(seed, nbuf);
  const size_t lens[] = {0,  1,   2,   3,   4,    5,    6,    7,    8,
                         9,  10,  11,  12,  13,   14,   15,   16,   17,
                         31, 32,  63,  64,  65,   255,  256,  257,  4095,
                         4096, 4097, 4101, 4105, 4106, 32761, 32762, 32768};
  const uint32_t inits[] = {0u, 0xffffffffu, 0x12345678u};
  FILE* f = open_out(dir, "corpus.json", "w");
  std::fprintf(f,
               "{\n  \"generator\": \"oracle/gen_golden.cc (reference util/crc32c.cc)\",\n"
               "  \"prng\": \"splitmix64\", \"seed\": %" PRIu64
               ", \"buffer_bytes\": %zu,\n  \"entries\": [\n",
               seed, nbuf);
  bool first = true;
  for (size_t len : lens)
    for (size_t off = 0; off < 4; ++off)
      for (uint32_t init : inits) {
        uint32_t c = leveldb::crc32c::Extend(
            init, reinterpret_cast<const char*>(buf.data() + off), len);
        std::fprintf(f, "%s    [%zu, %zu, %" PRIu32 ", %" PRIu32 "]",
                     first ? "" : ",\n", len, off, init, c);
        first = false;
      }
  std::fprintf(f, "\n  ]\n}\n");
  std::fclose(f);
}

void write_blocks1000(const std::string& dir) {
  const uint64_t seed = 0x1EDC6F41ull + 2;  // BASELINE config id 2
  const size_t n = 1000, len = 4096;
  std::vector<uint8_t> buf = splitmix_bytes(seed, n * len);
  FILE* f = open_out(dir, "blocks1000_crc.bin", "wb");
  for (size_t i = 0; i < n; ++i) {
    uint32_t c = leveldb::crc32c::Value(
        reinterpret_cast<const char*>(buf.data() + i * len), len);
    uint8_t le[4];
    leveldb::EncodeFixed32(reinterpret_cast<char*>(le), c);
    std::fwrite(le, 1, 4, f);
  }
  std::fclose(f);
}

void write_sst(const std::string& dir) {
  leveldb::Options opt;
  opt.compression = leveldb::kNoCompression;
  opt.block_size = 4096;
  const leveldb::FilterPolicy* bloom = leveldb::NewBloomFilterPolicy(10);
  opt.filter_policy = bloom;
  RecordingSink sink;
  leveldb::TableBuilder tb(opt, &sink);
  uint64_t st = 0x5357ull;  // "SW"
  char key[32];
  for (int i = 0; i < 1400; ++i) {
    std::snprintf(key, sizeof(key), "key%08d", i);
    size_t vlen = 16 + splitmix_next(&st) % 240;
    std::vector<uint8_t> v = splitmix_bytes(splitmix_next(&st), vlen);
    tb.Add(key, Slice(reinterpret_cast<const char*>(v.data()), v.size()));
  }
  Status s = tb.Finish();
  if (!s.ok()) {
    std::fprintf(stderr, "TableBuilder: %s\n", s.ToString().c_str());
    std::exit(1);
  }
  delete bloom;

  FILE* f = open_out(dir, "table.sst", "wb");
  std::fwrite(sink.contents.data(), 1, sink.contents.size(), f);
  std::fclose(f);

  // Pair up [contents, trailer(5)] appends; the last append is the footer.
  StringRandomAccess raf(&sink.contents);
  FILE* j = open_out(dir, "table_blocks.json", "w");
  std::fprintf(j,
               "{\n  \"generator\": \"oracle/gen_golden.cc (reference "
               "TableBuilder + ReadBlock)\",\n  \"file_bytes\": %zu,\n"
               "  \"blocks\": [\n",
               sink.contents.size());
  uint64_t off = 0;
  size_t nb = 0;
  for (size_t k = 0; k + 1 < sink.appends.size(); k += 2) {
    size_t n = sink.appends[k];
    if (sink.appends[k + 1] != leveldb::kBlockTrailerSize) break;
    const char* trailer = sink.contents.data() + off + n;
    uint8_t type = static_cast<uint8_t>(trailer[0]);
    uint32_t masked = leveldb::DecodeFixed32(trailer + 1);
    uint32_t crc = leveldb::crc32c::Value(sink.contents.data() + off, n + 1);
    // Re-verify through the reference read path (table/format.cc:69-100).
    leveldb::BlockHandle h;
    h.set_offset(off);
    h.set_size(n);
    leveldb::ReadOptions ro;
    ro.verify_checksums = true;
    leveldb::BlockContents bc;
    Status rs = leveldb::ReadBlock(&raf, ro, h, &bc);
    if (!rs.ok()) {
      std::fprintf(stderr, "ReadBlock failed at %" PRIu64 ": %s\n", off,
                   rs.ToString().c_str());
      std::exit(1);
    }
    if (bc.heap_allocated) delete[] bc.data.data();
    std::fprintf(j,
                 "%s    {\"offset\": %" PRIu64 ", \"size\": %zu, \"type\": %u, "
                 "\"masked_crc\": %" PRIu32 ", \"crc\": %" PRIu32 "}",
                 nb ? ",\n" : "", off, n, type, masked, crc);
    off += n + leveldb::kBlockTrailerSize;
    ++nb;
  }
  std::fprintf(j, "\n  ],\n  \"footer_offset\": %" PRIu64 "\n}\n", off);
  std::fclose(j);
}

void write_wal(const std::string& dir) {
  StringSink sink;
  leveldb::log::Writer w(&sink);
  const size_t sizes[] = {0,     1,    7,     100, 1000, 4096, 32761 - 7,
                          70000, 10,   20000, 3,   0,    32768, 500};
  uint64_t seed = 0x57414cull;  // "WAL"
  std::vector<std::string> logical;
  for (size_t n : sizes) {
    std::vector<uint8_t> p = splitmix_bytes(seed++, n);
    std::string rec(reinterpret_cast<const char*>(p.data()), p.size());
    logical.push_back(rec);
    Status s = w.AddRecord(rec);
    if (!s.ok()) std::exit(1);
  }
  FILE* f = open_out(dir, "wal.log", "wb");
  std::fwrite(sink.contents.data(), 1, sink.contents.size(), f);
  std::fclose(f);

  // Read back through the reference reader with checksums on
  // (db/log_reader.cc:189-271).
  StringSequential src(&sink.contents);
  CountingReporter rep;
  leveldb::log::Reader r(&src, &rep, /*checksum=*/true, 0);
  Slice rec;
  std::string scratch;
  size_t got = 0;
  while (r.ReadRecord(&rec, &scratch)) {
    if (got >= logical.size() || rec.ToString() != logical[got]) {
      std::fprintf(stderr, "log reader mismatch at record %zu\n", got);
      std::exit(1);
    }
    ++got;
  }
  if (got != logical.size() || rep.dropped != 0) {
    std::fprintf(stderr, "log reader: %zu/%zu records, %zu dropped\n", got,
                 logical.size(), rep.dropped);
    std::exit(1);
  }

  // Enumerate the physical records (db/log_format.h, doc/log_format.md).
  FILE* j = open_out(dir, "wal_records.json", "w");
  std::fprintf(j,
               "{\n  \"generator\": \"oracle/gen_golden.cc (reference "
               "log::Writer + log::Reader)\",\n  \"file_bytes\": %zu,\n"
               "  \"logical_records\": %zu,\n  \"records\": [\n",
               sink.contents.size(), logical.size());
  const std::string& c = sink.contents;
  size_t pos = 0, nrec = 0;
  while (pos < c.size()) {
    size_t in_block = pos % leveldb::log::kBlockSize;
    if (leveldb::log::kBlockSize - in_block < leveldb::log::kHeaderSize) {
      pos += leveldb::log::kBlockSize - in_block;
      continue;
    }
    const char* h = c.data() + pos;
    uint32_t masked = leveldb::DecodeFixed32(h);
    uint32_t len = static_cast<uint8_t>(h[4]) |
                   (static_cast<uint32_t>(static_cast<uint8_t>(h[5])) << 8);
    uint32_t type = static_cast<uint8_t>(h[6]);
    uint32_t crc = leveldb::crc32c::Value(h + 6, 1 + len);
    std::fprintf(j,
                 "%s    {\"offset\": %zu, \"length\": %" PRIu32
                 ", \"type\": %" PRIu32 ", \"masked_crc\": %" PRIu32
                 ", \"crc\": %" PRIu32 "}",
                 nrec ? ",\n" : "", pos, len, type, masked, crc);
    pos += leveldb::log::kHeaderSize + len;
    ++nrec;
  }
  std::fprintf(j, "\n  ]\n}\n");
  std::fclose(j);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 2) {
    std::fprintf(stderr, "usage: %s OUTDIR\n", argv[0]);
    return 2;
  }
  std::string dir = argv[1];
  write_kat(dir);
  write_corpus(dir);
  write_blocks1000(dir);
  write_sst(dir);
  write_wal(dir);
  std::printf("golden fixtures written to %s\n", dir.c_str());
  return 0;
}
