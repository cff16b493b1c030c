// TEST INFRASTRUCTURE ONLY — damaged-image verdicts from the reference itself.
//
// Built by `make -C oracle damage` against the reference sources where they
// lie under /root/reference (never copied). It takes the reference-written
// golden images (tests/golden/table.sst, wal.log), applies seeded damage
// patterns, and records what the reference's OWN readers report, so the
// device verify paths (lvkv_sst_verify_table(s)_device,
// lvkv_log_verify_blocks_device) are pinned to the reference, not to a
// Python restatement:
//
//   damage_sst.json  per case: the patches, then
//     * Table::Open(paranoid_checks = true) status (table/table.cc:38-79);
//     * Footer::DecodeFrom + ReadBlock(index, verify_checksums) (format.cc);
//     * every index entry through Block::Iter (table/block.cc) +
//       BlockHandle::DecodeFrom + ReadBlock(verify_checksums): per-entry
//       handle and status string, then the index iterator's status;
//     * Table::ReadMeta's steps (table.cc:81-105): metaindex ReadBlock, the
//       exact Seek("filter." + policy->Name()), ReadFilter's ReadBlock.
//   damage_wal.json  per case: the patches / truncation, then every
//     Reporter::Corruption(bytes, status) of log::Reader(checksum = true,
//     the case's initial_offset) (db/log_reader.cc) and every returned record
//     (LastRecordOffset, length, CRC32C of the contents).
//   sst_alt_filter.sst / sst_two_filters.sst  small tables whose metaindex
//     holds a filter key of another policy name, and two "filter." keys.
#include <algorithm>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "db/log_format.h"
#include "db/log_reader.h"
#include "leveldb/comparator.h"
#include "leveldb/env.h"
#include "leveldb/filter_policy.h"
#include "leveldb/iterator.h"
#include "leveldb/options.h"
#include "leveldb/table.h"
#include "leveldb/table_builder.h"
#include "table/block.h"
#include "table/block_builder.h"
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

std::string hex(const std::string& s) {
  static const char* d = "0123456789abcdef";
  std::string o;
  for (unsigned char c : s) {
    o.push_back(d[c >> 4]);
    o.push_back(d[c & 15]);
  }
  return o;
}

std::string esc(const std::string& s) {  // JSON string body
  std::string o;
  for (char c : s) {
    if (c == '"' || c == '\\') o.push_back('\\');
    o.push_back(c);
  }
  return o;
}

std::string read_file(const std::string& path) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) {
    std::perror(path.c_str());
    std::exit(1);
  }
  std::string s;
  char buf[65536];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) s.append(buf, n);
  std::fclose(f);
  return s;
}

void write_file(const std::string& path, const std::string& s) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) {
    std::perror(path.c_str());
    std::exit(1);
  }
  std::fwrite(s.data(), 1, s.size(), f);
  std::fclose(f);
}

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

class StringRandomAccess : public leveldb::RandomAccessFile {
 public:
  explicit StringRandomAccess(const std::string* s) : s_(s) {}
  Status Read(uint64_t offset, size_t n, Slice* result, char* scratch) const override {
    if (offset > s_->size()) {
      *result = Slice(scratch, 0);
      return Status::OK();  // a short read: ReadBlock reports "truncated block read"
    }
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

// A filter policy that only carries a name (the metaindex key is
// "filter." + Name(), table_builder.cc:228-231; table.cc:100-101).
class NamedPolicy : public leveldb::FilterPolicy {
 public:
  explicit NamedPolicy(std::string name) : name_(std::move(name)) {}
  const char* Name() const override { return name_.c_str(); }
  void CreateFilter(const Slice*, int n, std::string* dst) const override {
    dst->append(static_cast<size_t>(n % 7 + 3), 'f');
  }
  bool KeyMayMatch(const Slice&, const Slice&) const override { return true; }

 private:
  std::string name_;
};

struct Patch {
  uint64_t off;
  std::string bytes;
};

std::string apply(const std::string& base, const std::vector<Patch>& ps, size_t truncate_to) {
  std::string s = base;
  for (const Patch& p : ps)
    for (size_t i = 0; i < p.bytes.size() && p.off + i < s.size(); ++i) s[p.off + i] = p.bytes[i];
  if (truncate_to < s.size()) s.resize(truncate_to);
  return s;
}

std::string st(const Status& s) { return s.ok() ? "OK" : s.ToString(); }

// ---- SST ---------------------------------------------------------------

struct BlockRef {
  uint64_t off, size;
};

// The golden table's layout through the reference's own decoders.
void layout(const std::string& img, BlockRef* meta, BlockRef* index, std::vector<BlockRef>* data) {
  leveldb::Footer footer;
  Slice in(img.data() + img.size() - leveldb::Footer::kEncodedLength,
           leveldb::Footer::kEncodedLength);
  if (!footer.DecodeFrom(&in).ok()) std::exit(1);
  *meta = {footer.metaindex_handle().offset(), footer.metaindex_handle().size()};
  *index = {footer.index_handle().offset(), footer.index_handle().size()};
  StringRandomAccess raf(&img);
  leveldb::ReadOptions ro;
  ro.verify_checksums = true;
  leveldb::BlockContents bc;
  if (!leveldb::ReadBlock(&raf, ro, footer.index_handle(), &bc).ok()) std::exit(1);
  leveldb::Block b(bc);
  leveldb::Iterator* it = b.NewIterator(leveldb::BytewiseComparator());
  for (it->SeekToFirst(); it->Valid(); it->Next()) {
    leveldb::BlockHandle h;
    Slice v = it->value();
    if (!h.DecodeFrom(&v).ok()) std::exit(1);
    data->push_back({h.offset(), h.size()});
  }
  delete it;
}

// Masked CRC of [off, off + n] (contents + type) as WriteRawBlock stores it.
std::string fixed_crc(const std::string& img, uint64_t off, uint64_t n) {
  char buf[4];
  leveldb::EncodeFixed32(buf, leveldb::crc32c::Mask(leveldb::crc32c::Value(img.data() + off, n + 1)));
  return std::string(buf, 4);
}

void run_sst_case(FILE* j, bool first, const std::string& name, const std::string& base_name,
                  const std::string& base, const std::vector<Patch>& ps, size_t truncate_to,
                  const char* policy_name) {
  const std::string img = apply(base, ps, truncate_to);
  std::fprintf(j, "%s    {\"name\": \"%s\", \"base\": \"%s\", \"truncate_to\": %zu, \"patches\": [",
               first ? "" : ",\n", name.c_str(), base_name.c_str(),
               truncate_to < base.size() ? truncate_to : base.size());
  for (size_t i = 0; i < ps.size(); ++i)
    std::fprintf(j, "%s[%" PRIu64 ", \"%s\"]", i ? ", " : "", ps[i].off, hex(ps[i].bytes).c_str());
  std::fprintf(j, "], \"filter_policy\": %s%s%s", policy_name ? "\"" : "",
               policy_name ? policy_name : "null", policy_name ? "\"" : "");

  StringRandomAccess raf(&img);
  NamedPolicy* pol = policy_name ? new NamedPolicy(policy_name) : nullptr;
  leveldb::Options opt;
  opt.paranoid_checks = true;
  opt.filter_policy = pol;
  leveldb::Table* table = nullptr;
  Status os = leveldb::Table::Open(opt, &raf, img.size(), &table);
  std::fprintf(j, ", \"open\": \"%s\"", esc(st(os)).c_str());
  delete table;

  // The same steps, observable one by one.
  leveldb::ReadOptions ro;
  ro.verify_checksums = true;
  Status fs = img.size() < leveldb::Footer::kEncodedLength
                  ? Status::Corruption("file is too short to be an sstable")
                  : Status::OK();
  leveldb::Footer footer;
  if (fs.ok()) {
    Slice in(img.data() + img.size() - leveldb::Footer::kEncodedLength,
             leveldb::Footer::kEncodedLength);
    fs = footer.DecodeFrom(&in);
  }
  std::fprintf(j, ", \"footer\": \"%s\"", esc(st(fs)).c_str());
  if (fs.ok()) {
    leveldb::BlockContents ic;
    Status is = leveldb::ReadBlock(&raf, ro, footer.index_handle(), &ic);
    std::fprintf(j, ", \"index\": \"%s\", \"entries\": [", esc(st(is)).c_str());
    if (is.ok()) {
      leveldb::Block ib(ic);
      leveldb::Iterator* it = ib.NewIterator(leveldb::BytewiseComparator());
      bool f1 = true;
      for (it->SeekToFirst(); it->Valid(); it->Next()) {
        leveldb::BlockHandle h;
        Slice v = it->value();
        Status hs = h.DecodeFrom(&v);
        std::string bs;
        uint64_t off = 0, size = 0;
        if (!hs.ok()) {
          bs = st(hs);
        } else {
          off = h.offset();
          size = h.size();
          leveldb::BlockContents c;
          Status rs = leveldb::ReadBlock(&raf, ro, h, &c);
          if (rs.ok() && c.heap_allocated) delete[] c.data.data();
          bs = st(rs);
        }
        std::fprintf(j, "%s[%" PRIu64 ", %" PRIu64 ", \"%s\"]", f1 ? "" : ", ", off, size,
                     esc(bs).c_str());
        f1 = false;
      }
      std::fprintf(j, "], \"index_iter\": \"%s\"", esc(st(it->status())).c_str());
      delete it;
    } else {
      std::fprintf(j, "]");
    }
    // Table::ReadMeta (table.cc:81-105) and ReadFilter (:107-124).
    leveldb::BlockContents mc;
    Status ms = leveldb::ReadBlock(&raf, ro, footer.metaindex_handle(), &mc);
    std::fprintf(j, ", \"meta\": \"%s\"", esc(st(ms)).c_str());
    bool found = false;
    if (ms.ok() && pol) {
      leveldb::Block mb(mc);
      leveldb::Iterator* it = mb.NewIterator(leveldb::BytewiseComparator());
      std::string key = "filter.";
      key.append(pol->Name());
      it->Seek(key);
      if (it->Valid() && it->key() == Slice(key)) {
        found = true;
        leveldb::BlockHandle h;
        Slice v = it->value();
        Status hs = h.DecodeFrom(&v);
        std::string fst;
        if (!hs.ok()) {
          fst = st(hs);
        } else {
          leveldb::BlockContents c;
          Status rs = leveldb::ReadBlock(&raf, ro, h, &c);
          if (rs.ok() && c.heap_allocated) delete[] c.data.data();
          fst = st(rs);
        }
        std::fprintf(j, ", \"filter\": [%" PRIu64 ", %" PRIu64 ", \"%s\"]",
                     hs.ok() ? h.offset() : 0, hs.ok() ? h.size() : 0, esc(fst).c_str());
      }
      delete it;
    } else if (ms.ok() && mc.heap_allocated) {
      delete[] mc.data.data();
    }
    std::fprintf(j, ", \"filter_found\": %s", found ? "true" : "false");
  }
  std::fprintf(j, "}");
  delete pol;
}

std::string byte_at(const std::string& img, uint64_t off, int xorv) {
  return std::string(1, static_cast<char>(static_cast<unsigned char>(img[off]) ^ xorv));
}

void write_sst_cases(const std::string& dir) {
  const std::string base = read_file(dir + "/table.sst");
  BlockRef meta, index;
  std::vector<BlockRef> data;
  layout(base, &meta, &index, &data);
  const char* bloom = "leveldb.BuiltinBloomFilter2";
  FILE* j = std::fopen((dir + "/damage_sst.json").c_str(), "w");
  std::fprintf(j, "{\n  \"generator\": \"oracle/gen_damage.cc (reference Table::Open, ReadBlock, "
                  "Block::Iter, ReadMeta steps)\",\n  \"cases\": [\n");
  bool first = true;
  auto add = [&](const std::string& name, const std::vector<Patch>& ps, size_t trunc = SIZE_MAX,
                 const char* pol = "leveldb.BuiltinBloomFilter2",
                 const std::string& base_name = "table.sst", const std::string* img = nullptr) {
    run_sst_case(j, first, name, base_name, img ? *img : base, ps, trunc, pol);
    first = false;
  };
  const BlockRef& d0 = data[0];
  const BlockRef& dm = data[data.size() / 2];
  const BlockRef& dl = data.back();
  add("pristine", {});
  add("pristine_no_policy", {}, SIZE_MAX, nullptr);
  add("data_contents_flip", {{dm.off + dm.size / 3, byte_at(base, dm.off + dm.size / 3, 0x40)}});
  add("data_first_byte_flip", {{d0.off, byte_at(base, d0.off, 1)}});
  add("data_last_contents_flip", {{dl.off + dl.size - 1, byte_at(base, dl.off + dl.size - 1, 0x80)}});
  add("data_type_flip", {{dm.off + dm.size, byte_at(base, dm.off + dm.size, 1)}});
  add("data_crc_flip", {{dm.off + dm.size + 2, byte_at(base, dm.off + dm.size + 2, 0x10)}});
  // Type bytes whose CRC is fixed up: the CRC passes, the type decides.
  for (int t : {1, 2, 3, 0x80}) {
    std::string img = base;
    img[dm.off + dm.size] = static_cast<char>(t);
    add("data_type_" + std::to_string(t) + "_crc_fixed",
        {{dm.off + dm.size, std::string(1, static_cast<char>(t))},
         {dm.off + dm.size + 1, fixed_crc(img, dm.off, dm.size)}});
  }
  add("index_contents_flip", {{index.off + 5, byte_at(base, index.off + 5, 4)}});
  add("index_crc_flip", {{index.off + index.size + 1, byte_at(base, index.off + index.size + 1, 1)}});
  {
    std::string img = base;
    img[index.off + index.size] = 1;
    add("index_type_1_crc_fixed", {{index.off + index.size, std::string(1, '\1')},
                                   {index.off + index.size + 1, fixed_crc(img, index.off, index.size)}});
  }
  {
    // restart count larger than the block: Block's size_ = 0 (block.cc:28-37)
    std::string img = base;
    leveldb::EncodeFixed32(&img[index.off + index.size - 4], 0x00ffffffu);
    add("index_restart_count_crc_fixed",
        {{index.off + index.size - 4, img.substr(index.off + index.size - 4, 4)},
         {index.off + index.size + 1, fixed_crc(img, index.off, index.size)}});
  }
  add("meta_contents_flip", {{meta.off + 2, byte_at(base, meta.off + 2, 8)}});
  add("meta_crc_flip", {{meta.off + meta.size + 3, byte_at(base, meta.off + meta.size + 3, 1)}});
  add("filter_policy_other_name", {}, SIZE_MAX, "leveldb.BuiltinBloomFilter");
  add("filter_policy_longer_name", {}, SIZE_MAX, "leveldb.BuiltinBloomFilter2x");
  {
    // filter block: the one block after the data blocks (table_builder.cc:218-226)
    const uint64_t foff = dl.off + dl.size + leveldb::kBlockTrailerSize;
    add("filter_contents_flip", {{foff + 1, byte_at(base, foff + 1, 2)}});
  }
  add("footer_magic_flip", {{base.size() - 3, byte_at(base, base.size() - 3, 1)}});
  add("footer_handle_varint_bad",
      {{base.size() - leveldb::Footer::kEncodedLength, std::string(10, '\xff')}});
  add("truncated_to_47", {}, 47);
  add("truncated_tail", {}, base.size() - 100);
  {
    // A footer whose index handle has size 2^64-1 (ff x 9, 01): must be a
    // "truncated block read", never an overflow.
    std::string enc;
    leveldb::PutVarint64(&enc, meta.off);
    leveldb::PutVarint64(&enc, meta.size);
    leveldb::PutVarint64(&enc, index.off);
    leveldb::PutVarint64(&enc, ~uint64_t{0});
    enc.resize(2 * leveldb::BlockHandle::kMaxEncodedLength, '\0');
    add("footer_index_size_max", {{base.size() - leveldb::Footer::kEncodedLength, enc}});
    std::string enc2;
    leveldb::PutVarint64(&enc2, meta.off);
    leveldb::PutVarint64(&enc2, ~uint64_t{0});
    leveldb::PutVarint64(&enc2, index.off);
    leveldb::PutVarint64(&enc2, index.size);
    enc2.resize(2 * leveldb::BlockHandle::kMaxEncodedLength, '\0');
    add("footer_meta_size_max", {{base.size() - leveldb::Footer::kEncodedLength, enc2}});
  }
  // Seeded random single- and multi-byte damage anywhere in the file.
  uint64_t rs = 0xDA4A6Eull;
  for (int c = 0; c < 24; ++c) {
    std::vector<Patch> ps;
    const int nflip = 1 + static_cast<int>(splitmix_next(&rs) % 3);
    for (int k = 0; k < nflip; ++k) {
      const uint64_t off = splitmix_next(&rs) % base.size();
      const int x = 1 + static_cast<int>(splitmix_next(&rs) % 255);
      ps.push_back({off, byte_at(base, off, x)});
    }
    add("random_" + std::to_string(c), ps);
  }

  // Tables built here: a metaindex with another policy's filter key, and one
  // with two "filter." keys (the exact one second).
  {
    leveldb::Options o;
    o.compression = leveldb::kNoCompression;
    o.block_size = 1024;
    NamedPolicy other("test.OtherFilter");
    o.filter_policy = &other;
    StringSink sink;
    leveldb::TableBuilder tb(o, &sink);
    char key[32];
    for (int i = 0; i < 60; ++i) {
      std::snprintf(key, sizeof(key), "alt%06d", i);
      tb.Add(key, std::string(40 + i % 13, static_cast<char>('a' + i % 26)));
    }
    if (!tb.Finish().ok()) std::exit(1);
    write_file(dir + "/sst_alt_filter.sst", sink.contents);
    add("alt_filter_bloom_policy", {}, SIZE_MAX, bloom, "sst_alt_filter.sst", &sink.contents);
    add("alt_filter_own_policy", {}, SIZE_MAX, "test.OtherFilter", "sst_alt_filter.sst",
        &sink.contents);
  }
  {
    // Rebuild the golden table's metaindex with two entries, "filter.aaa"
    // -> the filter block and "filter.<bloom>" -> the filter block, written
    // after the footer's old position; new footer (table_builder.cc:228-268).
    std::string img = base.substr(0, base.size() - leveldb::Footer::kEncodedLength);
    leveldb::BlockBuilder mb(new leveldb::Options());
    const uint64_t foff = dl.off + dl.size + leveldb::kBlockTrailerSize;
    const uint64_t fsize = meta.off - leveldb::kBlockTrailerSize - foff;
    leveldb::BlockHandle fh;
    fh.set_offset(foff);
    fh.set_size(fsize);
    std::string hv;
    fh.EncodeTo(&hv);
    mb.Add("filter.aaa", hv);
    mb.Add(std::string("filter.") + bloom, hv);
    Slice raw = mb.Finish();
    leveldb::BlockHandle mh;
    mh.set_offset(img.size());
    mh.set_size(raw.size());
    img.append(raw.data(), raw.size());
    char trailer[leveldb::kBlockTrailerSize];
    trailer[0] = leveldb::kNoCompression;
    uint32_t crc = leveldb::crc32c::Value(raw.data(), raw.size());
    crc = leveldb::crc32c::Extend(crc, trailer, 1);
    leveldb::EncodeFixed32(trailer + 1, leveldb::crc32c::Mask(crc));
    img.append(trailer, leveldb::kBlockTrailerSize);
    leveldb::Footer ft;
    ft.set_metaindex_handle(mh);
    leveldb::BlockHandle ih;
    ih.set_offset(index.off);
    ih.set_size(index.size);
    ft.set_index_handle(ih);
    std::string fenc;
    ft.EncodeTo(&fenc);
    img.append(fenc);
    write_file(dir + "/sst_two_filters.sst", img);
    add("two_filter_keys_bloom", {}, SIZE_MAX, bloom, "sst_two_filters.sst", &img);
    add("two_filter_keys_aaa", {}, SIZE_MAX, "aaa", "sst_two_filters.sst", &img);
    add("two_filter_keys_none_match", {}, SIZE_MAX, "zzz", "sst_two_filters.sst", &img);
  }
  std::fprintf(j, "\n  ]\n}\n");
  std::fclose(j);
}

// ---- WAL ---------------------------------------------------------------

class RecordingReporter : public leveldb::log::Reader::Reporter {
 public:
  std::vector<std::pair<size_t, std::string>> reports;
  void Corruption(size_t bytes, const Status& s) override { reports.push_back({bytes, st(s)}); }
};

void run_wal_case(FILE* j, bool first, const std::string& name, const std::string& base,
                  const std::vector<Patch>& ps, size_t truncate_to, uint64_t initial_offset) {
  const std::string img = apply(base, ps, truncate_to);
  std::fprintf(j,
               "%s    {\"name\": \"%s\", \"truncate_to\": %zu, \"initial_offset\": %" PRIu64
               ", \"patches\": [",
               first ? "" : ",\n", name.c_str(),
               truncate_to < base.size() ? truncate_to : base.size(), initial_offset);
  for (size_t i = 0; i < ps.size(); ++i)
    std::fprintf(j, "%s[%" PRIu64 ", \"%s\"]", i ? ", " : "", ps[i].off, hex(ps[i].bytes).c_str());
  StringSequential src(&img);
  RecordingReporter rep;
  leveldb::log::Reader r(&src, &rep, /*checksum=*/true, initial_offset);
  Slice rec;
  std::string scratch;
  std::fprintf(j, "], \"records\": [");
  bool f1 = true;
  while (r.ReadRecord(&rec, &scratch)) {
    std::fprintf(j, "%s[%" PRIu64 ", %zu, %" PRIu32 "]", f1 ? "" : ", ", r.LastRecordOffset(),
                 rec.size(), leveldb::crc32c::Value(rec.data(), rec.size()));
    f1 = false;
  }
  std::fprintf(j, "], \"reports\": [");
  for (size_t i = 0; i < rep.reports.size(); ++i)
    std::fprintf(j, "%s[%zu, \"%s\"]", i ? ", " : "", rep.reports[i].first,
                 esc(rep.reports[i].second).c_str());
  std::fprintf(j, "]}");
}

void write_wal_cases(const std::string& dir) {
  const std::string base = read_file(dir + "/wal.log");
  // physical record headers of the golden log (log_format.h)
  std::vector<uint64_t> hdrs;
  for (size_t pos = 0; pos < base.size();) {
    const size_t in_block = pos % leveldb::log::kBlockSize;
    if (leveldb::log::kBlockSize - in_block < leveldb::log::kHeaderSize) {
      pos += leveldb::log::kBlockSize - in_block;
      continue;
    }
    hdrs.push_back(pos);
    const uint32_t len = static_cast<uint8_t>(base[pos + 4]) |
                         (static_cast<uint32_t>(static_cast<uint8_t>(base[pos + 5])) << 8);
    pos += leveldb::log::kHeaderSize + len;
  }
  FILE* j = std::fopen((dir + "/damage_wal.json").c_str(), "w");
  std::fprintf(j, "{\n  \"generator\": \"oracle/gen_damage.cc (reference log::Reader, "
                  "checksum = true, recording Reporter)\",\n  \"physical_headers\": %zu,\n"
                  "  \"cases\": [\n",
               hdrs.size());
  bool first = true;
  auto add = [&](const std::string& name, const std::vector<Patch>& ps, size_t trunc = SIZE_MAX,
                 uint64_t initial = 0) {
    run_wal_case(j, first, name, base, ps, trunc, initial);
    first = false;
  };
  auto flip = [&](uint64_t off, int x) { return Patch{off, byte_at(base, off, x)}; };
  add("pristine", {});
  for (size_t k : {size_t{0}, size_t{3}, hdrs.size() / 2, hdrs.size() - 1}) {
    const uint64_t h = hdrs[k];
    add("payload_flip_" + std::to_string(k), {flip(h + 7, 1)});
    add("crc_flip_" + std::to_string(k), {flip(h + 1, 0x20)});
    add("type_flip_" + std::to_string(k), {flip(h + 6, 2)});
    add("length_grow_" + std::to_string(k), {flip(h + 5, 0x40)});
  }
  // a zero-type zero-length header in the middle of a block (log_reader.cc:234-240)
  add("zero_record", {{hdrs[3], std::string(7, '\0')}});
  // bad record type with a fixed CRC: physical layer returns it, logical layer reports it
  {
    std::string img = base;
    const uint64_t h = hdrs[2];
    img[h + 6] = 9;
    const uint32_t len = static_cast<uint8_t>(img[h + 4]) |
                         (static_cast<uint32_t>(static_cast<uint8_t>(img[h + 5])) << 8);
    char c[4];
    leveldb::EncodeFixed32(c, leveldb::crc32c::Mask(leveldb::crc32c::Value(img.data() + h + 6, 1 + len)));
    add("unknown_type_crc_fixed", {{h + 6, std::string(1, '\x09')}, {h, std::string(c, 4)}});
  }
  // Every type byte 0..6 under a fixed CRC at a FULL record and at a FIRST,
  // MIDDLE and LAST fragment: the physical layer returns them all; the
  // logical layer (ReadRecord) sees kZeroType as unknown, 5 as kEof (stop)
  // and 6 as kBadRecord, and the fragment types start, continue or end the
  // record or report a missing start / partial record.
  {
    auto retype = [&](uint64_t h, int t) {
      std::string img = base;
      img[h + 6] = static_cast<char>(t);
      const uint32_t len = static_cast<uint8_t>(img[h + 4]) |
                           (static_cast<uint32_t>(static_cast<uint8_t>(img[h + 5])) << 8);
      char c[4];
      leveldb::EncodeFixed32(c,
                             leveldb::crc32c::Mask(leveldb::crc32c::Value(img.data() + h + 6, 1 + len)));
      return std::vector<Patch>{{h + 6, std::string(1, static_cast<char>(t))}, {h, std::string(c, 4)}};
    };
    const char* kind[] = {"zero", "full", "first", "middle", "last", "eof", "bad"};
    std::vector<std::pair<const char*, uint64_t>> at;
    for (int want : {1, 2, 3, 4}) {
      for (uint64_t h : hdrs) {
        if (static_cast<uint8_t>(base[h + 6]) == want) {
          at.push_back({kind[want], h});
          break;
        }
      }
    }
    for (const auto& [orig, h] : at)
      for (int t = 0; t <= 6; ++t)
        if (t != static_cast<uint8_t>(base[h + 6]))
          add(std::string("retype_") + orig + "_to_" + kind[t], retype(h, t));
  }
  add("truncated_mid_record", {}, hdrs[hdrs.size() - 2] + 20);
  add("truncated_mid_header", {}, hdrs.back() + 3);
  add("truncated_block_edge", {}, 32768 + 5);
  uint64_t rs = 0x1D4A6Eull;
  for (int c = 0; c < 24; ++c) {
    std::vector<Patch> ps;
    const int nflip = 1 + static_cast<int>(splitmix_next(&rs) % 3);
    for (int k = 0; k < nflip; ++k) {
      const uint64_t off = splitmix_next(&rs) % base.size();
      ps.push_back(flip(off, 1 + static_cast<int>(splitmix_next(&rs) % 255)));
    }
    add("random_" + std::to_string(c), ps);
  }
  // log::Reader's initial_offset (log_reader.cc:29-54, :80-89, :182-187,
  // :261-266): the skip to the first block that can hold the record, the
  // trailer rule, the resync over MIDDLE / LAST fragments at a block start,
  // silent physical records before the offset, and ReportDrop's filter.
  {
    const uint64_t kB = leveldb::log::kBlockSize;
    std::vector<uint64_t> offs = {1, kB - 7, kB - 6, kB - 5, kB, kB + 1, base.size(),
                                  base.size() + 1, base.size() + 3 * kB};
    for (size_t k = 0; k < hdrs.size(); ++k) {
      offs.push_back(hdrs[k]);
      offs.push_back(hdrs[k] + 1);
      if (hdrs[k] > 0) offs.push_back(hdrs[k] - 1);
    }
    for (uint64_t b = 2; b * kB < base.size(); ++b) {
      offs.push_back(b * kB);
      offs.push_back(b * kB - 6);
      offs.push_back(b * kB - 5);
    }
    std::sort(offs.begin(), offs.end());
    offs.erase(std::unique(offs.begin(), offs.end()), offs.end());
    for (uint64_t o : offs) add("offset_" + std::to_string(o), {}, SIZE_MAX, o);
    // damage on either side of the offset, in the block the reader starts in
    for (size_t k : {size_t{3}, size_t{4}, size_t{7}, size_t{9}, size_t{16}}) {
      const uint64_t h = hdrs[k];
      const std::string at = std::to_string(k);
      for (uint64_t o : {h, h + 1, h > 0 ? h - 1 : h + 2}) {
        const std::string sfx = "_" + at + "_from_" + std::to_string(o);
        add("offset_crc_flip" + sfx, {flip(h + 1, 0x20)}, SIZE_MAX, o);
        add("offset_length_grow" + sfx, {flip(h + 5, 0x40)}, SIZE_MAX, o);
      }
    }
    for (uint64_t o : {uint64_t{16}, uint64_t{30}, uint64_t{5247}}) {
      const std::string sfx = "_from_" + std::to_string(o);
      add("offset_zero_record" + sfx, {{hdrs[3], std::string(7, '\0')}}, SIZE_MAX, o);
      add("offset_crc_flip_2" + sfx, {flip(hdrs[2] + 1, 0x20)}, SIZE_MAX, o);
    }
    // retyped headers (CRC fixed) before, at and after the offset
    auto retyped = [&](uint64_t h, int t) {
      std::string img = base;
      img[h + 6] = static_cast<char>(t);
      const uint32_t len = static_cast<uint8_t>(img[h + 4]) |
                           (static_cast<uint32_t>(static_cast<uint8_t>(img[h + 5])) << 8);
      char c[4];
      leveldb::EncodeFixed32(c,
                             leveldb::crc32c::Mask(leveldb::crc32c::Value(img.data() + h + 6, 1 + len)));
      return std::vector<Patch>{{h + 6, std::string(1, static_cast<char>(t))}, {h, std::string(c, 4)}};
    };
    for (size_t k : {size_t{2}, size_t{7}, size_t{9}, size_t{10}, size_t{16}})
      for (int t : {0, 1, 2, 3, 4, 5, 6, 9})
        for (uint64_t o : {hdrs[k], hdrs[k] + 1}) {
          if (t == static_cast<uint8_t>(base[hdrs[k] + 6])) continue;
          add("offset_retype_" + std::to_string(k) + "_to_" + std::to_string(t) + "_from_" +
                  std::to_string(o),
              retyped(hdrs[k], t), SIZE_MAX, o);
        }
    add("offset_truncated_mid_record", {}, hdrs[hdrs.size() - 2] + 20, hdrs[hdrs.size() - 3] + 1);
    add("offset_truncated_block_edge", {}, kB + 5, kB);
  }
  std::fprintf(j, "\n  ]\n}\n");
  std::fclose(j);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 2) {
    std::fprintf(stderr, "usage: %s GOLDEN_DIR\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  write_sst_cases(dir);
  write_wal_cases(dir);
  std::printf("damage fixtures written to %s\n", dir.c_str());
  return 0;
}
