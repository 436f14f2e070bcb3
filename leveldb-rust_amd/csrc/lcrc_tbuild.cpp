// SSTable writer -- the reference's TableBuilder restated in C++ over this engine's CRCs (host side above the
// C ABI; the reference is Rust and there is no Rust toolchain in this image):
//   BlockBuilder::add / finish / current_size_estimate / reset  <- src/sstable/block.rs:296-377
//   TableBuilder::add / flush / finish                          <- src/sstable/table.rs:295-454
//     (index entries one block late with the shortest separator, table.rs:305-318; the index block restarts
//      at every entry, table.rs:272; the filter block written through write_raw_block with
//      options.compression_type as its type byte although its content is raw, table.rs:383-391)
//   write_block (Snappy frame kept iff < raw - raw/8)           <- src/sstable/table.rs:470-505
//   write_raw_block: content ++ [type][crc(content ++ type)]    <- src/sstable/table.rs:507-529
//   BlockHandle / Footer encode_to                              <- src/sstable/format.rs:51-54, 91-101
//   BitWiseComparator::find_shortest_separator / successor       <- src/util/cmp.rs:67-101
// Trailer CRCs either computed here, one per block as the reference does (seal on the host), or left zero with
// one {offset, n + 1, n + 1} descriptor per block (data, filter, metaindex, index) so that lcrc_batch_seal
// writes every trailer of the table in one device launch.
// Snappy: the `snap` crate's FrameEncoder is not in the image; frames are written in the
// published framing format (stream identifier, chunks of <= 64 KiB with the masked CRC-32C of the
// uncompressed bytes) with a greedy 4-byte-hash compressor -- valid for any Snappy decoder, byte-identical to
// the oracle's restatement, not to snap's own encoder output (parity with snap unpinned).
#include <stdint.h>
#include <string.h>

#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/lcrc.h"

namespace leveldb_gpu {

static void put_varint(std::vector<uint8_t>& out, uint64_t v) {
  while (v >= 128) {
    out.push_back((uint8_t)(v | 128));
    v >>= 7;
  }
  out.push_back((uint8_t)v);
}

static void put_le32(std::vector<uint8_t>& out, uint32_t v) {
  for (int i = 0; i < 4; ++i) out.push_back((uint8_t)(v >> (8 * i)));
}

// ---- BlockBuilder (block.rs:296-377) ----
class BlockBuilder {
 public:
  explicit BlockBuilder(int restart_interval) : interval_(restart_interval) { reset(); }
  void reset() {
    buf_.clear();
    restarts_.assign(1, 0);
    counter_ = 0;
    last_.clear();
  }
  void add(const uint8_t* key, size_t klen, const uint8_t* val, size_t vlen) {
    size_t shared = 0;
    if (counter_ < interval_) {
      const size_t m = last_.size() < klen ? last_.size() : klen;
      while (shared < m && last_[shared] == key[shared]) ++shared;
    } else {  // restart compression
      counter_ = 0;
      restarts_.push_back((uint32_t)buf_.size());
    }
    put_varint(buf_, shared);
    put_varint(buf_, klen - shared);
    put_varint(buf_, vlen);
    buf_.insert(buf_.end(), key + shared, key + klen);
    buf_.insert(buf_.end(), val, val + vlen);
    ++counter_;
    last_.assign(key, key + klen);
  }
  const std::vector<uint8_t>& finish() {
    for (uint32_t r : restarts_) put_le32(buf_, r);
    put_le32(buf_, (uint32_t)restarts_.size());
    return buf_;
  }
  size_t size_estimate() const { return buf_.size() + restarts_.size() * 4 + 4; }
  bool empty() const { return buf_.empty(); }

 private:
  int interval_;
  int counter_ = 0;
  std::vector<uint8_t> buf_;
  std::vector<uint32_t> restarts_;
  std::vector<uint8_t> last_;
};

// ---- Snappy raw format + framing (published formats; see the header comment) ----
static void snappy_literal(std::vector<uint8_t>& out, const uint8_t* d, size_t a, size_t b) {
  while (a < b) {
    const size_t n = b - a < 65536 ? b - a : 65536;
    if (n <= 60) {
      out.push_back((uint8_t)((n - 1) << 2));
    } else if (n <= 256) {
      out.push_back(60 << 2);
      out.push_back((uint8_t)(n - 1));
    } else {
      out.push_back(61 << 2);
      out.push_back((uint8_t)((n - 1) & 0xFF));
      out.push_back((uint8_t)((n - 1) >> 8));
    }
    out.insert(out.end(), d + a, d + a + n);
    a += n;
  }
}

static std::vector<uint8_t> snappy_compress_raw(const uint8_t* d, size_t n) {
  std::vector<uint8_t> out;
  put_varint(out, n);
  std::unordered_map<uint32_t, size_t> table;  // last position of each 4-byte string
  size_t i = 0, lit = 0;
  while (i + 4 <= n) {
    uint32_t k;
    memcpy(&k, d + i, 4);
    auto it = table.find(k);
    const bool hit = it != table.end() && i - it->second < 65536;
    const size_t j = hit ? it->second : 0;
    table[k] = i;
    if (hit) {
      size_t len = 4;
      while (i + len < n && d[j + len] == d[i + len] && len < 64) ++len;
      snappy_literal(out, d, lit, i);
      const size_t off = i - j;
      out.push_back((uint8_t)(((len - 1) << 2) | 2));
      out.push_back((uint8_t)(off & 0xFF));
      out.push_back((uint8_t)(off >> 8));
      i += len;
      lit = i;
    } else {
      ++i;
    }
  }
  snappy_literal(out, d, lit, n);
  return out;
}

static std::vector<uint8_t> snappy_frame_encode(const uint8_t* d, size_t n) {
  static const uint8_t kStream[10] = {0xff, 0x06, 0x00, 0x00, 's', 'N', 'a', 'P', 'p', 'Y'};
  std::vector<uint8_t> out(kStream, kStream + 10);
  for (size_t a = 0; a < n; a += 65536) {
    const size_t m = n - a < 65536 ? n - a : 65536;
    const uint32_t c = lcrc32c_mask(lcrc32c_value(d + a, m));
    std::vector<uint8_t> z = snappy_compress_raw(d + a, m);
    const bool keep = z.size() < m - m / 8;
    const size_t body = 4 + (keep ? z.size() : m);
    out.push_back(keep ? 0x00 : 0x01);
    out.push_back((uint8_t)(body & 0xFF));
    out.push_back((uint8_t)((body >> 8) & 0xFF));
    out.push_back((uint8_t)(body >> 16));
    put_le32(out, c);
    if (keep)
      out.insert(out.end(), z.begin(), z.end());
    else
      out.insert(out.end(), d + a, d + a + m);
  }
  return out;
}

// ---- comparator (util/cmp.rs:67-101) ----
static void find_shortest_separator(std::vector<uint8_t>& start, const uint8_t* limit, size_t llen) {
  const size_t m = start.size() < llen ? start.size() : llen;
  size_t i = 0;
  while (i < m && limit[i] == start[i]) ++i;
  if (i < m) {  // do not shorten if one is a prefix of the other
    const uint8_t b = start[i];
    if (b < 0xff && b + 1 < limit[i]) {
      start[i] = b + 1;
      start.resize(i + 1);
    }
  }
}

static void find_short_successor(std::vector<uint8_t>& key) {
  for (size_t i = 0; i < key.size(); ++i)
    if (key[i] != 0xff) {
      key[i] += 1;
      key.resize(i + 1);
      return;
    }
}

struct TableBlock {  // one block needing a trailer
  uint64_t offset, size;
  uint32_t crc;
  uint8_t kind, type;
};

// ---- TableBuilder (table.rs:242-454) ----
class TableBuilder {
 public:
  TableBuilder(uint32_t block_size, int restart_interval, uint8_t compression, int mode, uint32_t flags,
               bool host_seal)
      : block_size_(block_size), interval_(restart_interval), compression_(compression), mode_(mode),
        flags_(flags), host_seal_(host_seal), data_(restart_interval), index_(1) {}

  int add(const uint8_t* key, size_t klen, const uint8_t* val, size_t vlen) {
    if (closed_) return LCRC_EINVAL;
    if (num_entries_ > 0 && compare(key, klen, last_key_) <= 0) return LCRC_EINVAL;  // keys must increase
    if (pending_index_) {
      find_shortest_separator(last_key_, key, klen);
      add_index_entry();
    }
    last_key_.assign(key, key + klen);
    ++num_entries_;
    data_.add(key, klen, val, vlen);
    if (data_.size_estimate() >= block_size_) flush();
    return LCRC_OK;
  }

  void flush() {
    if (closed_ || data_.empty()) return;
    pending_handle_ = write_block(data_, LCRC_TBLK_DATA);
    pending_index_ = true;
  }

  // filter: the FilterBlockBuilder's finished content (the filter policy itself is outside the checksum
  // path); nullptr name = no filter policy
  int finish(const char* filter_name, const uint8_t* filter, size_t filter_len) {
    if (closed_) return LCRC_EINVAL;
    flush();
    closed_ = true;
    uint64_t fh_off = 0, fh_size = 0;
    if (filter_name) write_raw_block(filter, filter_len, compression_, LCRC_TBLK_FILTER, &fh_off, &fh_size);
    BlockBuilder meta(interval_);
    if (filter_name) {
      std::string key = std::string("filter") + filter_name;
      std::vector<uint8_t> h;
      put_varint(h, fh_off);
      put_varint(h, fh_size);
      meta.add((const uint8_t*)key.data(), key.size(), h.data(), h.size());
    }
    const std::pair<uint64_t, uint64_t> mh = write_block(meta, LCRC_TBLK_METAINDEX);
    if (pending_index_) {
      find_short_successor(last_key_);
      add_index_entry();
    }
    const std::pair<uint64_t, uint64_t> ih = write_block(index_, LCRC_TBLK_INDEX);
    std::vector<uint8_t> foot;
    put_varint(foot, mh.first);
    put_varint(foot, mh.second);
    put_varint(foot, ih.first);
    put_varint(foot, ih.second);
    foot.resize(40, 0);
    put_le32(foot, 0x8b80fb57u);  // TABLE_MAGIC_NUMBER 0xdb4775248b80fb57 (format.rs:19), low word first
    put_le32(foot, 0xdb477524u);
    file_.insert(file_.end(), foot.begin(), foot.end());
    return LCRC_OK;
  }

  const std::vector<uint8_t>& file() const { return file_; }
  const std::vector<TableBlock>& blocks() const { return blocks_; }

 private:
  static int compare(const uint8_t* a, size_t an, const std::vector<uint8_t>& b) {
    const size_t m = an < b.size() ? an : b.size();
    const int r = m ? memcmp(a, b.data(), m) : 0;
    if (r) return r;
    return an < b.size() ? -1 : an > b.size() ? 1 : 0;
  }

  void add_index_entry() {
    std::vector<uint8_t> h;
    put_varint(h, pending_handle_.first);
    put_varint(h, pending_handle_.second);
    index_.add(last_key_.data(), last_key_.size(), h.data(), h.size());
    pending_index_ = false;
  }

  std::pair<uint64_t, uint64_t> write_block(BlockBuilder& b, uint8_t kind) {
    const std::vector<uint8_t>& raw = b.finish();
    uint64_t off = 0, size = 0;
    if (compression_ == 1) {
      std::vector<uint8_t> z = snappy_frame_encode(raw.data(), raw.size());
      if (z.size() < raw.size() - raw.size() / 8) {
        write_raw_block(z.data(), z.size(), 1, kind, &off, &size);
        b.reset();
        return {off, size};
      }
    }
    write_raw_block(raw.data(), raw.size(), 0, kind, &off, &size);
    b.reset();
    return {off, size};
  }

  void write_raw_block(const uint8_t* content, size_t n, uint8_t type, uint8_t kind, uint64_t* off,
                       uint64_t* size) {
    *off = file_.size();
    *size = n;
    file_.insert(file_.end(), content, content + n);
    uint32_t crc = 0;
    if (host_seal_) {
      crc = lcrc_extend(mode_, lcrc_extend(mode_, 0, content, n), &type, 1);
      if (flags_ & LCRC_FLAG_MASK) crc = lcrc32c_mask(crc);
    }
    file_.push_back(type);
    put_le32(file_, crc);
    blocks_.push_back(TableBlock{*off, *size, crc, kind, type});
  }

  uint32_t block_size_;
  int interval_;
  uint8_t compression_;
  int mode_;
  uint32_t flags_;
  bool host_seal_;
  BlockBuilder data_, index_;
  std::vector<uint8_t> file_, last_key_;
  std::vector<TableBlock> blocks_;
  uint64_t num_entries_ = 0;
  bool closed_ = false, pending_index_ = false;
  std::pair<uint64_t, uint64_t> pending_handle_{0, 0};
};

}  // namespace leveldb_gpu

using leveldb_gpu::TableBuilder;

// extern "C" surface for the Python mirror (ctypes) and C callers
extern "C" {

void* lcrc_tb_create(uint32_t block_size, int restart_interval, uint8_t compression, int mode, uint32_t flags,
                     int host_seal) {
  if (restart_interval < 1 || compression > 1 || (mode != LCRC_MODE_REF && mode != LCRC_MODE_C)) return nullptr;
  return new TableBuilder(block_size, restart_interval, compression, mode, flags, host_seal != 0);
}
void lcrc_tb_destroy(void* t) { delete (TableBuilder*)t; }
int lcrc_tb_add(void* t, const uint8_t* key, size_t klen, const uint8_t* val, size_t vlen) {
  return ((TableBuilder*)t)->add(key, klen, val, vlen);
}
// n entries of fixed-size keys and values laid out back to back (keys[i * klen], vals[i * vlen]), in order
int lcrc_tb_add_many(void* t, const uint8_t* keys, size_t klen, const uint8_t* vals, size_t vlen, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    const int rc = ((TableBuilder*)t)->add(keys + i * klen, klen, vals + i * vlen, vlen);
    if (rc) return rc;
  }
  return 0;
}
void lcrc_tb_flush(void* t) { ((TableBuilder*)t)->flush(); }
int lcrc_tb_finish(void* t, const char* filter_name, const uint8_t* filter, size_t filter_len) {
  return ((TableBuilder*)t)->finish(filter_name, filter, filter_len);
}
size_t lcrc_tb_size(void* t) { return ((TableBuilder*)t)->file().size(); }
const uint8_t* lcrc_tb_data(void* t) { return ((TableBuilder*)t)->file().data(); }
// the blocks that carry a trailer, in file order (crc = 0 unless sealed on the host)
size_t lcrc_tb_blocks(void* t, lcrc_tblk* out, size_t cap) {
  const auto& b = ((TableBuilder*)t)->blocks();
  for (size_t i = 0; i < b.size() && i < cap; ++i) {
    out[i].offset = b[i].offset;
    out[i].size = b[i].size;
    out[i].crc = b[i].crc;
    out[i].kind = b[i].kind;
    out[i].type = b[i].type;
    out[i].status = LCRC_TBLK_OK;
    out[i].reserved = 0;
  }
  return b.size();
}
// one lcrc_batch_seal descriptor per block: {offset, n + 1, n + 1} (content ++ type, crc slot right after)
size_t lcrc_tb_seal_descs(void* t, lcrc_desc* out, size_t cap) {
  const auto& b = ((TableBuilder*)t)->blocks();
  for (size_t i = 0; i < b.size() && i < cap; ++i) {
    out[i].offset = b[i].offset;
    out[i].length = (uint32_t)(b[i].size + 1);
    out[i].expect_rel = (int32_t)(b[i].size + 1);
  }
  return b.size();
}

}  // extern "C"
