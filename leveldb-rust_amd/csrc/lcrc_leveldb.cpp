// Host side above the C ABI: C++ restatements of the leveldb-rust call sites that checksum blocks and
// records, wired to lcrc.h. The reference is Rust (no Rust toolchain in this image), so these classes
// are the drop-in demonstration: same framing, same error strings, same dropped-byte accounting.
//
//   LogWriter         <- src/db/log.rs:7-81     (add_record :21-52, emit_physical_record :58-80)
//   LogReader         <- src/db/log.rs:83-280   (read_record :106-201, read_physical_record :204-279)
//   BatchLogReader    <- the same reader contract, but every physical-record checksum of the file is
//                        verified in one device pass (lcrc_wal_scan) and the state machine replays the
//                        per-record verdicts
//   write_raw_block   <- src/sstable/table.rs:507-529
//   read_block        <- src/sstable/format.rs:146-213 (verify :162-171; type dispatch :175-210)
//
// Exposed to Python through the extern "C" functions at the bottom (ctypes; see __init__.py).
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/lcrc.h"

namespace leveldb_gpu {

constexpr size_t BLOCK_SIZE = 32768;  // src/db/mod.rs:45
constexpr size_t HEADER_SIZE = 7;     // src/db/mod.rs:48
constexpr size_t BLOCK_TRAILER_SIZE = 5;  // src/sstable/format.rs:22

// src/db/mod.rs:34-63
enum RecordType : int {
  ZeroType = 0,
  FullType = 1,
  FirstType = 2,
  MiddleType = 3,
  LastType = 4,
  Eof = 5,
  BadRecord = 6,
  UnKnown = 7,
};
inline RecordType record_type_from(uint8_t n) { return n <= 6 ? (RecordType)n : UnKnown; }

static inline void put_le32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)v;
  p[1] = (uint8_t)(v >> 8);
  p[2] = (uint8_t)(v >> 16);
  p[3] = (uint8_t)(v >> 24);
}
static inline uint32_t get_le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// ------------------------------------------------------------------------------------------------
class LogWriter {
 public:
  explicit LogWriter(size_t offset = 0) : offset_(offset) {}
  // log.rs:21-52
  void add_record(const uint8_t* p, size_t left_total) {
    bool begin = true;
    size_t left = left_total;
    while (left > 0) {  // empty input emits nothing (log.rs:24-26)
      size_t leftover = BLOCK_SIZE - offset_;
      if (leftover < HEADER_SIZE) {
        static const uint8_t zeros[HEADER_SIZE] = {0};
        file_.insert(file_.end(), zeros, zeros + leftover);
        offset_ = 0;
      }
      const size_t avail = BLOCK_SIZE - offset_ - HEADER_SIZE;
      RecordType t;
      size_t frag;
      if (begin && left <= avail) {
        t = FullType;
        frag = left;
      } else if (begin) {
        t = FirstType;
        frag = avail;
      } else if (left <= avail) {
        t = LastType;
        frag = left;
      } else {
        t = MiddleType;
        frag = avail;
      }
      emit_physical_record(t, p, frag);
      p += frag;
      left -= frag;
      begin = false;
    }
  }
  const std::vector<uint8_t>& file() const { return file_; }
  std::vector<uint8_t>& file() { return file_; }

 private:
  // log.rs:58-80; checksum = crc32fast over [type] ++ data (call site 1)
  void emit_physical_record(RecordType t, const uint8_t* p, size_t n) {
    lcrc_hasher h;
    lcrc_hasher_init(&h, LCRC_MODE_REF);
    const uint8_t tb = (uint8_t)t;
    lcrc_hasher_update(&h, &tb, 1);
    lcrc_hasher_update(&h, p, n);
    uint8_t header[HEADER_SIZE];
    put_le32(header, lcrc_hasher_finalize(&h));
    header[4] = (uint8_t)(n & 0xff);
    header[5] = (uint8_t)((n >> 8) & 0xff);
    header[6] = tb;
    file_.insert(file_.end(), header, header + HEADER_SIZE);
    file_.insert(file_.end(), p, p + n);
    offset_ += HEADER_SIZE + n;
  }
  std::vector<uint8_t> file_;
  size_t offset_;
};

// Reporter (src/db/mod.rs:90-92) as used by the reference tests (log.rs:371-393): sum of dropped bytes
// and the concatenation of the status strings.
struct Reporter {
  size_t dropped = 0;
  std::string message;
  void corruption(size_t n, const char* status) {
    dropped += n;
    message += status;
  }
};

// In-memory SequentialFile (the reference's MemoryFile test double, log.rs:292-369).
struct MemorySequentialFile {
  const uint8_t* data = nullptr;
  size_t len = 0;
  size_t consumed = 0;
  bool force_error = false;
  // returns -1 on a (forced) read error
  long read(uint8_t* buf, size_t n) {
    if (force_error) {
      force_error = false;
      return -1;
    }
    size_t remain = len - consumed;
    size_t k = remain < n ? remain : n;
    memcpy(buf, data + consumed, k);
    consumed += k;
    return (long)k;
  }
};

enum ReadStatus { READ_OK = 0, READ_EOF = 1 };

// Physical-record source: either computes the checksum on the host (LogReader) or looks it up in the
// per-record verdicts of a device scan (BatchLogReader). Both follow log.rs:204-279 step by step.
class LogReaderBase {
 public:
  explicit LogReaderBase(MemorySequentialFile f) : file_(f), buffer_(BLOCK_SIZE, 0) {}
  virtual ~LogReaderBase() {}

  // log.rs:106-201
  ReadStatus read_record(std::vector<uint8_t>& record) {
    bool in_fragment_record = false;
    record.clear();
    for (;;) {
      size_t n = 0;
      RecordType t = read_physical_record(record, n);
      switch (t) {
        case FullType:
          if (in_fragment_record && !record.empty()) {
            size_t dropped = record.size() - n;
            if (dropped > 0) reporter_.corruption(dropped, "partial record without end(1)");
            record.erase(record.begin(), record.begin() + dropped);
          }
          return READ_OK;
        case FirstType:
          if (in_fragment_record && !record.empty()) {
            size_t dropped = record.size() - n;
            if (dropped > 0) reporter_.corruption(dropped, "partial record without end(2)");
            record.erase(record.begin(), record.begin() + dropped);
          }
          in_fragment_record = true;
          break;
        case MiddleType:
          if (!in_fragment_record) {
            reporter_.corruption(n, "missing start of fragmented record(1)");
            record.resize(record.size() - n);
          }
          break;
        case LastType:
          if (!in_fragment_record) {
            reporter_.corruption(n, "missing start of fragmented record(2)");
            record.resize(record.size() - n);
          } else {
            return READ_OK;
          }
          break;
        case Eof:
          if (in_fragment_record) record.clear();
          return READ_EOF;
        case BadRecord:
          if (in_fragment_record) {
            reporter_.corruption(record.size(), "error in middle of record");
            record.clear();
            in_fragment_record = false;
          }
          break;
        default:  // ZeroType with a payload, UnKnown
          reporter_.corruption(record.size(), "unknown record type");
          in_fragment_record = false;
          record.clear();
          break;
      }
    }
  }

  const Reporter& reporter() const { return reporter_; }
  MemorySequentialFile& file() { return file_; }

 protected:
  // log.rs:204-279. Returns the record type; `n` = bytes appended to record.
  RecordType read_physical_record(std::vector<uint8_t>& record, size_t& n) {
    n = 0;
    for (;;) {
      if (cap_ - consumed_ < HEADER_SIZE) {
        if (!eof_) {
          consumed_ = 0;
          long got = file_.read(buffer_.data(), BLOCK_SIZE);
          if (got < 0) {
            reporter_.corruption(BLOCK_SIZE, "read error");
            eof_ = true;
            return Eof;
          }
          block_start_ = file_.consumed - (size_t)got;
          cap_ = (size_t)got;
          if (cap_ < BLOCK_SIZE) eof_ = true;
          continue;
        } else {
          consumed_ = 0;
          cap_ = 0;
          return Eof;
        }
      }
      const uint8_t* h = buffer_.data() + consumed_;
      const uint32_t checksum = get_le32(h);
      const size_t length = (size_t)h[4] | ((size_t)h[5] << 8);
      const uint8_t type = h[6];
      if (HEADER_SIZE + length > cap_ - consumed_) {
        const size_t dropped = cap_ - consumed_;
        consumed_ = 0;
        cap_ = 0;
        if (!eof_) {
          reporter_.corruption(dropped, "bad record length");
          return BadRecord;
        }
        return Eof;
      }
      if (type == ZeroType && length == 0) {
        consumed_ = 0;
        cap_ = 0;
        return BadRecord;
      }
      const uint8_t* data = h + HEADER_SIZE;
      if (!checksum_ok(block_start_ + consumed_, checksum, type, data, length)) {
        const size_t dropped = cap_ - consumed_;
        consumed_ = 0;
        cap_ = 0;
        reporter_.corruption(dropped, "checksum mismatch");
        n = length;
        return BadRecord;
      }
      consumed_ += HEADER_SIZE + length;
      record.insert(record.end(), data, data + length);
      n = length;
      return record_type_from(type);
    }
  }

  // header_off: file offset of the record header
  virtual bool checksum_ok(size_t header_off, uint32_t expect, uint8_t type, const uint8_t* data, size_t n) = 0;

  MemorySequentialFile file_;
  Reporter reporter_;
  std::vector<uint8_t> buffer_;
  size_t consumed_ = 0, cap_ = 0, block_start_ = 0;
  bool eof_ = false;
};

class LogReader : public LogReaderBase {
 public:
  using LogReaderBase::LogReaderBase;

 protected:
  // call site 2 (log.rs:260-264): host scalar crc over [type] ++ data
  bool checksum_ok(size_t, uint32_t expect, uint8_t type, const uint8_t* data, size_t n) override {
    lcrc_hasher h;
    lcrc_hasher_init(&h, LCRC_MODE_REF);
    lcrc_hasher_update(&h, &type, 1);
    lcrc_hasher_update(&h, data, n);
    return lcrc_hasher_finalize(&h) == expect;
  }
};

// Same contract; the checksums were computed for every record of the file by one lcrc_wal_scan.
class BatchLogReader : public LogReaderBase {
 public:
  BatchLogReader(MemorySequentialFile f, std::vector<lcrc_wal_rec> recs) : LogReaderBase(f), recs_(std::move(recs)) {}
  int consistency_errors() const { return consistency_errors_; }

 protected:
  bool checksum_ok(size_t header_off, uint32_t expect, uint8_t type, const uint8_t*, size_t n) override {
    // the device parse walked the same header chain, so the record at header_off is next in file order
    while (pos_ < recs_.size() && recs_[pos_].header < header_off) ++pos_;
    if (pos_ >= recs_.size() || recs_[pos_].header != header_off || recs_[pos_].length != n ||
        recs_[pos_].type != type) {
      ++consistency_errors_;
      return false;
    }
    const lcrc_wal_rec& r = recs_[pos_++];
    (void)expect;
    return r.status == LCRC_WAL_OK;
  }

 private:
  std::vector<lcrc_wal_rec> recs_;
  size_t pos_ = 0;
  int consistency_errors_ = 0;
};

// ------------------------------------------------------------------------------------------------
// SSTable block trailer (table.rs:507-529): content ++ [type u8][crc32fast(content ++ type) u32 LE]
void write_raw_block(std::vector<uint8_t>& file, const uint8_t* content, size_t n, uint8_t type,
                     uint64_t* handle_offset, uint64_t* handle_size) {
  *handle_offset = file.size();
  *handle_size = n;
  file.insert(file.end(), content, content + n);
  lcrc_hasher h;
  lcrc_hasher_init(&h, LCRC_MODE_REF);
  lcrc_hasher_update(&h, content, n);
  lcrc_hasher_update(&h, &type, 1);
  uint8_t trailer[BLOCK_TRAILER_SIZE];
  trailer[0] = type;
  put_le32(trailer + 1, lcrc_hasher_finalize(&h));
  file.insert(file.end(), trailer, trailer + BLOCK_TRAILER_SIZE);
}

// format.rs:146-213 up to the type dispatch. Returns 0 and the stored bytes on success, else an error
// string identical to the reference's StatusError::Corruption text.
const char* read_block(const uint8_t* file, size_t file_len, uint64_t off, uint64_t n, bool verify,
                       const uint8_t** data, uint8_t* type) {
  if (off > file_len || n + BLOCK_TRAILER_SIZE > file_len - off) return "truncated block read";
  const uint8_t* d = file + off;
  if (verify) {
    const uint32_t expect = get_le32(d + n + 1);
    if (lcrc32_value(d, n + 1) != expect) return "block checksum mismatch";
  }
  if (d[n] != 0 && d[n] != 1) return "bad block type";
  *data = d;
  *type = d[n];
  return nullptr;
}

}  // namespace leveldb_gpu

// ------------------------------------------------------------------------------------------------
// extern "C" surface for the Python mirror (ctypes)
// ------------------------------------------------------------------------------------------------
using namespace leveldb_gpu;

extern "C" {

void* lcrc_logw_create(uint64_t offset) { return new LogWriter((size_t)offset); }
void lcrc_logw_destroy(void* w) { delete (LogWriter*)w; }
void lcrc_logw_add(void* w, const uint8_t* p, size_t n) { ((LogWriter*)w)->add_record(p, n); }
size_t lcrc_logw_size(void* w) { return ((LogWriter*)w)->file().size(); }
const uint8_t* lcrc_logw_data(void* w) { return ((LogWriter*)w)->file().data(); }
// append raw bytes (a previous file's content when "reopening for append")
void lcrc_logw_prepend(void* w, const uint8_t* p, size_t n) {
  auto& f = ((LogWriter*)w)->file();
  f.insert(f.begin(), p, p + n);
}

struct ReaderHandle {
  std::vector<uint8_t> file;  // owned copy
  LogReaderBase* reader = nullptr;
  std::vector<uint8_t> record;
  ~ReaderHandle() { delete reader; }
};

void* lcrc_logr_create(const uint8_t* p, size_t n) {
  ReaderHandle* h = new ReaderHandle();
  h->file.assign(p, p + n);
  MemorySequentialFile f;
  f.data = h->file.data();
  f.len = n;
  h->reader = new LogReader(f);
  return h;
}

// Batch reader: file is a host copy of the log; recs are the (host) results of lcrc_wal_scan.
void* lcrc_logr_create_batch(const uint8_t* p, size_t n, const lcrc_wal_rec* recs, size_t nrecs) {
  ReaderHandle* h = new ReaderHandle();
  h->file.assign(p, p + n);
  MemorySequentialFile f;
  f.data = h->file.data();
  f.len = n;
  h->reader = new BatchLogReader(f, std::vector<lcrc_wal_rec>(recs, recs + nrecs));
  return h;
}
void lcrc_logr_destroy(void* h) { delete (ReaderHandle*)h; }
void lcrc_logr_force_error(void* h) { ((ReaderHandle*)h)->reader->file().force_error = true; }
// 0 = record available (lcrc_logr_record), 1 = EOF ("meet a eof")
int lcrc_logr_read(void* h) { return ((ReaderHandle*)h)->reader->read_record(((ReaderHandle*)h)->record); }
size_t lcrc_logr_record(void* h, const uint8_t** p) {
  *p = ((ReaderHandle*)h)->record.data();
  return ((ReaderHandle*)h)->record.size();
}
size_t lcrc_logr_dropped(void* h) { return ((ReaderHandle*)h)->reader->reporter().dropped; }
const char* lcrc_logr_message(void* h) { return ((ReaderHandle*)h)->reader->reporter().message.c_str(); }
int lcrc_logr_consistency_errors(void* h) {
  BatchLogReader* b = dynamic_cast<BatchLogReader*>(((ReaderHandle*)h)->reader);
  return b ? b->consistency_errors() : 0;
}

// SSTable trailer writer: appends to a growable buffer owned by the handle
void* lcrc_tbl_create(void) { return new std::vector<uint8_t>(); }
void lcrc_tbl_destroy(void* t) { delete (std::vector<uint8_t>*)t; }
void lcrc_tbl_write_raw_block(void* t, const uint8_t* content, size_t n, uint8_t type, uint64_t* off, uint64_t* size) {
  write_raw_block(*(std::vector<uint8_t>*)t, content, n, type, off, size);
}
size_t lcrc_tbl_size(void* t) { return ((std::vector<uint8_t>*)t)->size(); }
const uint8_t* lcrc_tbl_data(void* t) { return ((std::vector<uint8_t>*)t)->data(); }
void lcrc_tbl_append(void* t, const uint8_t* p, size_t n) {
  auto& f = *(std::vector<uint8_t>*)t;
  f.insert(f.end(), p, p + n);
}
// returns nullptr on success, else the reference's error string
const char* lcrc_tbl_read_block(const uint8_t* file, size_t len, uint64_t off, uint64_t n, int verify, uint8_t* type) {
  const uint8_t* d = nullptr;
  return read_block(file, len, off, n, verify != 0, &d, type);
}

}  // extern "C"
