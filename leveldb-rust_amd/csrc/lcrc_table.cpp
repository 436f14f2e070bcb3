// SSTable structure walk for the whole-table verify scan, host side.
// Restates the parts of the reference's table reader that locate blocks -- the checksums themselves are
// computed on the device by lcrc_table_scan (lcrc_api.cpp):
//   varint32/64 decode              <- src/util/coding.rs:92-130 (DecodeVarint for &[u8])
//   BlockHandle::decode_from        <- src/sstable/format.rs:55-59
//   Footer::decoded_from            <- src/sstable/format.rs:103-118 (magic 0xdb4775248b80fb57, :19)
//   read_block_from_file            <- src/sstable/format.rs:146-213 (verify :162-171, type dispatch
//                                      :175-210, "corrupted compressed block content" :199-203)
//   Block::from_content             <- src/sstable/block.rs:21-41
//   BlockIter::decode_entry         <- src/sstable/block.rs:124-148 (+ the shared-prefix check of
//                                      parse_next_key :150-175)
//   Table::open / read_meta         <- src/sstable/table.rs:39-103 (index verified iff paranoid_checks;
//                                      metaindex errors are swallowed; filter key = "filter" + name)
//   snap::read::FrameDecoder        <- the published Snappy framing format (stream identifier
//                                      ff 06 00 00 "sNaPpY"; chunks [type][u24 len][masked CRC-32C of
//                                      the uncompressed data]); the crate itself is not in the image
//                                      (SURVEY.md §8(c)), every decode error maps to the reference's one
//                                      message.
#include <stdint.h>
#include <string.h>

#include <functional>
#include <string>
#include <vector>

#include "../../include/lcrc.h"
#include "lcrc_table.h"

namespace lcrc_tbl {

static inline uint32_t le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

bool get_varint32(const uint8_t*& p, const uint8_t* end, uint32_t& out) {
  uint32_t result = 0;
  for (uint32_t shift = 0; shift <= 28; shift += 7) {
    if (p >= end) return false;
    const uint32_t b = *p++;
    result |= (b & 127u) << shift;
    if (!(b & 128u)) {
      out = result;
      return true;
    }
  }
  return false;
}

bool get_varint64(const uint8_t*& p, const uint8_t* end, uint64_t& out) {
  uint64_t result = 0;
  for (uint32_t shift = 0; shift <= 63; shift += 7) {
    if (p >= end) return false;
    const uint64_t b = *p++;
    result |= (b & 127u) << shift;
    if (!(b & 128u)) {
      out = result;
      return true;
    }
  }
  return false;
}

const char* decode_handle(const uint8_t*& p, const uint8_t* end, Handle& h) {
  if (!get_varint64(p, end, h.offset) || !get_varint64(p, end, h.size)) return "Error when decoding varint64";
  return nullptr;
}

const char* decode_footer(const uint8_t* f, Handle& metaindex, Handle& index) {
  const uint64_t magic = (uint64_t)le32(f + FOOTER_ENCODED_LENGTH - 8) |
                         ((uint64_t)le32(f + FOOTER_ENCODED_LENGTH - 4) << 32);
  if (magic != TABLE_MAGIC_NUMBER) return "not an sstable (bad magic number)";
  const uint8_t* p = f;
  const uint8_t* end = f + FOOTER_ENCODED_LENGTH;
  if (const char* e = decode_handle(p, end, metaindex)) return e;
  return decode_handle(p, end, index);
}

// ---- Snappy ---------------------------------------------------------------------------------------
// The length preamble as snap's bytes::read_varu64 reads it (up to 10 bytes, mod 2^64), accepted only up to the
// frame decoder's MAX_BLOCK_SIZE (65,536): a 5-byte preamble of 2^32 is an error, not a zero length.
static bool snappy_preamble(const uint8_t*& p, const uint8_t* end, uint32_t& out) {
  uint64_t v = 0;
  for (uint32_t i = 0; i < 10 && p < end; ++i) {
    const uint64_t b = *p++;
    v |= (b & 127u) << (7 * i);
    if (!(b & 128u)) {
      out = (uint32_t)v;
      return v <= 65536;
    }
  }
  return false;
}

bool snappy_raw_decompress(const uint8_t* p, size_t n, std::vector<uint8_t>& out) {
  const uint8_t* end = p + n;
  uint32_t ulen;
  if (!snappy_preamble(p, end, ulen)) return false;
  const size_t base = out.size();
  out.reserve(base + ulen);
  while (p < end) {
    const uint32_t tag = *p++;
    uint64_t len, offset;
    switch (tag & 3) {
      case 0: {  // literal
        len = tag >> 2;
        if (len >= 60) {
          const uint32_t nb = (uint32_t)len - 59;  // 1..4 little-endian length bytes
          if ((size_t)(end - p) < 4) return false;  // snap reads the length as one 4-byte word, whatever nb is
          len = 0;
          for (uint32_t i = 0; i < nb; ++i) len |= (uint64_t)p[i] << (8 * i);
          p += nb;
        }
        len += 1;
        if ((uint64_t)(end - p) < len || out.size() - base + len > ulen) return false;
        out.insert(out.end(), p, p + len);
        p += len;
        continue;
      }
      case 1:  // copy, 11-bit offset
        if (p >= end) return false;
        len = 4 + ((tag >> 2) & 7);
        offset = ((uint64_t)(tag >> 5) << 8) | *p++;
        break;
      case 2:  // copy, 16-bit offset
        if (end - p < 2) return false;
        len = 1 + (tag >> 2);
        offset = (uint64_t)p[0] | ((uint64_t)p[1] << 8);
        p += 2;
        break;
      default:  // copy, 32-bit offset
        if (end - p < 4) return false;
        len = 1 + (tag >> 2);
        offset = le32(p);
        p += 4;
        break;
    }
    const size_t have = out.size() - base;
    if (offset == 0 || offset > have || have + len > ulen) return false;
    for (uint64_t i = 0; i < len; ++i) out.push_back(out[out.size() - offset]);  // overlap allowed
  }
  return out.size() - base == ulen;
}

bool snappy_frame_decode(const uint8_t* p, size_t n, std::vector<uint8_t>& out) {
  static const uint8_t kStreamId[6] = {'s', 'N', 'a', 'P', 'p', 'Y'};
  const uint8_t* end = p + n;
  bool seen_id = false;
  while (p < end) {
    if (end - p < 4) return false;
    const uint32_t type = p[0];
    const uint32_t len = (uint32_t)p[1] | ((uint32_t)p[2] << 8) | ((uint32_t)p[3] << 16);
    p += 4;
    if ((uint64_t)(end - p) < len || len > 76490) return false;  // snap: MAX_COMPRESS_BLOCK_SIZE, any chunk type
    const uint8_t* body = p;
    p += len;
    if (type == 0xff) {  // stream identifier (may repeat)
      if (len != 6 || memcmp(body, kStreamId, 6) != 0) return false;
      seen_id = true;
      continue;
    }
    if (!seen_id) return false;
    if (type == 0x00 || type == 0x01) {
      if (len < 4) return false;
      const uint32_t want = le32(body);
      const size_t start = out.size();
      if (type == 0x00) {
        if (!snappy_raw_decompress(body + 4, len - 4, out)) return false;
      } else {
        out.insert(out.end(), body + 4, body + len);
      }
      if (out.size() - start > 65536) return false;
      if (lcrc32c_mask(lcrc32c_value(out.data() + start, out.size() - start)) != want) return false;
      continue;
    }
    if (type <= 0x7f) return false;  // reserved unskippable chunk
    // 0x80..0xfe: reserved skippable / padding
  }
  return true;
}

// ---- blocks ---------------------------------------------------------------------------------------
const char* block_contents(const uint8_t* blk, uint64_t n, bool verify, int mode, uint32_t flags,
                           std::vector<uint8_t>& out) {
  if (verify) {
    uint32_t c = lcrc_extend(mode, 0, blk, n + 1);
    if (flags & LCRC_FLAG_MASK) c = lcrc32c_mask(c);
    if (c != le32(blk + n + 1)) return "block checksum mismatch";
  }
  out.clear();
  switch (blk[n]) {
    case 0:
      out.assign(blk, blk + n);
      return nullptr;
    case 1:
      if (!snappy_frame_decode(blk, n, out)) return "corrupted compressed block content";
      return nullptr;
    default:
      return "bad block type";
  }
}

const char* block_entries(const std::vector<uint8_t>& d,
                          const std::function<bool(const std::string&, const uint8_t*, uint32_t)>& f) {
  const size_t n = d.size();
  if (n < 4) return "bad block contents, size smaller than u32";
  const uint32_t num_restarts = le32(d.data() + n - 4);
  if ((uint64_t)num_restarts > (n - 4) / 4) return "bad block contents";
  const uint32_t restarts = (uint32_t)(n - (1 + (uint64_t)num_restarts) * 4);
  std::string key;
  uint32_t off = 0;
  while (off < restarts) {
    if (restarts - off < 3) return "bad entry in block";
    const uint8_t* p = d.data() + off;
    const uint8_t* lim = d.data() + restarts;
    uint32_t shared, non_shared, value_len;
    if (!get_varint32(p, lim, shared) || !get_varint32(p, lim, non_shared) || !get_varint32(p, lim, value_len))
      return "bad entry in block";
    const uint32_t step = (uint32_t)(p - (d.data() + off));
    if ((uint64_t)restarts - off - step < (uint64_t)non_shared + value_len) return "bad entry in block";
    if (key.size() < shared) return "bad entry in block";
    key.resize(shared);
    key.append((const char*)p, non_shared);
    if (!f(key, p + non_shared, value_len)) return nullptr;
    off += step + non_shared + value_len;
  }
  return nullptr;
}

}  // namespace lcrc_tbl

// ------------------------------------------------------------------------------------------------
// test surface (Python mirror): the Snappy framing decoder on host bytes
// ------------------------------------------------------------------------------------------------
extern "C" {
// Decodes a Snappy-framed buffer; returns the uncompressed size and copies up to cap bytes to out,
// or -1 when the stream is corrupt (including a chunk CRC-32C mismatch).
int64_t lcrc_snappy_frame_decode(const uint8_t* p, size_t n, uint8_t* out, size_t cap) {
  std::vector<uint8_t> v;
  if (!lcrc_tbl::snappy_frame_decode(p, n, v)) return -1;
  if (out) memcpy(out, v.data(), v.size() < cap ? v.size() : cap);
  return (int64_t)v.size();
}
}
