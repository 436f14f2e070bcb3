// Scalar host API: the drop-in for the four crc32fast::Hasher call sites of leveldb-rust
// (src/db/log.rs:61-64 and :261-264, src/sstable/table.rs:519-522, src/sstable/format.rs:164-166),
// plus the crc32c value/extend/mask/unmask surface named by the north star.
//
// A single WAL record or a single table block is a few bytes to a few KiB: a device round trip would
// cost far more than the checksum, so these entry points run on the calling host thread (slice-by-8
// tables, SSE4.2 crc32 for CRC-32C when the CPU has it). Bulk work goes through lcrc_batch*, which is
// GPU-only (see lcrc_api.cpp) and never falls back to this code.
#include "../../include/lcrc.h"
#include "lcrc_math.h"

#include <string.h>
#if defined(__x86_64__)
#include <nmmintrin.h>
#endif

namespace {

struct Slice8 {
  uint32_t t[8][256];
  explicit Slice8(uint32_t poly) { lcrc::make_slice_tables(poly, &t[0][0], 8); }
};

const Slice8& tables_ref() {
  static const Slice8 s(lcrc::POLY_REF);
  return s;
}
const Slice8& tables_c() {
  static const Slice8 s(lcrc::POLY_C);
  return s;
}

// raw register walk (no init/xorout), slice-by-8
uint32_t walk_slice8(const Slice8& T, uint32_t r, const uint8_t* p, size_t n) {
  while (n && ((uintptr_t)p & 7)) {
    r = (r >> 8) ^ T.t[0][(r ^ *p++) & 0xff];
    --n;
  }
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= r;
    r = T.t[7][lo & 0xff] ^ T.t[6][(lo >> 8) & 0xff] ^ T.t[5][(lo >> 16) & 0xff] ^ T.t[4][lo >> 24] ^
        T.t[3][hi & 0xff] ^ T.t[2][(hi >> 8) & 0xff] ^ T.t[1][(hi >> 16) & 0xff] ^ T.t[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) r = (r >> 8) ^ T.t[0][(r ^ *p++) & 0xff];
  return r;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t walk_sse42(uint32_t r, const uint8_t* p, size_t n) {
  uint64_t r64 = r;
  while (n && ((uintptr_t)p & 7)) {
    r64 = _mm_crc32_u8((uint32_t)r64, *p++);
    --n;
  }
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    r64 = _mm_crc32_u64(r64, v);
    p += 8;
    n -= 8;
  }
  while (n--) r64 = _mm_crc32_u8((uint32_t)r64, *p++);
  return (uint32_t)r64;
}
bool have_sse42() {
  static const bool v = __builtin_cpu_supports("sse4.2");
  return v;
}
#endif

uint32_t walk_c(uint32_t r, const uint8_t* p, size_t n) {
#if defined(__x86_64__)
  if (have_sse42()) return walk_sse42(r, p, n);
#endif
  return walk_slice8(tables_c(), r, p, n);
}

}  // namespace

extern "C" {

uint32_t lcrc32_extend(uint32_t crc, const uint8_t* p, size_t n) {
  if (n == 0) return crc;
  return walk_slice8(tables_ref(), crc ^ lcrc::CRC_XOROUT, p, n) ^ lcrc::CRC_XOROUT;
}
uint32_t lcrc32_value(const uint8_t* p, size_t n) { return lcrc32_extend(0, p, n); }

uint32_t lcrc32c_extend(uint32_t crc, const uint8_t* p, size_t n) {
  if (n == 0) return crc;
  return walk_c(crc ^ lcrc::CRC_XOROUT, p, n) ^ lcrc::CRC_XOROUT;
}
uint32_t lcrc32c_value(const uint8_t* p, size_t n) { return lcrc32c_extend(0, p, n); }

uint32_t lcrc32c_mask(uint32_t crc) { return lcrc::mask32c(crc); }
uint32_t lcrc32c_unmask(uint32_t masked) { return lcrc::unmask32c(masked); }

uint32_t lcrc_combine(int mode, uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
  return lcrc::combine(crc_a, crc_b, len_b, lcrc::poly_of(mode));
}

uint32_t lcrc_extend(int mode, uint32_t crc, const uint8_t* p, size_t n) {
  return mode == LCRC_MODE_C ? lcrc32c_extend(crc, p, n) : lcrc32_extend(crc, p, n);
}

void lcrc_hasher_init(lcrc_hasher* h, int mode) {
  h->state = 0;
  h->mode = mode;
  h->amount = 0;
}
void lcrc_hasher_update(lcrc_hasher* h, const uint8_t* p, size_t n) {
  h->state = lcrc_extend(h->mode, h->state, p, n);
  h->amount += n;
}
uint32_t lcrc_hasher_finalize(const lcrc_hasher* h) { return h->state; }

}  // extern "C"
