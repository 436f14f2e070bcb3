// Scalar host API: the drop-in for the four crc32fast::Hasher call sites of leveldb-rust
// (src/db/log.rs:61-64 and :261-264, src/sstable/table.rs:519-522, src/sstable/format.rs:164-166),
// plus the crc32c value/extend/mask/unmask surface named by the north star.
//
// A single WAL record or a single table block is a few bytes to a few KiB: a device round trip would
// cost far more than the checksum, so these entry points run on the calling host thread: both CRCs by
// carry-less multiply folding from 64 bytes on (as crc32fast does for CRC-32 on x86-64), CRC-32C tails
// with the SSE4.2 crc32 instruction, slice-by-8 tables otherwise and on CPUs without the instructions.
// Bulk work goes through lcrc_batch*, which is GPU-only (see lcrc_api.cpp) and never falls back to this
// code.
#include "../../include/lcrc.h"
#include "lcrc_math.h"

#include <string.h>
#if defined(__x86_64__)
#include <nmmintrin.h>
#include <smmintrin.h>
#include <wmmintrin.h>
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

// Raw reflected-CRC register walk over n >= 64 bytes, n a multiple of 16, by PCLMULQDQ folding (the
// published scheme: four 128-bit lanes folded 512 bits forward, then to one lane, 128 -> 64 -> 32 bits
// and a Barrett reduction). The constants are x^k mod P for the fold distances, bit-reflected in 32 bits
// and shifted left by one: R1 = x^(4*128+32), R2 = x^(4*128-32), R3 = x^(128+32), R4 = x^(128-32),
// R5 = x^64; then mu = floor(x^64 / P) and P, reflected in 33 bits (recomputed from P by
// tests/test_oracle.py::test_host_clmul_constants).
struct ClmulK {
  long long r1, r2, r3, r4, r5, mu, p;
};
constexpr ClmulK K_REF = {0x0154442bd4LL, 0x01c6e41596LL, 0x01751997d0LL, 0x00ccaa009eLL,
                          0x0163cd6124LL, 0x01f7011641LL, 0x01db710641LL};  // P = 0x104C11DB7
constexpr ClmulK K_C = {0x00740eef02LL, 0x009e4addf8LL, 0x00f20c0dfeLL, 0x014cd00bd6LL,
                        0x00dd45aab8LL, 0x00dea713f1LL, 0x0105ec76f1LL};  // P = 0x11EDC6F41

__attribute__((target("pclmul,sse4.1"))) inline __m128i clmul_fold(__m128i x, __m128i k, __m128i next) {
  return _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x, k, 0x00), _mm_clmulepi64_si128(x, k, 0x11)), next);
}

__attribute__((target("pclmul,sse4.1"))) uint32_t walk_clmul(const ClmulK& K, uint32_t r, const uint8_t* p,
                                                             size_t n) {
  const __m128i k12 = _mm_set_epi64x(K.r2, K.r1);
  const __m128i k34 = _mm_set_epi64x(K.r4, K.r3);
  const __m128i k5 = _mm_set_epi64x(0, K.r5);
  const __m128i pmu = _mm_set_epi64x(K.mu, K.p);
  const __m128i m32 = _mm_set_epi32(0, 0, 0, -1);
  auto ld = [](const uint8_t* q) { return _mm_loadu_si128((const __m128i*)q); };
  __m128i x1 = _mm_xor_si128(ld(p), _mm_cvtsi32_si128((int)r)), x2 = ld(p + 16), x3 = ld(p + 32), x4 = ld(p + 48);
  p += 64;
  n -= 64;
  for (; n >= 64; p += 64, n -= 64) {
    x1 = clmul_fold(x1, k12, ld(p));
    x2 = clmul_fold(x2, k12, ld(p + 16));
    x3 = clmul_fold(x3, k12, ld(p + 32));
    x4 = clmul_fold(x4, k12, ld(p + 48));
  }
  x1 = clmul_fold(x1, k34, x2);
  x1 = clmul_fold(x1, k34, x3);
  x1 = clmul_fold(x1, k34, x4);
  for (; n >= 16; p += 16, n -= 16) x1 = clmul_fold(x1, k34, ld(p));
  // 128 -> 64 (R4 times the low half, appends 32 zero bits), 64 -> 32 (R5), Barrett
  x1 = _mm_xor_si128(_mm_srli_si128(x1, 8), _mm_clmulepi64_si128(k34, x1, 0x01));
  __m128i t = _mm_and_si128(x1, m32);
  x1 = _mm_xor_si128(_mm_srli_si128(x1, 4), _mm_clmulepi64_si128(t, k5, 0x00));
  t = _mm_and_si128(_mm_clmulepi64_si128(_mm_and_si128(x1, m32), pmu, 0x10), m32);
  x1 = _mm_xor_si128(x1, _mm_clmulepi64_si128(t, pmu, 0x00));
  return (uint32_t)_mm_extract_epi32(x1, 1);
}
bool have_clmul() {
  static const bool v = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
  return v;
}
#endif

uint32_t walk_ref(uint32_t r, const uint8_t* p, size_t n) {
#if defined(__x86_64__)
  if (n >= 64 && have_clmul()) {
    const size_t m = n & ~(size_t)15;
    r = walk_clmul(K_REF, r, p, m);
    p += m;
    n -= m;
  }
#endif
  return walk_slice8(tables_ref(), r, p, n);
}

uint32_t walk_c(uint32_t r, const uint8_t* p, size_t n) {
#if defined(__x86_64__)
  if (n >= 64 && have_clmul()) {  // folding outruns the serial crc32 instruction (one 8 B step per 3 cycles)
    const size_t m = n & ~(size_t)15;
    r = walk_clmul(K_C, r, p, m);
    p += m;
    n -= m;
  }
  if (have_sse42()) return walk_sse42(r, p, n);
#endif
  return walk_slice8(tables_c(), r, p, n);
}

}  // namespace

extern "C" {

uint32_t lcrc32_extend(uint32_t crc, const uint8_t* p, size_t n) {
  if (n == 0) return crc;
  return walk_ref(crc ^ lcrc::CRC_XOROUT, p, n) ^ lcrc::CRC_XOROUT;
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
