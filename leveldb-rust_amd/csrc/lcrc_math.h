// Host-side CRC arithmetic shared by the C ABI (scalar API, table generation for the kernels).
//
// Both CRCs on the leveldb-rust checksum path are reflected 32-bit CRCs with init = xorout = ~0:
//   LCRC_MODE_REF: CRC-32/ISO-HDLC, reflected poly 0xEDB88320 -- what crc32fast::Hasher computes at
//                  src/db/log.rs:61-64,261-264, src/sstable/table.rs:519-522, src/sstable/format.rs:164-166.
//   LCRC_MODE_C:   CRC-32C (Castagnoli), reflected poly 0x82F63B78 -- the masked CRC the `snap` framing
//                  stores per chunk (src/sstable/table.rs:486, format.rs:196) and the north-star metric.
//
// "walk(r, M)" below is the raw register recurrence r <- (r >> 8) ^ T0[(r ^ b) & 0xff] over the bytes of M
// starting from register r (no init/xorout). It is linear: walk(r, M) = Z_|M|(r) ^ walk(0, M), where
// Z_n(r) = r * x^(8n) mod P ("advance r over n zero bytes"). Every kernel in this package is built from
// these two facts.
#pragma once
#include <stdint.h>
#include <stddef.h>

namespace lcrc {

constexpr uint32_t POLY_REF = 0xEDB88320u;  // CRC-32/ISO-HDLC (zlib, crc32fast)
constexpr uint32_t POLY_C = 0x82F63B78u;    // CRC-32C (Castagnoli)
constexpr uint32_t CRC_INIT = 0xFFFFFFFFu;
constexpr uint32_t CRC_XOROUT = 0xFFFFFFFFu;
constexpr uint32_t MASK_DELTA = 0xa282ead8u;  // LevelDB crc32c::Mask constant

inline uint32_t poly_of(int mode) { return mode == 1 ? POLY_C : POLY_REF; }

inline uint32_t mask32c(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + MASK_DELTA; }
inline uint32_t unmask32c(uint32_t m) {
  uint32_t rot = m - MASK_DELTA;
  return (rot >> 17) | (rot << 15);
}

// a * b mod P in the reflected representation (bit 31 = x^0). Same recurrence as zlib's multmodp.
inline uint32_t multmodp(uint32_t a, uint32_t b, uint32_t poly) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ poly : b >> 1;
  }
  return p;
}

// x^(8n) mod P. x^(2^k) is obtained by repeated squaring starting from x^1 = 0x40000000.
inline uint32_t x8n(uint64_t n, uint32_t poly) {
  uint32_t p = 1u << 31;       // x^0
  uint32_t sq = 1u << 23;      // x^8
  while (n) {
    if (n & 1) p = multmodp(sq, p, poly);
    sq = multmodp(sq, sq, poly);
    n >>= 1;
  }
  return p;
}

// Z_n(r): advance register r over n zero bytes.
inline uint32_t zshift(uint32_t r, uint64_t n, uint32_t poly) { return multmodp(x8n(n, poly), r, poly); }

// crc(A || B) from crc(A), crc(B), |B| for init = xorout = ~0 (zlib crc32_combine semantics).
inline uint32_t combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b, uint32_t poly) {
  return zshift(crc_a, len_b, poly) ^ crc_b;
}

// slice-by-N tables: T[t][b] = walk(0, [b, 0 x t]) restricted to the register -- T[0] is the byte table.
inline void make_slice_tables(uint32_t poly, uint32_t* T, int nslices) {
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t c = b;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (poly & (0u - (c & 1)));
    T[b] = c;
  }
  for (int t = 1; t < nslices; ++t)
    for (int b = 0; b < 256; ++b) {
      uint32_t prev = T[(t - 1) * 256 + b];
      T[t * 256 + b] = (prev >> 8) ^ T[prev & 0xff];
    }
}

// Byte-sliced form of Z_n: Zt[k][b] = Z_n(b << 8k), so Z_n(r) = xor_k Zt[k][byte_k(r)].
inline void make_shift_tables(uint32_t poly, uint64_t n, uint32_t* Z) {
  uint32_t xp = x8n(n, poly);
  for (int k = 0; k < 4; ++k)
    for (uint32_t b = 0; b < 256; ++b) Z[k * 256 + b] = multmodp(xp, b << (8 * k), poly);
}

}  // namespace lcrc
