/*
 * crc_oracle.c -- TEST INFRASTRUCTURE. CPU restatement of the checksum arithmetic on the leveldb-rust
 * block/record path. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker or the CPU baseline -- never as the thing measured or shipped.
 *
 * What it restates:
 *  - The reference's checksum is the external crate `crc32fast` ("1.2.0", Cargo.toml:11; source not in
 *    /root/reference, Cargo.lock git-ignored -> patch version unpinned). crc32fast computes
 *    CRC-32/ISO-HDLC (reflected poly 0xEDB88320, init 0xFFFFFFFF, xorout 0xFFFFFFFF). Its published
 *    algorithm: a PCLMULQDQ 4x128-bit folding path on x86 (SSE4.1 + PCLMULQDQ detected at run time),
 *    otherwise slice-by-16 tables. Call sites: src/db/log.rs:61-64, :261-264, :482-484 (test),
 *    src/sstable/table.rs:519-522, src/sstable/format.rs:164-166.
 *  - The masked CRC-32C of the `snap` crate ("1", Cargo.toml:15) framing: CRC-32C (reflected poly
 *    0x82F63B78) masked as rotr15(crc) + 0xa282ead8 per chunk; snap's x86 path uses the SSE4.2 crc32
 *    instruction, else slice-by-16.
 *  - orc_crc_bitwise is the definition, bit by bit (the pinning reference for everything else).
 *
 * Parity pinning: the reference's own tests hold no CRC literal. The oracle is pinned
 * by published check values (CRC-32 "123456789" = 0xCBF43926, CRC-32C = 0xE3069283, RFC 3720 B.4
 * vectors) and cross-checked against Python's zlib.crc32 (tests/test_oracle.py).
 */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <time.h>

#if defined(__x86_64__)
#include <immintrin.h>
#include <nmmintrin.h>
#include <wmmintrin.h>
#endif

#define ORC_POLY_REF 0xEDB88320u
#define ORC_POLY_C 0x82F63B78u

/* ---- definition: bitwise reflected CRC ---- */
uint32_t orc_crc_bitwise(uint32_t poly, uint32_t init, uint32_t xorout, const uint8_t* p, size_t n) {
  uint32_t c = init;
  for (size_t i = 0; i < n; ++i) {
    c ^= p[i];
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (poly & (0u - (c & 1u)));
  }
  return c ^ xorout;
}

uint32_t orc_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }
uint32_t orc_unmask(uint32_t m) {
  uint32_t rot = m - 0xa282ead8u;
  return (rot >> 17) | (rot << 15);
}

/* ---- slice-by-16 (crc32fast's and snap's table fallback) ---- */
static uint32_t s16_ref[16][256], s16_c[16][256];
static int s16_ready = 0;
static void s16_init(void) {
  if (s16_ready) return;
  for (int m = 0; m < 2; ++m) {
    uint32_t(*T)[256] = m ? s16_c : s16_ref;
    uint32_t poly = m ? ORC_POLY_C : ORC_POLY_REF;
    for (uint32_t b = 0; b < 256; ++b) {
      uint32_t c = b;
      for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (poly & (0u - (c & 1u)));
      T[0][b] = c;
    }
    for (int t = 1; t < 16; ++t)
      for (int b = 0; b < 256; ++b) T[t][b] = (T[t - 1][b] >> 8) ^ T[0][T[t - 1][b] & 0xff];
  }
  s16_ready = 1;
}

/* crc = finalized crc of the previous bytes (0 for none), like Hasher::new_with_initial */
uint32_t orc_crc_s16(int mode, uint32_t crc, const uint8_t* p, size_t n) {
  s16_init();
  uint32_t(*T)[256] = mode ? s16_c : s16_ref;
  uint32_t c = ~crc;
  while (n >= 16) {
    uint32_t w0, w1, w2, w3;
    memcpy(&w0, p, 4);
    memcpy(&w1, p + 4, 4);
    memcpy(&w2, p + 8, 4);
    memcpy(&w3, p + 12, 4);
    w0 ^= c;
    c = T[15][w0 & 0xff] ^ T[14][(w0 >> 8) & 0xff] ^ T[13][(w0 >> 16) & 0xff] ^ T[12][w0 >> 24] ^
        T[11][w1 & 0xff] ^ T[10][(w1 >> 8) & 0xff] ^ T[9][(w1 >> 16) & 0xff] ^ T[8][w1 >> 24] ^
        T[7][w2 & 0xff] ^ T[6][(w2 >> 8) & 0xff] ^ T[5][(w2 >> 16) & 0xff] ^ T[4][w2 >> 24] ^
        T[3][w3 & 0xff] ^ T[2][(w3 >> 8) & 0xff] ^ T[1][(w3 >> 16) & 0xff] ^ T[0][w3 >> 24];
    p += 16;
    n -= 16;
  }
  while (n--) c = (c >> 8) ^ T[0][(c ^ *p++) & 0xff];
  return ~c;
}

#if defined(__x86_64__)
/* ---- SSE4.2 crc32 instruction (snap's CRC-32C hardware path) ---- */
__attribute__((target("sse4.2"))) uint32_t orc_crc_sse42(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = ~crc;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  while (n--) c = _mm_crc32_u8((uint32_t)c, *p++);
  return ~(uint32_t)c;
}

/* ---- PCLMULQDQ folding for CRC-32/ISO-HDLC (crc32fast's x86 path; Gopal et al., "Fast CRC
 * computation for generic polynomials using PCLMULQDQ", fold-by-4 then Barrett reduction) ---- */
#define K1 0x154442bd4ull
#define K2 0x1c6e41596ull
#define K3 0x1751997d0ull
#define K4 0x0ccaa009eull
#define K5 0x163cd6124ull
#define P_X 0x1DB710641ull
#define U_PRIME 0x1F7011641ull

__attribute__((target("sse4.1,pclmul"))) static __m128i fold_16(__m128i x, __m128i data, __m128i k) {
  __m128i h = _mm_clmulepi64_si128(x, k, 0x11);
  __m128i l = _mm_clmulepi64_si128(x, k, 0x00);
  return _mm_xor_si128(_mm_xor_si128(h, l), data);
}

__attribute__((target("sse4.1,pclmul"))) uint32_t orc_crc_pclmul(uint32_t crc, const uint8_t* p, size_t n) {
  if (n < 128) return orc_crc_s16(0, crc, p, n);
  uint32_t c = ~crc;
  __m128i x0 = _mm_loadu_si128((const __m128i*)(p + 0x00));
  __m128i x1 = _mm_loadu_si128((const __m128i*)(p + 0x10));
  __m128i x2 = _mm_loadu_si128((const __m128i*)(p + 0x20));
  __m128i x3 = _mm_loadu_si128((const __m128i*)(p + 0x30));
  x0 = _mm_xor_si128(x0, _mm_cvtsi32_si128((int)c));
  p += 64;
  n -= 64;
  __m128i k = _mm_set_epi64x((long long)K2, (long long)K1);
  while (n >= 64) {
    x0 = fold_16(x0, _mm_loadu_si128((const __m128i*)(p + 0x00)), k);
    x1 = fold_16(x1, _mm_loadu_si128((const __m128i*)(p + 0x10)), k);
    x2 = fold_16(x2, _mm_loadu_si128((const __m128i*)(p + 0x20)), k);
    x3 = fold_16(x3, _mm_loadu_si128((const __m128i*)(p + 0x30)), k);
    p += 64;
    n -= 64;
  }
  k = _mm_set_epi64x((long long)K4, (long long)K3);
  __m128i x = fold_16(x0, x1, k);
  x = fold_16(x, x2, k);
  x = fold_16(x, x3, k);
  while (n >= 16) {
    x = fold_16(x, _mm_loadu_si128((const __m128i*)p), k);
    p += 16;
    n -= 16;
  }
  /* 128 -> 64 bits */
  const __m128i lo32 = _mm_set_epi32(0, 0, 0, -1);
  x = _mm_xor_si128(_mm_clmulepi64_si128(x, k, 0x10), _mm_srli_si128(x, 8));
  x = _mm_xor_si128(_mm_clmulepi64_si128(_mm_and_si128(x, lo32), _mm_set_epi64x(0, (long long)K5), 0x00),
                    _mm_srli_si128(x, 4));
  /* Barrett reduction 64 -> 32 */
  const __m128i pu = _mm_set_epi64x((long long)U_PRIME, (long long)P_X);
  __m128i t1 = _mm_clmulepi64_si128(_mm_and_si128(x, lo32), pu, 0x10);
  __m128i t2 = _mm_clmulepi64_si128(_mm_and_si128(t1, lo32), pu, 0x00);
  c = (uint32_t)_mm_extract_epi32(_mm_xor_si128(x, t2), 1);
  return orc_crc_s16(0, ~c, p, n);
}
#else
uint32_t orc_crc_sse42(uint32_t crc, const uint8_t* p, size_t n) { return orc_crc_s16(1, crc, p, n); }
uint32_t orc_crc_pclmul(uint32_t crc, const uint8_t* p, size_t n) { return orc_crc_s16(0, crc, p, n); }
#endif

/* ---- per-block batch (for golden vectors and the CPU baseline) ---- */
/* algo: 0 = bitwise REF, 1 = bitwise C, 2 = slice16 REF, 3 = slice16 C, 4 = pclmul REF, 5 = sse42 C */
static uint32_t crc_algo(int algo, const uint8_t* p, size_t n) {
  switch (algo) {
    case 0: return orc_crc_bitwise(ORC_POLY_REF, 0xFFFFFFFFu, 0xFFFFFFFFu, p, n);
    case 1: return orc_crc_bitwise(ORC_POLY_C, 0xFFFFFFFFu, 0xFFFFFFFFu, p, n);
    case 2: return orc_crc_s16(0, 0, p, n);
    case 3: return orc_crc_s16(1, 0, p, n);
    case 4: return orc_crc_pclmul(0, p, n);
    default: return orc_crc_sse42(0, p, n);
  }
}

/* CRC of ranges [offs[i], offs[i]+lens[i]) of base */
void orc_crc_ranges(int algo, const uint8_t* base, const uint64_t* offs, const uint32_t* lens, size_t n, uint32_t* out) {
  for (size_t i = 0; i < n; ++i) out[i] = crc_algo(algo, base + offs[i], lens[i]);
}

typedef struct {
  int algo;
  const uint8_t* base;
  size_t first, count, blen, stride;
  uint32_t* out;
} job_t;

static void* run_job(void* a) {
  job_t* j = (job_t*)a;
  for (size_t i = 0; i < j->count; ++i) j->out[j->first + i] = crc_algo(j->algo, j->base + (j->first + i) * j->stride, j->blen);
  return 0;
}

/* Uniform blocks with `threads` POSIX threads, blocks partitioned evenly; returns wall seconds. */
double orc_crc_uniform_mt(int algo, const uint8_t* base, size_t nblocks, size_t blen, size_t stride, int threads,
                          uint32_t* out) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  job_t jobs[256];
  s16_init(); /* tables built before any thread reads them */
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  size_t per = nblocks / (size_t)threads, rem = nblocks % (size_t)threads, first = 0;
  for (int t = 0; t < threads; ++t) {
    size_t cnt = per + ((size_t)t < rem ? 1 : 0);
    jobs[t] = (job_t){algo, base, first, cnt, blen, stride, out};
    first += cnt;
    pthread_create(&th[t], 0, run_job, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], 0);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

typedef struct {
  int algo;
  const uint8_t* base;
  const uint64_t* offs;
  const uint32_t* lens;
  size_t first, count;
  uint32_t* out;
} rjob_t;

static void* run_rjob(void* a) {
  rjob_t* j = (rjob_t*)a;
  for (size_t i = j->first; i < j->first + j->count; ++i) j->out[i] = crc_algo(j->algo, j->base + j->offs[i], j->lens[i]);
  return 0;
}

/* Arbitrary ranges (SSTable blocks of mixed sizes, WAL records) with `threads` POSIX threads, the ranges split
   into contiguous shares of about equal byte counts; returns wall seconds. */
double orc_crc_ranges_mt(int algo, const uint8_t* base, const uint64_t* offs, const uint32_t* lens, size_t n,
                         int threads, uint32_t* out) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  rjob_t jobs[256];
  s16_init();
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i) total += lens[i];
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  size_t first = 0;
  uint64_t acc = 0;
  int started = 0;
  for (int t = 0; t < threads && first < n; ++t) {
    const uint64_t goal = total / (uint64_t)threads * (uint64_t)(t + 1);
    size_t last = first;
    while (last < n && (acc < goal || t == threads - 1)) acc += lens[last++];
    if (last == first) last = first + 1, acc += lens[first];
    jobs[t] = (rjob_t){algo, base, offs, lens, first, last - first, out};
    first = last;
    pthread_create(&th[t], 0, run_rjob, &jobs[t]);
    ++started;
  }
  for (int t = 0; t < started; ++t) pthread_join(th[t], 0);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* splitmix64 byte stream (SURVEY.md 8c/8d synthetic inputs): s += 0x9E3779B97F4A7C15, mix, 8 LE bytes */
void orc_splitmix_fill(uint64_t seed, uint8_t* out, size_t n) {
  uint64_t s = seed;
  size_t i = 0;
  while (i < n) {
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    for (int k = 0; k < 8 && i < n; ++k, ++i) out[i] = (uint8_t)(z >> (8 * k));
  }
}

/* ---- read_block_from_file over a table's blocks (format.rs:146-213): the table-scan CPU baseline ----
   Block i: content [offs[i], offs[i] + sizes[i]), then its type byte and the stored trailer (crc32fast over
   content || type, table.rs:519-522). The trailer CRC (algo) is compared; a Snappy-framed block (type 1) is then
   walked, every data chunk decoded (raw Snappy) and its masked CRC-32C compared with the stored one, as the snap
   crate's FrameDecoder does (format.rs:194-206). status: 0 ok, 1 checksum mismatch, 3 bad content, 4 bad type
   (lcrc.h LCRC_TBLK_*). */
static int snappy_raw(const uint8_t* p, size_t n, uint8_t* out, size_t ulen) {
  size_t q = 0, w = 0;
  while (q < n) {
    const uint32_t t = p[q++];
    size_t len, off;
    if ((t & 3) == 0) {
      len = t >> 2;
      if (len >= 60) {
        const size_t nb = len - 59;
        if (n - q < 4) return 1; /* snap's read_literal: 4 input bytes after the tag whatever nb is */
        len = 0;
        for (size_t k = 0; k < nb; ++k) len |= (size_t)p[q + k] << (8 * k);
        q += nb;
      }
      len += 1;
      if (n - q < len || ulen - w < len) return 1;
      memcpy(out + w, p + q, len);
      q += len;
      w += len;
      continue;
    }
    if ((t & 3) == 1) {
      if (n - q < 1) return 1;
      len = 4 + ((t >> 2) & 7);
      off = ((size_t)(t >> 5) << 8) | p[q];
      q += 1;
    } else if ((t & 3) == 2) {
      if (n - q < 2) return 1;
      len = 1 + (t >> 2);
      off = p[q] | ((size_t)p[q + 1] << 8);
      q += 2;
    } else {
      if (n - q < 4) return 1;
      len = 1 + (t >> 2);
      off = p[q] | ((size_t)p[q + 1] << 8) | ((size_t)p[q + 2] << 16) | ((size_t)p[q + 3] << 24);
      q += 4;
    }
    if (off == 0 || off > w || ulen - w < len) return 1;
    if (off >= len) {  /* no overlap: one copy (the snap crate copies in wide words too) */
      memcpy(out + w, out + w - off, len);
      w += len;
    } else {
      for (size_t k = 0; k < len; ++k, ++w) out[w] = out[w - off];
    }
  }
  return w != ulen;
}

static int frame_check(const uint8_t* p, size_t n, uint8_t* scratch) {
  size_t at = 0;
  int seen_id = 0;
  while (at < n) {
    if (n - at < 4) return 1;
    const uint32_t type = p[at];
    const size_t cl = p[at + 1] | ((size_t)p[at + 2] << 8) | ((size_t)p[at + 3] << 16);
    at += 4;
    if (n - at < cl || cl > 76490) return 1; /* snap: MAX_COMPRESS_BLOCK_SIZE, any chunk type */
    const uint8_t* b = p + at;
    at += cl;
    if (type == 0xff) {
      if (cl != 6 || memcmp(b, "sNaPpY", 6) != 0) return 1;
      seen_id = 1;
    } else if (!seen_id) {
      return 1;
    } else if (type <= 1) {
      if (cl < 4) return 1;
      const uint32_t want = b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
      const uint8_t* data;
      size_t ulen;
      if (type == 1) {
        data = b + 4;
        ulen = cl - 4;
      } else {
        /* the preamble as snap's bytes::read_varu64: up to 10 bytes, the value mod 2^64 */
        size_t q = 4;
        uint64_t v = 0;
        int sh = 0, done = 0;
        while (q < cl && sh <= 63) {
          const uint32_t c = b[q++];
          v |= (uint64_t)(c & 127) << sh;
          sh += 7;
          if (!(c & 128)) {
            done = 1;
            break;
          }
        }
        if (!done || v > 65536 || snappy_raw(b + q, cl - q, scratch, v)) return 1;
        data = scratch;
        ulen = v;
      }
      if (ulen > 65536 || orc_mask(orc_crc_sse42(0, data, ulen)) != want) return 1;
    } else if (type <= 0x7f) {
      return 1; /* reserved unskippable */
    }
  }
  return 0;
}

typedef struct {
  int algo;
  const uint8_t* file;
  const uint64_t *offs, *sizes;
  size_t first, count;
  uint32_t* crc;
  uint8_t* status;
} tjob_t;

static void* run_tjob(void* a) {
  tjob_t* j = (tjob_t*)a;
  uint8_t* scratch = (uint8_t*)malloc(65536 + 64);
  for (size_t i = j->first; i < j->first + j->count; ++i) {
    const uint8_t* b = j->file + j->offs[i];
    const size_t n = j->sizes[i];
    const uint32_t c = crc_algo(j->algo, b, n + 1);
    const uint32_t want = b[n + 1] | ((uint32_t)b[n + 2] << 8) | ((uint32_t)b[n + 3] << 16) | ((uint32_t)b[n + 4] << 24);
    uint8_t st = c != want;
    if (!st && b[n] > 1) st = 4;
    if (!st && b[n] == 1 && frame_check(b, n, scratch)) st = 3;
    j->crc[i] = c;
    j->status[i] = st;
  }
  free(scratch);
  return 0;
}

/* `threads` POSIX threads over contiguous shares of about equal stored bytes; returns wall seconds. */
double orc_table_blocks_mt(int algo, const uint8_t* file, const uint64_t* offs, const uint64_t* sizes, size_t n,
                           int threads, uint32_t* crc_out, uint8_t* status_out) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  tjob_t jobs[256];
  s16_init();
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i) total += sizes[i] + 1;
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  size_t first = 0;
  uint64_t acc = 0;
  int started = 0;
  for (int t = 0; t < threads && first < n; ++t) {
    const uint64_t goal = total / (uint64_t)threads * (uint64_t)(t + 1);
    size_t last = first;
    while (last < n && (acc < goal || t == threads - 1)) acc += sizes[last++] + 1;
    if (last == first) last = first + 1, acc += sizes[first] + 1;
    jobs[t] = (tjob_t){algo, file, offs, sizes, first, last - first, crc_out, status_out};
    first = last;
    pthread_create(&th[t], 0, run_tjob, &jobs[t]);
    ++started;
  }
  for (int t = 0; t < started; ++t) pthread_join(th[t], 0);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
