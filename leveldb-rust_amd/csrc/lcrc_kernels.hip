// gfx950 (MI355X / CDNA4) kernels of the block/record checksum engine.
//
// Algorithm (see DESIGN.md for the derivation and the rooflines):
//   * A CRC register walk is linear: walk(r, M) = Z_|M|(r) ^ walk(0, M), Z_n = "advance over n zero
//     bytes" = multiplication by x^(8n) mod P. So any split of a byte range into pieces can be walked
//     independently and recombined with fixed shift operators.
//   * k_windows (the hot kernel) streams the buffer in 16 KiB wave tiles with fully coalesced 16 B/lane
//     buffer loads (1 KiB per wave instruction), transposes the 16 loaded pieces inside each 16-lane DPP
//     row so that every lane owns one contiguous 256 B window, and walks the window with slice-by-4
//     lookups into LDS tables replicated 32x (one replica per bank -> conflict-free ds_read_b32).
//     It emits the raw register value of every 256 B window (general path) or, for the uniform
//     4 KiB layout, folds the 16 windows of each 4 KiB block with a 4-level lane tree and writes the
//     final (optionally masked, optionally verified) CRC directly.
//   * k_blocks finishes arbitrary ranges from the window values: each 16-lane row owns one range, walks
//     its partial head/tail windows from the data, and folds the full windows in between.
//   * k_wal_parse walks the 7-byte headers of every 32 KiB log block (src/db/log.rs:204-279) into
//     record descriptors for k_blocks.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lcrc_device.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// Unaligned 16-byte view: gfx950 global/buffer loads accept any byte alignment (unaligned access mode
// is enabled by the ROCm runtime); this type only tells the compiler to emit one dwordx4.
typedef u32x4 u32x4_ua __attribute__((aligned(1)));

namespace lcrc_dev {

// ---------------------------------------------------------------------------------------------------
// k_windows LDS image (static, 152 KiB -> one 1024-thread workgroup per CU):
//   [0, 128 KiB): slice-by-4 tables T0..T3, 256 entries each, 32 replicas. Table t lives in region
//                 t>>1 (64 KiB each); entry e of that region is a 256 B row holding table 2*region's
//                 32 replicas in its first 128 B and table 2*region+1's in the second. Lane l reads
//                 replica l&31 -> bank (l&31): the 32 lanes of each ds_read_b32 half-wave group never
//                 conflict. The byte address of (t, e, l) = (t>>1)<<16 | e<<8 | (t&1)<<7 | (l&31)<<2,
//                 built with ONE v_perm_b32 from a per-lane base and the data byte.
//   [128 KiB, 152 KiB): byte-sliced shift tables Z64 (chain join), Z128 .. Z2048 (window tree),
//                 unreplicated: they serve a few lookups per tile.
// ---------------------------------------------------------------------------------------------------
constexpr int A_SLICE_BYTES = 131072;
constexpr int A_Z64 = A_SLICE_BYTES;       // Z64, then Z128, Z256, Z512, Z1024, Z2048 at +4 KiB steps
constexpr int A_ZTREE = A_Z64 + 4096;      // Z128 .. Z2048: level m of the tree shifts 128 << m bytes
constexpr int A_LDS_BYTES = A_Z64 + 6 * 4096;
#ifndef LCRC_A_THREADS
#define LCRC_A_THREADS 1024
#endif
constexpr int A_THREADS = LCRC_A_THREADS;
constexpr int TILE = 8192;  // bytes per wave tile (8 loads x 64 lanes x 16 B)

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops (lgkmcnt(0)) but not for its
// outstanding global loads -- __syncthreads() would add vmcnt(0) and expose the first tile's latency.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
}

__device__ __forceinline__ uint32_t lds_u32(const void* lds_base, uint32_t byte_addr) {
  return *(const uint32_t*)((const char*)lds_base + byte_addr);
}

// v_perm_b32 selector building the table address from base (S0) and data byte k of x (S1):
// out = { 0x00, base.b2, x.bk, base.b0 }
template <int K>
__device__ __forceinline__ uint32_t tab_addr(uint32_t base, uint32_t x) {
  return __builtin_amdgcn_perm(base, x, 0x0C060004u | (K << 8));
}

// a ^ b ^ c in one gfx950 v_bitop3_b32 (truth table 0x96); gfx9 has no v_xor3
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// one slice-by-4 step on x = r ^ w (already folded); returns walk(r, w) ^ w_next
__device__ __forceinline__ uint32_t step4x(const void* L, uint32_t x, uint32_t w_next, uint32_t b0, uint32_t b1,
                                           uint32_t b2, uint32_t b3) {
  uint32_t t3 = lds_u32(L, tab_addr<0>(b3, x));
  uint32_t t2 = lds_u32(L, tab_addr<1>(b2, x));
  uint32_t t1 = lds_u32(L, tab_addr<2>(b1, x));
  uint32_t t0 = lds_u32(L, tab_addr<3>(b0, x));
  return xor3(xor3(t0, t1, w_next), t2, t3);
}

// In-register transpose. Lane l = 8*c + k (k = l & 7, c = l >> 3) loads, in instruction j, the 16 B piece
// at tile byte 1024*j + 128*k + 16*c (each instruction still reads one contiguous 1 KiB). Within each group
// k the 8 lanes c and 8 registers j form an 8x8 matrix of pieces; transposing it gives lane (k, c) the
// pieces at 1024*c + 128*k + 16*j', j' = 0..7: one contiguous 128 B window whose index inside the tile is
// 8*c + k = l. The three butterfly stages run over lane bits 3..5:
//   bit 3: v_mov_b32_dpp row_shr:8 / row_shl:8 with a bank_mask -- disabled banks keep `old`, so the DPP
//          move is also the select (one instruction per register)
//   bit 4: v_permlane16_swap (odd rows of a <-> even rows of b), bit 5: v_permlane32_swap (one
//          instruction per register pair)
template <int LB>
__device__ __forceinline__ void transpose_stage(u32x4 (&v)[8]) {
  constexpr int D = 1 << (LB - 3);  // register-index bit paired with lane bit LB
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (j & D) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t a = v[j][q], b = v[j + D][q];
      if constexpr (LB == 3) {
        // lanes 8..15 of each row (banks 2, 3) have bit 3 set
        uint32_t na = (uint32_t)__builtin_amdgcn_update_dpp((int)a, (int)b, 0x118, 0xF, 0xC, false);
        uint32_t nb = (uint32_t)__builtin_amdgcn_update_dpp((int)b, (int)a, 0x108, 0xF, 0x3, false);
        v[j][q] = na;
        v[j + D][q] = nb;
      } else if constexpr (LB == 4) {
        auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
        v[j][q] = r[0];
        v[j + D][q] = r[1];
      } else {
        auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
        v[j][q] = r[0];
        v[j + D][q] = r[1];
      }
    }
  }
}

__device__ __forceinline__ uint32_t zlook(const void* L, uint32_t tab_byte_off, uint32_t r) {
  const char* z = (const char*)L + tab_byte_off;
  return *(const uint32_t*)(z + ((r & 0xff) << 2)) ^ *(const uint32_t*)(z + 1024 + (((r >> 8) & 0xff) << 2)) ^
         *(const uint32_t*)(z + 2048 + (((r >> 16) & 0xff) << 2)) ^ *(const uint32_t*)(z + 3072 + ((r >> 24) << 2));
}

// one level of the window tree: lane g (g % 2^(M+1) == 0) <- Z_{128*2^M}(p_g) ^ p_{g+2^M}. Only the
// combining lanes look up (exec-masked ds_reads: fewer bank conflicts on the unreplicated tables).
template <int M>
__device__ __forceinline__ uint32_t tree_level(const void* L, uint32_t p, uint32_t lane) {
  uint32_t pn;
  if constexpr (M < 4)
    pn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)p, 0x100 + (1 << M), 0xF, 0xF, false);  // row_shl
  else
    pn = __shfl_down(p, 1 << M, 64);
  if ((lane & ((2u << M) - 1)) == 0) p = zlook(L, A_ZTREE + M * 4096, p) ^ pn;
  return p;
}

__device__ __forceinline__ uint32_t mask32c(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }

// wave-uniform descriptor for tile t: loads past the end of the span (or of a non-existent tile) return 0
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const uint8_t* base, uint64_t span, uint64_t t,
                                                            uint64_t ntiles) {
  uint32_t nrec = 0;
  uint64_t toff = 0;
#ifdef LCRC_PROBE_NOLOAD  // ablation build: no memory traffic, loads return zeros
  ntiles = 0;
#endif
  if (t < ntiles) {
#ifdef LCRC_PROBE_L2  // ablation build: every tile aliases one of the first 64 (512 KiB, L2-resident)
    toff = (t & 63) * (uint64_t)TILE;
#else
    toff = t * (uint64_t)TILE;
#endif
    const uint64_t rem = span - toff;
    nrec = rem < (uint64_t)TILE ? (uint32_t)rem : (uint32_t)TILE;
  }
  return __builtin_amdgcn_make_buffer_rsrc((void*)(base + toff), (short)0, (int)nrec, 0x00020000);
}

#ifdef LCRC_PROBE_LDSDATA  // ablation build: random data from an 8 KiB LDS tile, no VMEM at all
__shared__ u32x4 lcrc_probe_tile[512];
#define LCRC_REFILL(rs, off) (lcrc_probe_tile[((off) >> 4) & 511])
#else
#define LCRC_REFILL(rs, off) __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, LCRC_LOAD_AUX)
#endif

__device__ __forceinline__ void load_tile(u32x4 (&v)[8], __amdgpu_buffer_rsrc_t rs, uint32_t voff) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = LCRC_REFILL(rs, voff + j * 1024);
}

// Transpose + walk one tile already in registers; returns walk(0, window l) of this lane (128 B).
// As each register pair is consumed it is refilled from `rs` (the tile after next), so every wave keeps
// between one and two tiles of loads in flight while it computes.
__device__ __forceinline__ uint32_t walk_tile(const void* L, u32x4 (&v)[8], uint32_t b0, uint32_t b1, uint32_t b2,
                                              uint32_t b3, __amdgpu_buffer_rsrc_t rs, uint32_t voff) {
  transpose_stage<3>(v);
  transpose_stage<4>(v);
  transpose_stage<5>(v);
#ifdef LCRC_PROBE_NOWALK  // ablation build: fold the data with xor only
  uint32_t p = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    p ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    v[j] = LCRC_REFILL(rs, voff + j * 1024);
  }
  return p;
#else
  // two independent chains over the 64 B halves (pieces 0..3 and 4..7); x carries the chain register
  // already xored with its next data word
  uint32_t xa = v[0].x, xb = v[4].x;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    xa = step4x(L, xa, v[j].y, b0, b1, b2, b3);
    xb = step4x(L, xb, v[4 + j].y, b0, b1, b2, b3);
    xa = step4x(L, xa, v[j].z, b0, b1, b2, b3);
    xb = step4x(L, xb, v[4 + j].z, b0, b1, b2, b3);
    xa = step4x(L, xa, v[j].w, b0, b1, b2, b3);
    xb = step4x(L, xb, v[4 + j].w, b0, b1, b2, b3);
    xa = step4x(L, xa, j < 3 ? v[j + 1].x : 0u, b0, b1, b2, b3);
    xb = step4x(L, xb, j < 3 ? v[5 + j].x : 0u, b0, b1, b2, b3);
    v[j] = LCRC_REFILL(rs, voff + j * 1024);
    v[4 + j] = LCRC_REFILL(rs, voff + (4 + j) * 1024);
    __builtin_amdgcn_sched_barrier(0);  // keep the refill here: hipcc would otherwise sink it past the walk
  }
  return zlook(L, A_Z64, xa) ^ xb;
#endif
}

// FINAL = false: out[t*32 + w] = walk(0, 256 B window w of tile t) (raw partials for k_blocks)
// FINAL = true : span = nblk * 4096; out[b] = crc of 4 KiB block b (xor fin, optional mask, verify)
template <bool FINAL>
__device__ __forceinline__ void finish_tile(const void* L, uint32_t p, uint64_t t, uint32_t lane,
                                           uint32_t* __restrict__ out, uint64_t nblk, uint32_t fin, uint32_t flags,
                                           const uint32_t* __restrict__ expected, uint32_t* __restrict__ mismatch) {
  p = tree_level<0>(L, p, lane);  // 128 B windows -> 256 B windows
  if (!FINAL) {
    if ((lane & 1) == 0) out[t * 32 + (lane >> 1)] = p;
    return;
  }
  p = tree_level<1>(L, p, lane);
  p = tree_level<2>(L, p, lane);
  p = tree_level<3>(L, p, lane);
  p = tree_level<4>(L, p, lane);
  const uint64_t blk = t * 2 + (lane >> 5);
  if ((lane & 31) == 0 && blk < nblk) {
    uint32_t crc = p ^ fin;
    if (flags & LCRC_FLAG_MASK) crc = mask32c(crc);
    out[blk] = crc;
    if (expected && expected[blk] != crc) atomicOr(&mismatch[blk >> 5], 1u << (blk & 31));
  }
}

#ifdef LCRC_PROBE_CLOCK  // diagnostic build: per-workgroup shader/real clock stamps around the tile loop
__device__ unsigned long long lcrc_dbg_clock[4096];
#endif

template <bool FINAL>
__global__ void __launch_bounds__(A_THREADS) k_windows(const uint8_t* __restrict__ base, uint64_t span,
                                                      uint64_t ntiles, const uint32_t* __restrict__ gtab,
                                                      uint32_t* __restrict__ out, uint64_t nblk, uint32_t fin,
                                                      uint32_t flags, const uint32_t* __restrict__ expected,
                                                      uint32_t* __restrict__ mismatch) {
  __shared__ __attribute__((aligned(16))) uint32_t L[A_LDS_BYTES / 4];
  const uint32_t lane = __lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * (A_THREADS / 64);
  uint64_t t = (uint64_t)blockIdx.x * (A_THREADS / 64) + wave;
#ifdef LCRC_PROBE_LDSDATA
  for (uint32_t i = threadIdx.x; i < 512; i += A_THREADS) {
    uint32_t h = i * 0x9E3779B9u + blockIdx.x * 0x85EBCA6Bu;
    h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12;
    lcrc_probe_tile[i] = u32x4{h, h * 0x27D4EB2Fu, h ^ 0x165667B1u, h * 0x94D049BBu};
  }
  __syncthreads();
#endif
  // lane (k, c) = (lane & 7, lane >> 3) reads piece 8*k + c of every 1 KiB of the tile
  const uint32_t voff = 16u * (8u * (lane & 7) + (lane >> 3));

  // two register tiles: while one is transposed and walked, the next one is in flight
  u32x4 va[8], vb[8];
  load_tile(va, tile_rsrc(base, span, t, ntiles), voff);  // before the LDS fill: HBM streams meanwhile

  {
    // Table image in one global round trip: every thread issues its loads up front.
    //   slice T0..T3 (4 KiB)   -> staged in the Z-table area, then replicated 32x LDS->LDS
    //   Z64, Z128..Z2048 (24 KiB) -> held in registers until the staging area is free again
    const uint32_t tid = threadIdx.x;
    const u32x4* gsl = (const u32x4*)(gtab + TAB_SLICE);
    const u32x4* gz64 = (const u32x4*)(gtab + TAB_ZPIECE + 2 * 1024);  // Z64, Z128 (adjacent)
    const u32x4* gzw = (const u32x4*)(gtab + TAB_ZWIN);                // Z256 .. Z2048
    u32x4 sl = {0, 0, 0, 0}, za = {0, 0, 0, 0};
    if (tid < 256) sl = gsl[tid];
    if (tid < 512) za = gz64[tid];
    const u32x4 zb = gzw[tid];
    if (tid < 256) *(u32x4*)((char*)L + A_Z64 + (tid << 4)) = sl;
    lds_barrier();
    const uint32_t* stage = (const uint32_t*)((const char*)L + A_Z64);
#pragma unroll
    for (int k = 0; k < A_SLICE_BYTES / 16 / A_THREADS; ++k) {
      const uint32_t off = (tid + k * A_THREADS) << 4;
      const uint32_t tbl = ((off >> 16) << 1) | ((off >> 7) & 1);
      const uint32_t val = stage[tbl * 256 + ((off >> 8) & 255)];
      *(u32x4*)((char*)L + off) = u32x4{val, val, val, val};
    }
    lds_barrier();
    if (tid < 512) *(u32x4*)((char*)L + A_Z64 + (tid << 4)) = za;
    *(u32x4*)((char*)L + A_Z64 + 8192 + (tid << 4)) = zb;
  }
  lds_barrier();

  const uint32_t rep = (lane & 31) << 2;
  const uint32_t b0 = rep, b1 = (1u << 7) | rep, b2 = (1u << 16) | rep, b3 = (1u << 16) | (1u << 7) | rep;
#ifdef LCRC_PROBE_CLOCK
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#endif

  // va holds tile t, vb tile t + nwaves; walking a buffer refills it with the tile two steps ahead.
  // The steady-state loop walks both buffers (no early exit inside, so the compiler's vmcnt bookkeeping
  // sees one fixed issue order: each walk waits only for its own buffer); an odd tail tile follows.
  load_tile(vb, tile_rsrc(base, span, t + nwaves, ntiles), voff);
  for (; t + nwaves < ntiles; t += 2 * nwaves) {
    __builtin_amdgcn_sched_barrier(0);
    uint32_t p = walk_tile(L, va, b0, b1, b2, b3, tile_rsrc(base, span, t + 2 * nwaves, ntiles), voff);
    finish_tile<FINAL>(L, p, t, lane, out, nblk, fin, flags, expected, mismatch);
    __builtin_amdgcn_sched_barrier(0);
    p = walk_tile(L, vb, b0, b1, b2, b3, tile_rsrc(base, span, t + 3 * nwaves, ntiles), voff);
    finish_tile<FINAL>(L, p, t + nwaves, lane, out, nblk, fin, flags, expected, mismatch);
  }
  if (t < ntiles) {
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t p = walk_tile(L, va, b0, b1, b2, b3, tile_rsrc(base, span, ntiles, ntiles), voff);
    finish_tile<FINAL>(L, p, t, lane, out, nblk, fin, flags, expected, mismatch);
  }
#ifdef LCRC_PROBE_CLOCK
  const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x < 1024) {
    lcrc_dbg_clock[blockIdx.x * 4 + 0] = c1 - c0;
    lcrc_dbg_clock[blockIdx.x * 4 + 1] = r1 - r0;
  }
#endif
}

// ---------------------------------------------------------------------------------------------------
// k_blocks: one 16-lane row per range. LDS (40 KiB): T0..T3 [4 KiB], Z16..Z128 [16 KiB],
// Z256..Z2048 [16 KiB], Z4096 [4 KiB], unreplicated (the hot loop is in k_windows).
// ---------------------------------------------------------------------------------------------------
constexpr int B_THREADS = 256;
constexpr int B_LDS_DWORDS = TAB_TOTAL;

__device__ __forceinline__ uint32_t byte_step(const uint32_t* L, uint32_t r, uint32_t b) {
  return (r >> 8) ^ L[TAB_SLICE + ((r ^ b) & 0xff)];
}
__device__ __forceinline__ uint32_t step4(const uint32_t* L, uint32_t r, uint32_t w) {
  uint32_t x = r ^ w;
  return L[TAB_SLICE + 768 + (x & 0xff)] ^ L[TAB_SLICE + 512 + ((x >> 8) & 0xff)] ^
         L[TAB_SLICE + 256 + ((x >> 16) & 0xff)] ^ L[TAB_SLICE + (x >> 24)];
}
__device__ __forceinline__ uint32_t zl(const uint32_t* L, int off, uint32_t r) {
  return L[off + (r & 0xff)] ^ L[off + 256 + ((r >> 8) & 0xff)] ^ L[off + 512 + ((r >> 16) & 0xff)] ^
         L[off + 768 + (r >> 24)];
}

// Returns walk(R0, base[a, e)) for 0 <= e - a <= 256 to every lane of the 16-lane row (g = lane in row).
// Pieces are aligned to END at e: piece g covers [e - 16*(16-g), e - 16*(15-g)).
// Must be called by all 64 lanes (contains cross-lane ops).
__device__ uint32_t row_walk(const uint32_t* L, const uint8_t* __restrict__ base, uint64_t a, uint64_t e,
                             uint32_t R0, uint32_t g, uint32_t lane) {
  const int64_t pe = (int64_t)e - 16 * (15 - (int)g);
  const int64_t ps = pe - 16;
  uint32_t cv = 0;
  if (pe > (int64_t)a) {
    if (ps >= (int64_t)a) {
      u32x4 w = *(const u32x4_ua*)(base + ps);
      uint32_t rr = (ps == (int64_t)a) ? R0 : 0u;
      rr = step4(L, rr, w.x);
      rr = step4(L, rr, w.y);
      rr = step4(L, rr, w.z);
      rr = step4(L, rr, w.w);
      cv = rr;
    } else {
      // straddle: bytes [a, pe) (1..15 of them), walked from R0 at a
      uint32_t rr = R0;
      const uint32_t first = (uint32_t)((int64_t)a - ps);
#pragma unroll
      for (int i = 1; i < 16; ++i) {
        if ((uint32_t)i >= first) rr = byte_step(L, rr, base[ps + i]);
      }
      cv = rr;
    }
  }
  // row tree: level m joins lane g with g + 2^m, shifting the left part by 16*2^m bytes
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    uint32_t pn = __shfl_down(cv, 1 << m, 16);
    uint32_t sh = zl(L, TAB_ZPIECE + m * 1024, cv);
    if ((g & ((2u << m) - 1)) == 0) cv = sh ^ pn;
  }
  uint32_t res = __shfl(cv, lane & ~15u, 64);
  return (a == e) ? R0 : res;
}

__device__ __forceinline__ uint32_t load_le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

template <bool UNIFORM>
__global__ void __launch_bounds__(B_THREADS) k_blocks(const uint8_t* __restrict__ base, uint64_t base_len,
                                                     const lcrc_desc_dev* __restrict__ descs, uint64_t n,
                                                     uint64_t ustride, uint32_t ulen,
                                                     const uint32_t* __restrict__ uexp,
                                                     const uint32_t* __restrict__ win, const uint32_t* __restrict__ gtab,
                                                     uint32_t init, uint32_t xorout, uint32_t flags,
                                                     uint32_t* __restrict__ out, uint32_t* __restrict__ mismatch) {
  __shared__ uint32_t L[B_LDS_DWORDS];
  for (uint32_t i = threadIdx.x; i < B_LDS_DWORDS; i += B_THREADS) L[i] = gtab[i];
  __syncthreads();

  const uint32_t lane = __lane_id();
  const uint32_t g = lane & 15, row = lane >> 4;
  const uint64_t wave = (uint64_t)blockIdx.x * (B_THREADS / 64) + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * (B_THREADS / 64);
  const bool use_win = win != nullptr;

  for (uint64_t i0 = wave * 4; i0 < n; i0 += nwaves * 4) {
    const uint64_t i = i0 + row;
    const bool valid = i < n;
    uint64_t s = 0;
    uint32_t len = 0;
    int32_t xrel = LCRC_NO_EXPECT_DEV;
    if (valid) {
      if (UNIFORM) {
        s = i * ustride;
        len = ulen;
      } else {
        lcrc_desc_dev d = descs[i];
        s = d.offset;
        len = d.length;
        xrel = d.expect_rel;
      }
    }
    const uint64_t e = s + len;
    uint32_t acc;
    if (use_win) {
      const uint64_t ws = s >> 8;
      const uint64_t wl = len ? (e - 1) >> 8 : ws;
      const bool single = (ws == wl);
      const uint64_t head_end = single ? e : (ws + 1) << 8;
      const uint32_t head = row_walk(L, base, s, head_end, init, g, lane);
      // middle: virtual items [pad zeros..., head, win[ws+1 .. wfull]] folded 16 per round
      const uint64_t wfull = ((e & 255) == 0) ? wl : wl - 1;
      const uint64_t items = single ? 0 : (wfull - ws) + 1;  // head + full windows
      const uint64_t npad = (16 - (items & 15)) & 15;
      const uint64_t rounds = single ? 0 : (npad + items) >> 4;
      uint32_t rmax = (uint32_t)rounds;
      rmax = max(rmax, (uint32_t)__shfl_xor((int)rmax, 16, 64));
      rmax = max(rmax, (uint32_t)__shfl_xor((int)rmax, 32, 64));
      uint32_t a = 0;
      for (uint32_t q = 0; q < rmax; ++q) {
        const uint64_t u = 16 * q + g;
        uint32_t val = 0;
        if (q < rounds) {
          if (u >= npad) val = (u == npad) ? head : win[ws + (u - npad)];
          a = zl(L, TAB_Z4096, a) ^ val;
        }
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        uint32_t pn = __shfl_down(a, 1 << m, 16);
        uint32_t sh = zl(L, TAB_ZWIN + m * 1024, a);
        if ((g & ((2u << m) - 1)) == 0) a = sh ^ pn;
      }
      const uint32_t mid = __shfl(a, lane & ~15u, 64);
      acc = single ? head : mid;
      // tail: the partial last window, walked from the folded value
      const uint64_t ta = (single || (e & 255) == 0) ? e : (wl << 8);
      acc = row_walk(L, base, ta, e, acc, g, lane);
    } else {
      // direct: walk the whole range in 256 B chunks (sparse batches)
      uint32_t nch = (uint32_t)(((uint64_t)len + 255) >> 8);
      uint32_t cmax = nch;
      cmax = max(cmax, (uint32_t)__shfl_xor((int)cmax, 16, 64));
      cmax = max(cmax, (uint32_t)__shfl_xor((int)cmax, 32, 64));
      acc = init;
      for (uint32_t k = 0; k < cmax; ++k) {
        uint64_t ca = s + 256 * k;
        uint64_t ce = ca + 256 < e ? ca + 256 : e;
        if (k >= nch) ca = ce = e;
        acc = row_walk(L, base, ca, ce, acc, g, lane);
      }
    }
    if (valid && g == 0) {
      uint32_t crc = acc ^ xorout;
      if (flags & LCRC_FLAG_MASK) crc = mask32c(crc);
      out[i] = crc;
      bool bad = false;
      if (UNIFORM) {
        if (uexp) bad = uexp[i] != crc;
      } else if (xrel != LCRC_NO_EXPECT_DEV) {
        const int64_t xp = (int64_t)s + xrel;
        bad = (xp < 0 || (uint64_t)xp + 4 > base_len) ? true : load_le32(base + xp) != crc;
      }
      if (bad) atomicOr(&mismatch[i >> 5], 1u << (i & 31));
    }
  }
}

// ---------------------------------------------------------------------------------------------------
// k_wal_parse: one lane per 32 KiB log block, walking the record headers exactly as
// LogReader::read_physical_record (src/db/log.rs:204-279) does, minus the checksum (k_blocks computes
// it afterwards, in parallel over all records). Pass 1 (recs == nullptr) counts records per block;
// pass 2 writes them at the exclusive-scan offsets.
// ---------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_wal_parse(const uint8_t* __restrict__ file, uint64_t file_len,
                                                   uint64_t nblocks, uint32_t* __restrict__ counts,
                                                   const uint64_t* __restrict__ offsets,
                                                   lcrc_wal_rec_dev* __restrict__ recs,
                                                   lcrc_desc_dev* __restrict__ descs) {
  const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  const uint64_t bstart = b * 32768ull;
  const uint64_t rem = file_len - bstart;
  const uint32_t cap = rem < 32768ull ? (uint32_t)rem : 32768u;
  uint32_t consumed = 0;
  uint32_t nrec = 0;
  uint64_t o = recs ? offsets[b] : 0;
  uint32_t stop = LCRC_WAL_STOP_TRAILER_DEV;
  while (cap - consumed >= 7) {
    const uint8_t* h = file + bstart + consumed;
    const uint32_t length = (uint32_t)h[4] | ((uint32_t)h[5] << 8);
    const uint32_t type = h[6];
    if (7 + length > cap - consumed) {
      stop = LCRC_WAL_STOP_BAD_LENGTH_DEV;
      break;
    }
    if (type == 0 && length == 0) {
      stop = LCRC_WAL_STOP_ZERO_DEV;
      break;
    }
    if (recs) {
      lcrc_wal_rec_dev rr;
      rr.header = bstart + consumed;
      rr.length = length;
      rr.type = (uint8_t)type;
      rr.status = 0;
      rr.block_end = 0;
      rr.crc = 0;
      rr.stop = 0;
      recs[o] = rr;
      lcrc_desc_dev d;
      d.offset = bstart + consumed + 6;
      d.length = 1 + length;
      d.expect_rel = -6;
      descs[o] = d;
      ++o;
    }
    ++nrec;
    consumed += 7 + length;
  }
  if (!recs) {
    counts[b] = nrec;
  } else if (nrec) {
    recs[o - 1].block_end = 1;
    recs[o - 1].stop = stop;
  }
}

// Per-record verdicts from the k_blocks outputs; the first mismatch of a 32 KiB block ends the block
// (the reader drops the rest of it, log.rs:260-273): later records of that block are marked by stop.
__global__ void __launch_bounds__(256) k_wal_finish(lcrc_wal_rec_dev* __restrict__ recs, uint64_t n,
                                                    const uint32_t* __restrict__ crcs,
                                                    const uint32_t* __restrict__ mismatch) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  recs[i].crc = crcs[i];
  recs[i].status = (mismatch[i >> 5] >> (i & 31)) & 1;
}

}  // namespace lcrc_dev

// ---------------------------------------------------------------------------------------------------
// host-side launchers (called from lcrc_api.cpp)
// ---------------------------------------------------------------------------------------------------
extern "C" {

#ifdef LCRC_PROBE_CLOCK
// effective shader clock (MHz) of the last k_windows launch: median over workgroups of
// d(s_memtime) / d(s_memrealtime) * 100 MHz
double lcrc_probe_clock_mhz(int nwg) {
  static unsigned long long h[4096];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(lcrc_dev::lcrc_dbg_clock), sizeof(h)) != hipSuccess) return -1;
  double v[1024];
  int n = 0;
  for (int i = 0; i < nwg && i < 1024; ++i)
    if (h[i * 4 + 1]) v[n++] = 100.0 * (double)h[i * 4] / (double)h[i * 4 + 1];
  for (int i = 1; i < n; ++i)
    for (int j = i; j > 0 && v[j - 1] > v[j]; --j) {
      double t = v[j]; v[j] = v[j - 1]; v[j - 1] = t;
    }
  return n ? v[n / 2] : -1;
}
#endif

hipError_t lcrc_launch_windows(bool final_mode, int grid, const uint8_t* base, uint64_t span, const uint32_t* gtab,
                               uint32_t* out, uint64_t nblk, uint32_t fin, uint32_t flags,
                               const uint32_t* expected, uint32_t* mismatch, hipStream_t st) {
  const uint64_t ntiles = (span + lcrc_dev::TILE - 1) / lcrc_dev::TILE;
  if (ntiles == 0) return hipSuccess;
  uint64_t need = (ntiles + 15) / 16;
  int g = (int)(need < (uint64_t)grid ? need : (uint64_t)grid);
  if (final_mode)
    hipLaunchKernelGGL(lcrc_dev::k_windows<true>, dim3(g), dim3(lcrc_dev::A_THREADS), 0, st, base, span, ntiles, gtab,
                       out, nblk, fin, flags, expected, mismatch);
  else
    hipLaunchKernelGGL(lcrc_dev::k_windows<false>, dim3(g), dim3(lcrc_dev::A_THREADS), 0, st, base, span, ntiles,
                       gtab, out, nblk, fin, flags, expected, mismatch);
  return hipGetLastError();
}

hipError_t lcrc_launch_blocks(bool uniform, int grid, const uint8_t* base, uint64_t base_len,
                              const lcrc_desc_dev* descs, uint64_t n, uint64_t ustride, uint32_t ulen,
                              const uint32_t* uexp, const uint32_t* win, const uint32_t* gtab, uint32_t init,
                              uint32_t xorout, uint32_t flags, uint32_t* out, uint32_t* mismatch, hipStream_t st) {
  if (n == 0) return hipSuccess;
  uint64_t need = (n + 15) / 16;  // 16 ranges per 256-thread workgroup
  int g = (int)(need < (uint64_t)grid ? need : (uint64_t)grid);
  if (uniform)
    hipLaunchKernelGGL(lcrc_dev::k_blocks<true>, dim3(g), dim3(lcrc_dev::B_THREADS), 0, st, base, base_len, descs, n,
                       ustride, ulen, uexp, win, gtab, init, xorout, flags, out, mismatch);
  else
    hipLaunchKernelGGL(lcrc_dev::k_blocks<false>, dim3(g), dim3(lcrc_dev::B_THREADS), 0, st, base, base_len, descs,
                       n, ustride, ulen, uexp, win, gtab, init, xorout, flags, out, mismatch);
  return hipGetLastError();
}

hipError_t lcrc_launch_wal_parse(const uint8_t* file, uint64_t file_len, uint64_t nblocks, uint32_t* counts,
                                 const uint64_t* offsets, lcrc_wal_rec_dev* recs, lcrc_desc_dev* descs,
                                 hipStream_t st) {
  if (nblocks == 0) return hipSuccess;
  int g = (int)((nblocks + 255) / 256);
  hipLaunchKernelGGL(lcrc_dev::k_wal_parse, dim3(g), dim3(256), 0, st, file, file_len, nblocks, counts, offsets, recs,
                     descs);
  return hipGetLastError();
}

hipError_t lcrc_launch_wal_finish(lcrc_wal_rec_dev* recs, uint64_t n, const uint32_t* crcs, const uint32_t* mismatch,
                                  hipStream_t st) {
  if (n == 0) return hipSuccess;
  int g = (int)((n + 255) / 256);
  hipLaunchKernelGGL(lcrc_dev::k_wal_finish, dim3(g), dim3(256), 0, st, recs, n, crcs, mismatch);
  return hipGetLastError();
}

}  // extern "C"
