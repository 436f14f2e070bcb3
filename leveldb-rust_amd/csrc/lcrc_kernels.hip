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
//   * k_ranges does arbitrary ranges in one pass instead: 4 KiB chunks per 16-lane row with k_windows'
//     loads and walk, zero-padded by the buffer range check, the padding undone by one GF(2) multiply.
//   * Snappy framing: k_snappy_size (framing walk), k_snappy_decode_wave (one wave per frame, LDS-staged,
//     data-parallel element parse), k_snappy_check; table scan: k_idx_parse, k_tbl_finish, k_tbl_content
//     (host-walked index), and the device-only scan k_ts_open2 (a framed index), k_ts_windows (the window
//     pass with Table::open's index walk beside it), k_ts_finish, k_ts_decode.
//   * k_wal_parse walks the 7-byte headers of every 32 KiB log block (src/db/log.rs:204-279) into
//     record descriptors for k_blocks.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <string.h>

#include "lcrc_device.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// Unaligned 16-byte view: gfx950 global/buffer loads accept any byte alignment (unaligned access mode
// is enabled by the ROCm runtime); this type only tells the compiler to emit one dwordx4.
typedef u32x4 u32x4_ua __attribute__((aligned(1)));

namespace lcrc_dev {

// ---------------------------------------------------------------------------------------------------
// k_windows LDS image (76 KiB -> two 512-thread workgroups per CU)
//
// Two replicated "table sets" of four byte tables each: S0 = slice-by-4 T0..T3, S1 = Z64 (Z_n[k][b] =
// byte b at position k advanced over n zero bytes). Set s occupies half s of every 256 B row of the first
// 64 KiB, row e holding entry e. Inside a half-row (32 dwords = the 32 LDS banks) dword 8*p + r is replica
// r (0..7) of the set's table at position p; position p is indexed by data byte 3 - p (slice: T_p;
// shifts: Z[3 - p]).
// Compact rotated lookups: lane l (r = l & 7, q = (l >> 3) & 3) performs the four lookups of one step
// as instructions i = 0..3 on position (i + q) & 3, replica r. In every 32-lane ds_read group the banks
// 8*((i + q) & 3) + r are pairwise distinct, so all lookups are conflict-free with 8 replicas per table
// instead of 32. The address is one v_perm_b32 of a per-lane base (byte 0: half/position/replica) and the
// data byte.
//   [64 KiB, 76 KiB): Z256, Z512, Z1024 (unreplicated) for the block tree (its top level applies Z1024
//   twice).
// One 512-thread workgroup is launched per CU (measured: 1.3-1.7 us per 256 MiB launch faster than two
// per CU, and than 256- or 1024-thread shapes). 76 KiB of LDS lets a second one be resident: the next
// launch's workgroups fill a CU while this launch's tail is still on it.
// ---------------------------------------------------------------------------------------------------
#ifndef LCRC_A_WGCU
#define LCRC_A_WGCU 1
#endif
#ifndef LCRC_A_THREADS
#define LCRC_A_THREADS 512
#endif
constexpr int A_WG_PER_CU = LCRC_A_WGCU;  // workgroups launched per CU (LDS allows two to be resident)
constexpr int A_THREADS = LCRC_A_THREADS;
constexpr int A_REP_BYTES = 65536;
constexpr int A_ZT = A_REP_BYTES;
constexpr int A_LDS_BYTES = A_ZT + 3 * 4096;
constexpr int REGION = 16384;  // bytes per wave iteration: two 8 KiB half-tiles, 64 windows of 256 B
#ifndef LCRC_R_WGCU
#define LCRC_R_WGCU 2
#endif
constexpr int R_WG_PER_CU = LCRC_R_WGCU;  // k_ranges workgroups per CU (no refill pipeline: two resident)
constexpr uint32_t SET_S1 = 1u << 7;

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops (lgkmcnt(0)) but not for its
// outstanding global loads -- __syncthreads() would add vmcnt(0) and expose the first tile's latency.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
}

__device__ __forceinline__ uint32_t lds_u32(const void* lds_base, uint32_t byte_addr) {
  return *(const uint32_t*)((const char*)lds_base + byte_addr);
}

// a ^ b ^ c in one gfx950 v_bitop3_b32 (truth table 0x96); gfx9 has no v_xor3
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// per-lane lookup parameters of the rotated layout: base byte 0 and the v_perm selector of instruction i
// (out = { 0x00, base.b2, x.b(3 - p), base.b0 })
struct Rot {
  uint32_t b[4], s[4];
};

__device__ __forceinline__ Rot make_rot(uint32_t lane) {
  Rot R;
  const uint32_t r = lane & 7, q = (lane >> 3) & 3;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t p = (i + q) & 3;
    R.b[i] = (p << 5) | (r << 2);
    R.s[i] = 0x0C060004u | ((3 - p) << 8);
  }
  return R;
}

// one slice-by-4 step on x = r ^ w (already folded); returns walk(r, w) ^ w_next
__device__ __forceinline__ uint32_t step4x(const void* L, const Rot& R, uint32_t x, uint32_t w_next) {
  const uint32_t a0 = lds_u32(L, __builtin_amdgcn_perm(R.b[0], x, R.s[0]));
  const uint32_t a1 = lds_u32(L, __builtin_amdgcn_perm(R.b[1], x, R.s[1]));
  const uint32_t a2 = lds_u32(L, __builtin_amdgcn_perm(R.b[2], x, R.s[2]));
  const uint32_t a3 = lds_u32(L, __builtin_amdgcn_perm(R.b[3], x, R.s[3]));
  return xor3(xor3(a0, a1, w_next), a2, a3);
}

// Z_n(x) through replicated set SET (conflict-free)
template <uint32_t SET>
__device__ __forceinline__ uint32_t zrot(const void* L, const Rot& R, uint32_t x) {
  const uint32_t a0 = lds_u32(L, __builtin_amdgcn_perm(R.b[0] | SET, x, R.s[0]));
  const uint32_t a1 = lds_u32(L, __builtin_amdgcn_perm(R.b[1] | SET, x, R.s[1]));
  const uint32_t a2 = lds_u32(L, __builtin_amdgcn_perm(R.b[2] | SET, x, R.s[2]));
  const uint32_t a3 = lds_u32(L, __builtin_amdgcn_perm(R.b[3] | SET, x, R.s[3]));
  return xor3(a0, a1, a2 ^ a3);
}

// Z_n(x) through an unreplicated byte-sliced table (4 x 256 entries at tab_byte_off)
__device__ __forceinline__ uint32_t zlook(const void* L, uint32_t tab_byte_off, uint32_t r) {
  const char* z = (const char*)L + tab_byte_off;
  return *(const uint32_t*)(z + ((r & 0xff) << 2)) ^ *(const uint32_t*)(z + 1024 + (((r >> 8) & 0xff) << 2)) ^
         *(const uint32_t*)(z + 2048 + (((r >> 16) & 0xff) << 2)) ^ *(const uint32_t*)(z + 3072 + ((r >> 24) << 2));
}

// In-register transpose. In half-tile h (0: bytes [0, 128) of every 256 B window, 1: [128, 256)), lane
// l = 8*c + k (k = l & 7, c = l >> 3) loads in instruction j the 16 B piece at region byte
// 2048*j + 256*k + 128*h + 16*c: each instruction reads eight full 128 B lines. Within each group k the
// 8 lanes c and 8 registers j form an 8x8 matrix of pieces; transposing it leaves lane (k, c) with the
// pieces 2048*c + 256*k + 128*h + 16*j', j' = 0..7: half h of window 8*c + k = l. The butterfly stages
// run over lane bits 3..5:
//   bit 3: a DPP select (below)
//   bit 4: v_permlane16_swap (odd rows of a <-> even rows of b), bit 5: v_permlane32_swap (one
//          instruction per register pair)
// Lane bit 3 (register pairs j, j + 1): per output one v_cndmask_b32 with a DPP source (row_shr:8 / row_shl:8
// folded into the select) writing a fresh register -- the bank-masked v_mov_b32_dpp form needs its destination to
// hold the kept value first, i.e. a copy per pair (32 more VALU per region). VCC holds the lanes whose bit 3 is
// clear (0x00ff00ff per half), then set. bound_ctrl: a source lane outside the row reads 0 (the write happens and
// the select discards it).
__device__ __forceinline__ void transpose_pair3(u32x4& a, u32x4& b) {
  u32x4 na, nb;
  __asm__ volatile(
      "s_nop 1\n\t"
      "s_mov_b32 vcc_lo, 0x00ff00ff\n\t"
      "s_mov_b32 vcc_hi, 0x00ff00ff\n\t"
      "v_cndmask_b32_dpp %0, %8, %12, vcc row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_cndmask_b32_dpp %1, %9, %13, vcc row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_cndmask_b32_dpp %2, %10, %14, vcc row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_cndmask_b32_dpp %3, %11, %15, vcc row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "s_mov_b32 vcc_lo, 0xff00ff00\n\t"
      "s_mov_b32 vcc_hi, 0xff00ff00\n\t"
      "v_cndmask_b32_dpp %4, %12, %8, vcc row_shl:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_cndmask_b32_dpp %5, %13, %9, vcc row_shl:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_cndmask_b32_dpp %6, %14, %10, vcc row_shl:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_cndmask_b32_dpp %7, %15, %11, vcc row_shl:8 row_mask:0xf bank_mask:0xf bound_ctrl:1"
      : "=&v"(na.x), "=&v"(na.y), "=&v"(na.z), "=&v"(na.w), "=&v"(nb.x), "=&v"(nb.y), "=&v"(nb.z), "=&v"(nb.w)
      : "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w), "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w)
      : "vcc");
  a = na;
  b = nb;
}

template <int LB, int D = 1 << (LB - 3)>  // D: the register-index bit paired with lane bit LB
__device__ __forceinline__ void transpose_stage(u32x4 (&v)[8]) {
  if constexpr (LB == 3) {
    static_assert(D == 1, "stage 3 pairs registers j, j + 1");
#pragma unroll
    for (int j = 0; j < 8; j += 2) transpose_pair3(v[j], v[j + 1]);
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (j & D) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t a = v[j][q], b = v[j + D][q];
      if constexpr (LB == 4) {
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

__device__ __forceinline__ uint32_t mask32c(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }

// wave-uniform descriptor for region t: loads past the end of the span (or of a non-existent region)
// return 0 without touching memory
__device__ __forceinline__ __amdgpu_buffer_rsrc_t region_rsrc(const uint8_t* base, uint64_t span, uint64_t t,
                                                              uint64_t nreg) {
  uint32_t nrec = 0;
  uint64_t toff = 0;
  if (t < nreg) {
    toff = t * (uint64_t)REGION;
    const uint64_t rem = span - toff;
    nrec = rem < (uint64_t)REGION ? (uint32_t)rem : (uint32_t)REGION;
  }
  return __builtin_amdgcn_make_buffer_rsrc((void*)(base + toff), (short)0, (int)nrec, 0x00020000);
}

#define LCRC_REFILL(rs, off) __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, LCRC_LOAD_AUX)

// Load layouts of a 16 KiB region (half h = bytes [128 h, 128 h + 128) of every 256 B window). Both read eight
// whole 128 B lines per instruction; they differ in which lane gets which 16 B piece, i.e. in which transposes
// follow. (A third, L4 -- four lanes per 64 B half-line, a 4x4 transpose -- measured slower: the memory side lost
// more than the VALU saved.)
//  L8 (k_ranges): instruction j, lane l = 8c + k reads region byte 2048 j + 256 k + 128 h + 16 c; a transpose
//      over lane bits 3, 4 (register bits 0, 1) and a lane-bit-5 chunk join (walk_half) leave lane l with half h
//      of window l.
//  LX (k_windows, k_windows_q): piece c = c0 + 2 c1 + 4 c2 of a line goes to lane bit 4 (c0), 5 (c1) and 3 (c2):
//      lane l = k + 8 c2 + 16 c0 + 32 c1 reads byte 2048 pi(j) + 256 k + 128 h + 16 c, pi swapping bits 0 and 2
//      of j. The two permlane transposes (lane bits 4, 5 x register bits 0, 1; no DPP stage) leave lane l with
//      the contiguous 64 B chunk c2 of windows W0 and W0 + 8; a row_ror:8 chunk join gives it window
//      w(l) = (l & 15) | ((l >> 5) & 1) << 4 | ((l >> 4) & 1) << 5: its 4 KiB block's 16 windows stay in one DPP
//      row, block (lane >> 4) with its two bits swapped.
constexpr int LAY_L8 = 0, LAY_LX = 2;
template <int LAY>
__device__ __forceinline__ uint32_t lane_voff(uint32_t lane, uint32_t h) {
  if constexpr (LAY == LAY_LX)
    return 256u * (lane & 7) + 16u * (((lane >> 4) & 1) | (((lane >> 5) & 1) << 1) | (((lane >> 3) & 1) << 2)) + 128u * h;
  return 256u * (lane & 7) + 16u * (lane >> 3) + 128u * h;
}
template <int LAY>
__device__ __forceinline__ constexpr uint32_t j_off(int j) {
  return LAY == LAY_LX ? 2048u * (((j & 1) << 2) | (j & 2) | ((j >> 2) & 1)) : 2048u * j;
}
// the window a lane holds after walk_half, and the block (of the region's four) its 16-lane row finishes
template <int LAY>
__device__ __forceinline__ uint32_t window_of_lane(uint32_t lane) {
  return LAY == LAY_LX ? (lane & 15) | (((lane >> 5) & 1) << 4) | (((lane >> 4) & 1) << 5) : lane;
}
template <int LAY>
__device__ __forceinline__ uint32_t block_of_row(uint32_t lane) {
  return window_of_lane<LAY>(lane) >> 4;
}

constexpr int KW_LAY = LAY_LX;  // k_windows' load layout (see lane_voff)

template <int LAY = LAY_L8>
__device__ __forceinline__ void load_half(u32x4 (&v)[8], __amdgpu_buffer_rsrc_t rs, uint32_t voff) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = LCRC_REFILL(rs, voff + j_off<LAY>(j));
}

// LX chunk join over lane bit 3: lanes with bit 3 clear hold chunk 0 of their own window in xa and chunk 0 of
// the partner's (lane ^ 8) window in xb; lanes with bit 3 set hold chunk 1 of the partner's window in xa and of
// their own in xb. Out: c0 = own chunk 0, c1 = own chunk 1 (two v_cndmask_b32 with a row_ror:8 DPP source).
__device__ __forceinline__ void join_lx(uint32_t xa, uint32_t xb, uint32_t& c0, uint32_t& c1) {
  __asm__ volatile(
      "s_nop 1\n\t"
      "s_mov_b32 vcc_lo, 0x00ff00ff\n\t"
      "s_mov_b32 vcc_hi, 0x00ff00ff\n\t"
      "v_cndmask_b32_dpp %0, %3, %2, vcc row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
      "s_mov_b32 vcc_lo, 0xff00ff00\n\t"
      "s_mov_b32 vcc_hi, 0xff00ff00\n\t"
      "v_cndmask_b32_dpp %1, %2, %3, vcc row_ror:8 row_mask:0xf bank_mask:0xf"
      : "=&v"(c0), "=&v"(c1)
      : "v"(xa), "v"(xb)
      : "vcc");
}
// LX init routing: lanes with bit 3 clear start their window from init and the partner's from init[lane ^ 8];
// lanes with bit 3 set (chunk 1) start both from 0
__device__ __forceinline__ void init_lx(uint32_t init, uint32_t& ia, uint32_t& ib) {
  const uint32_t zero = 0;
  __asm__ volatile(
      "s_nop 1\n\t"
      "s_mov_b32 vcc_lo, 0xff00ff00\n\t"
      "s_mov_b32 vcc_hi, 0xff00ff00\n\t"
      "v_cndmask_b32_e32 %0, %2, %3, vcc\n\t"
      "v_cndmask_b32_dpp %1, %2, %3, vcc row_ror:8 row_mask:0xf bank_mask:0xf"
      : "=&v"(ia), "=&v"(ib)
      : "v"(init), "v"(zero)
      : "vcc");
}

// Transpose + walk one half-tile already in registers, from the register value `init` of the lane's window:
// returns walk(init, 128 B half of window l). As each register pair is consumed it is refilled from `rs`
// (the same half of the next region), so every wave keeps between one and two half-tiles in flight.
//
// L8: the transpose stops after lane bits 3 and 4: lane l then holds the 64 B chunk l >> 5 of the half of windows
// (l & 31) (registers 0..3) and (l & 31) + 32 (registers 4..7), contiguous, so the two chains walk them unchanged;
// one v_permlane32_swap of the two chain values (lane bit 5) then gives every lane both chunks of its own window l,
// joined by Z64. The init register goes the other way: the chunk-0 lanes (l < 32) start window l from init[l] and
// window l + 32 from init[l + 32], the chunk-1 lanes from 0. 16 permlane32 swaps per half become two.
// LX: lane bits 4, 5 x register bits 0, 1, then the row_ror:8 chunk join (join_lx).
template <bool REFILL = true, int LAY = LAY_L8, bool INIT = true>
__device__ __forceinline__ uint32_t walk_half(const void* L, const Rot& R, u32x4 (&v)[8], uint32_t init,
                                              __amdgpu_buffer_rsrc_t rs, uint32_t voff) {
  constexpr bool JOIN = LAY == LAY_L8;
  if constexpr (LAY == LAY_LX) {
    transpose_stage<4, 1>(v);
    transpose_stage<5, 2>(v);
  } else {
    transpose_stage<3>(v);
    transpose_stage<4>(v);
  }
  // two independent chains over the 64 B quarters (pieces 0..3 and 4..7); x carries the chain register
  // already xored with its next data word. Pair (j, 4 + j) is refilled as soon as it is consumed.
  uint32_t ia = INIT ? init : 0u, ib = 0u;
  if constexpr (JOIN && INIT) {  // lanes < 32: init[l] and init[l + 32]; lanes >= 32: 0 and 0
    const auto r = __builtin_amdgcn_permlane32_swap(init, 0u, false, false);
    ia = r[0];
    ib = r[1];
  }
  if constexpr (LAY == LAY_LX && INIT) init_lx(init, ia, ib);
  uint32_t xa = v[0].x ^ ia, xb = v[4].x ^ ib;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    xa = step4x(L, R, xa, v[j].y);
    xb = step4x(L, R, xb, v[4 + j].y);
    xa = step4x(L, R, xa, v[j].z);
    xb = step4x(L, R, xb, v[4 + j].z);
    xa = step4x(L, R, xa, v[j].w);
    xb = step4x(L, R, xb, v[4 + j].w);
    xa = step4x(L, R, xa, j < 3 ? v[j + 1].x : 0u);
    xb = step4x(L, R, xb, j < 3 ? v[5 + j].x : 0u);
    if (REFILL) {
      v[j] = LCRC_REFILL(rs, voff + j_off<LAY>(j));
      v[4 + j] = LCRC_REFILL(rs, voff + j_off<LAY>(4 + j));
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the refill here: hipcc would otherwise sink it past the walk
  }
  if constexpr (JOIN) {  // both chunks of the lane's own window: chunk 0 in xa, chunk 1 in xb
    const auto r = __builtin_amdgcn_permlane32_swap(xa, xb, false, false);
    xa = r[0];
    xb = r[1];
  }
  if constexpr (LAY == LAY_LX) {
    uint32_t c0, c1;
    join_lx(xa, xb, c0, c1);
    xa = c0;
    xb = c1;
  }
  return zrot<SET_S1>(L, R, xa) ^ xb;  // Z64 join of the two 64 B chunks
}

// one level of the block tree inside a 16-lane DPP row: lane g (g % 2^(M+1) == 0) <-
// Z_{256*2^M}(p_g) ^ p_{g+2^M}. Only the combining lanes look up (exec-masked ds_reads).
template <int M>
__device__ __forceinline__ uint32_t tree_level(const void* L, const Rot& R, uint32_t p, uint32_t lane) {
  const uint32_t pn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)p, 0x100 + (1 << M), 0xF, 0xF, false);
  if ((lane & ((2u << M) - 1)) == 0) {
    if constexpr (M < 3)
      p = zlook(L, A_ZT + M * 4096, p) ^ pn;
    else
      p = zlook(L, A_ZT + 2 * 4096, zlook(L, A_ZT + 2 * 4096, p)) ^ pn;  // Z2048 = Z1024 o Z1024
  }
  return p;
}

// FINAL = false: out[t*64 + l] = walk(0, 256 B window l of region t) (raw partials for k_blocks)
// FINAL = true : span = nblk * 4096; out[b] = crc of 4 KiB block b (xor fin, optional mask, verify)
template <bool FINAL, bool SHIFT, class Src>
__device__ __forceinline__ void finish_region(const void* L, const Rot& R, const Rot& SR, uint32_t p, uint64_t t,
                                              uint32_t h, uint32_t lane, const Src& src, uint32_t fin,
                                              uint32_t flags, uint32_t ev) {
  if (!FINAL) {
    src.out_of(h)[t * 64 + window_of_lane<KW_LAY>(lane)] = p;
    return;
  }
  if constexpr (SHIFT) {
    // window g's register moved to the block end (Z_{256 (15 - g)}), then the 16 windows xored into lane 0
    const uint32_t a0 = lds_u32(L, __builtin_amdgcn_perm(SR.b[0], p, SR.s[0]));
    const uint32_t a1 = lds_u32(L, __builtin_amdgcn_perm(SR.b[1], p, SR.s[1]));
    const uint32_t a2 = lds_u32(L, __builtin_amdgcn_perm(SR.b[2], p, SR.s[2]));
    const uint32_t a3 = lds_u32(L, __builtin_amdgcn_perm(SR.b[3], p, SR.s[3]));
    p = xor3(a0, a1, a2 ^ a3);
    p ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)p, 0x101, 0xF, 0xF, false);  // row_shl:1
    p ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)p, 0x102, 0xF, 0xF, false);  // row_shl:2
    p ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)p, 0x104, 0xF, 0xF, false);  // row_shl:4
    p ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)p, 0x108, 0xF, 0xF, false);  // row_shl:8
  } else {
    p = tree_level<0>(L, R, p, lane);
    p = tree_level<1>(L, R, p, lane);
    p = tree_level<2>(L, R, p, lane);
    p = tree_level<3>(L, R, p, lane);
  }
  bool ok;
  const uint64_t blk = src.block(t, h, block_of_row<KW_LAY>(lane), ok);
  if ((lane & 15) == 0 && ok) {
    uint32_t crc = p ^ fin;
    if (flags & LCRC_FLAG_MASK) crc = mask32c(crc);
    src.out_of(h)[blk] = crc;
    uint32_t* mismatch = src.mismatch_of(h);
    if (src.expected_of(h) && mismatch && ev != crc) atomicOr(&mismatch[blk >> 5], 1u << (blk & 31));
  }
}

// Region scheduler: the regions are split into equal contiguous shares, one per workgroup, and dealt to
// the workgroup's waves from a counter in LDS. Inside a CU the instruction arbiter favours older waves
// (with a fixed per-wave split the first wave of each SIMD finished in ~60% of the time of the fourth).
// An LDS atomic returns through lgkmcnt, never behind the HBM loads. CUs do not stream at one rate
// (whole XCDs differ by up to 10 %, so per-CU end times spread over ~5 us), but every way tried to
// balance them cost more than the spread: a global pool, work stealing with one global atomic per claim
// (61 us instead of 46: a wave's loads issued after an atomic return only after it), and more, smaller
// workgroups left to the hardware dispatcher (49-55 us: more prologues, a coarser tail). In a 5-batch
// queued launch (tools/probe/qstamps.py) the CUs end within 205.5-213.3 us, 4.2 us (2 %) idle on average,
// the odd XCCs ~4.5 us behind the even ones; a tail pool (the last 2048 regions claimed one at a time from
// one device counter) took 269 us instead of 205: same-address device atomics serialise.
constexpr uint64_t NO_REGION = ~0ull;

// A workgroup's share: regions lo + v * step below `end` (tickets v).
struct Share {
  uint64_t lo, step, end;
  __device__ __forceinline__ uint64_t region(uint64_t v) const {
    const uint64_t r = lo + v * step;
    return r < end ? r : NO_REGION;
  }
};

__device__ __forceinline__ Share make_share(uint64_t nreg, uint32_t nwg = 0) {
  Share sh;
  // regions dealt round-robin over the workgroups: at any moment the whole chip streams one contiguous
  // stretch of the buffer (memory skeleton: 39.9 us per 256 MiB against 41.4-42.0 with a contiguous
  // range per workgroup, tools/probe/probe_skel.hip). No ticket count: a 64-bit division in the prologue.
  sh.lo = blockIdx.x;
  sh.step = nwg ? nwg : gridDim.x;  // nwg: the launch's window workgroups (k_ts_windows: the first nwg)
  sh.end = nreg;
  return sh;
}

__device__ __forceinline__ uint64_t take_region(uint32_t* lctr, const Share& sh, uint32_t lane) {
  uint32_t v = 0;
  if (lane == 0) v = atomicAdd(lctr, 1u);
  v = __builtin_amdgcn_readfirstlane(v);
  return sh.region(v);
}

// Entry e of a linear byte table from its 8 columns c[i] = table[1 << i] (wave-uniform): xor of the
// columns of the set bits of e.
__device__ __forceinline__ uint32_t lin8(const uint32_t* __restrict__ col, uint32_t e) {
  uint32_t c[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = col[i];  // all loaded unconditionally: one s_load_dwordx8
  uint32_t v = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) v ^= c[i] & (0u - ((e >> i) & 1u));
  return v;
}

// The queued kernel's LDS image instead keeps, from 64 KiB on, the per-window block shifts: row e (256 B)
// holds in dword c = 4 k + p the entry Z_{256 k}(e << 8 (3 - p)) (k = 0..15, p = 0..3): 64 byte tables, 288
// wave passes in all. Window g of a block row is shifted by Z_{256 (15 - g)} to the block end, and the
// rotated lookup order (the slice sets' q = (lane >> 3) & 3) keeps the 32 lanes of an LDS read group on
// distinct banks: lanes g and g + 8 share 4 k mod 32 but differ in q, as do the two rows of the group.
constexpr int A_SHIFT = 65536;       // LDS offset of the block shifts (queued kernel)
constexpr int AQ_LDS_BYTES = 131072;

// Lane c of every wave owns column c (table 4 k + p); wave w writes rows e = gray(32 w + i), i = 0..31, so one
// store instruction fills one 256 B row (conflict-free) and consecutive rows differ in one index bit: each
// entry after the first is ONE xor with a column (the table is linear in e). `cols` = the lane's 8 columns,
// loaded before the first region's HBM loads are issued (they return first).
struct ShiftCols {
  u32x4 lo, hi;
};
__device__ __forceinline__ ShiftCols load_shift_cols(const uint32_t* __restrict__ gtab, uint32_t lane) {
  const uint32_t c = lane;
  const uint32_t src = (c & ~3u) + (3 - (c & 3));  // TAB_SCOLS table 4 k + byte position (3 - p)
  const u32x4* q = (const u32x4*)(gtab + TAB_SCOLS + src * 8);
  return ShiftCols{q[0], q[1]};
}
__device__ __forceinline__ void build_shift_tables(uint32_t* L, const ShiftCols& sc, uint32_t wv, uint32_t lane) {
  constexpr int WAVES = A_THREADS / 64;
  constexpr int PER = 256 / WAVES;
  static_assert(PER >= 2 && (PER & (PER - 1)) == 0, "rows per wave");
  const uint32_t col[8] = {sc.lo.x, sc.lo.y, sc.lo.z, sc.lo.w, sc.hi.x, sc.hi.y, sc.hi.z, sc.hi.w};
  const uint32_t n0 = wv * PER;  // uniform
  const uint32_t g0 = n0 ^ (n0 >> 1);
  uint32_t v = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if ((g0 >> i) & 1) v ^= col[i];
  L[A_SHIFT / 4 + g0 * 64 + lane] = v;
#pragma unroll
  for (int i = 1; i < PER; ++i) {
    v ^= col[__builtin_ctz(i)];  // gray(n) = gray(n - 1) ^ (1 << ctz(n)); ctz(n0 + i) = ctz(i)
    const uint32_t n = n0 + i;
    L[A_SHIFT / 4 + (n ^ (n >> 1)) * 64 + lane] = v;
  }
}

// lane-dependent lookup parameters of the block shifts: table 4 k + p, k = 15 - (lane & 15)
__device__ __forceinline__ Rot make_shift_rot(uint32_t lane) {
  Rot R;
  const uint32_t k = 15 - (lane & 15), q = (lane >> 3) & 3;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t p = (i + q) & 3;
    R.b[i] = (1u << 16) | ((4 * k + p) << 2);
    R.s[i] = 0x0C060004u | ((3 - p) << 8);
  }
  return R;
}

// k_windows' LDS image built from the column block TAB_COLS. 80 wave passes of 64 entries each, one
// byte table per pass (uniform columns -> scalar loads): passes 0..31 the replicated sets (set s,
// position p), passes 32..79 the tree's Z256/Z512/Z1024 (same word order as the global TAB_ZWIN).
// Without the tree (queued kernel) a wave makes 4 passes; their 32 columns can be loaded (SliceCols) before the
// region loads are issued, so the build waits on no scalar load of its own.
constexpr int SLICE_PASSES = 32 / (A_THREADS / 64);
struct SliceCols {
  uint32_t c[SLICE_PASSES][8];
};
__device__ __forceinline__ SliceCols load_slice_cols(const uint32_t* __restrict__ gtab, uint32_t wv) {
  SliceCols sc;
#pragma unroll
  for (int k = 0; k < SLICE_PASSES; ++k)
#pragma unroll
    for (int i = 0; i < 8; ++i) sc.c[k][i] = gtab[TAB_COLS + ((wv + (A_THREADS / 64) * k) >> 2) * 8 + i];
  return sc;
}
__device__ __forceinline__ uint32_t lin8v(const uint32_t (&c)[8], uint32_t e) {
  uint32_t v = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) v ^= c[i] & (0u - ((e >> i) & 1u));
  return v;
}

template <bool TREE = true>
__device__ __forceinline__ void build_tables(uint32_t* L, const uint32_t* __restrict__ gtab, uint32_t wv,
                                             uint32_t lane, const SliceCols* pre = nullptr) {
  constexpr int WAVES = A_THREADS / 64;
  static_assert(80 % WAVES == 0, "passes per wave");
#pragma unroll
  for (int k = 0; k < (TREE ? 80 : 32) / WAVES; ++k) {
    const uint32_t P = wv + WAVES * k;  // uniform
    const uint32_t e = ((P & 3) << 6) | lane;
    if (P < 32) {
      const uint32_t set = P >> 4, p = (P >> 2) & 3;
      // S0: T_p | S1: Z64[3 - p]
      const uint32_t v = (!TREE && pre) ? lin8v(pre->c[k < SLICE_PASSES ? k : 0], e)
                                        : lin8(gtab + TAB_COLS + (P >> 2) * 8, e);
      u32x4* dst = (u32x4*)((char*)L + e * 256 + set * 128 + p * 32);
      dst[0] = u32x4{v, v, v, v};
      dst[1] = u32x4{v, v, v, v};
    } else {
      const uint32_t zt = (P - 32) >> 2;  // level * 4 + byte position
      L[A_ZT / 4 + zt * 256 + e] = lin8(gtab + TAB_COLS + (8 + zt) * 8, e);
    }
  }
}

#ifdef LCRC_PROBE_CLOCK  // diagnostic build: per-workgroup shader/real clock stamps around the tile loop
__device__ unsigned long long lcrc_dbg_clock[4096];   // k_windows per workgroup: shader and real clock
__device__ unsigned long long lcrc_dbg_stamp[4096 * 8];  // k_windows per wave: entry, tables ready, first half,
                                                        // end, table source loaded, staged, HW_ID, XCC_ID
__device__ unsigned long long lcrc_dbg_bstamp[8192 * 8];  // k_blocks per wave: entry, tables, the ends of the
                                                         // first 5 iterations, end
#endif

// Where k_windows' regions come from. WinOne: one contiguous span (a batch, a file). WinQueue: a queue of
// independent uniform 4 KiB batches (lcrc_batch_uniform_queue) numbered into one region space, so that one
// launch streams them all: the LDS image is built and the per-CU end spread paid once per launch, not once
// per batch. Both answer, for a region t: its buffer descriptor, and where its blocks' CRCs go. A region's
// job is found from a wave-uniform handle `find(t, hint)`; a wave's regions increase monotonically
// (tickets), so the previous region's handle is always a valid hint.
struct WinOne {
  const uint8_t* base;
  uint64_t span, nreg;
  uint32_t* out;
  uint64_t nblk;
  const uint32_t* expected;
  uint32_t* mismatch;
  __device__ __forceinline__ uint64_t regions() const { return nreg; }
  __device__ __forceinline__ uint32_t find(uint64_t, uint32_t) const { return 0; }
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(uint64_t t, uint32_t) const {
    return region_rsrc(base, span, t, nreg);
  }
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t first(uint64_t t, uint32_t& h) const {
    h = 0;
    return rsrc(t, 0);
  }
  // block q of region t: (output slot, valid)
  __device__ __forceinline__ uint64_t block(uint64_t t, uint32_t, uint32_t q, bool& ok) const {
    const uint64_t b = t * 4 + q;
    ok = b < nblk;
    return b;
  }
  __device__ __forceinline__ uint32_t* out_of(uint32_t) const { return out; }
  __device__ __forceinline__ const uint32_t* expected_of(uint32_t) const { return expected; }
  __device__ __forceinline__ uint32_t* mismatch_of(uint32_t) const { return mismatch; }
};

#ifndef LCRC_MAX_QJOBS
#define LCRC_MAX_QJOBS 32
#endif
constexpr int MAX_QJOBS = LCRC_MAX_QJOBS;  // batches per queued launch (kernel-argument space: 32 x 48 B)
struct QJobDev {
  const uint8_t* base;
  uint32_t* out;
  const uint32_t* expected;
  uint32_t* mismatch;
  uint64_t nblk;
  uint64_t reg0;  // the job's first region in the launch's region space
};
struct QJobsArg {
  QJobDev j[MAX_QJOBS];
  uint64_t nreg;
  uint32_t n;
};

struct WinQueue {
  const QJobDev* J;
  uint32_t nj;
  uint64_t nreg;
  const uint8_t* b0;  // job 0's base and blocks, job 1's first region (first())
  uint64_t n0, r1;
  __device__ __forceinline__ uint64_t regions() const { return nreg; }
  __device__ __forceinline__ uint32_t find(uint64_t t, uint32_t from) const {
    uint32_t j = from;
    if (t >= nreg) return j;
    while (j + 1 < nj && t >= J[j + 1].reg0) ++j;
    return j;
  }
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(uint64_t t, uint32_t j) const {
    uint32_t nrec = 0;
    const uint8_t* b = J[j].base;
    if (t < nreg) {
      const uint64_t local = t - J[j].reg0;
      b += local * (uint64_t)REGION;
      const uint64_t rem = J[j].nblk * 4096 - local * (uint64_t)REGION;
      nrec = rem < (uint64_t)REGION ? (uint32_t)rem : (uint32_t)REGION;
    }
    return __builtin_amdgcn_make_buffer_rsrc((void*)b, (short)0, (int)nrec, 0x00020000);
  }
  // a wave's first region: in the common case (job 0) from kernel-argument loads that do not wait on each other
  // (find + rsrc are a chain of four dependent scalar round trips)
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t first(uint64_t t, uint32_t& h) const {
    if (t < nreg && (nj == 1 || t < r1)) {
      h = 0;
      const uint64_t rem = n0 * 4096 - t * (uint64_t)REGION;
      const uint32_t nrec = rem < (uint64_t)REGION ? (uint32_t)rem : (uint32_t)REGION;
      return __builtin_amdgcn_make_buffer_rsrc((void*)(b0 + t * (uint64_t)REGION), (short)0, (int)nrec, 0x00020000);
    }
    h = find(t, 0);
    return rsrc(t, h);
  }
  __device__ __forceinline__ uint64_t block(uint64_t t, uint32_t j, uint32_t q, bool& ok) const {
    const uint64_t b = (t - J[j].reg0) * 4 + q;
    ok = b < J[j].nblk;
    return b;
  }
  __device__ __forceinline__ uint32_t* out_of(uint32_t j) const { return J[j].out; }
  __device__ __forceinline__ const uint32_t* expected_of(uint32_t j) const { return J[j].expected; }
  __device__ __forceinline__ uint32_t* mismatch_of(uint32_t j) const { return J[j].mismatch; }
};

// expected values of region t's blocks (verify), loaded ahead of the refills that follow so the compare at
// the end of the region does not wait for them (vmcnt retires in issue order)
template <bool FINAL, class Src>
__device__ __forceinline__ uint32_t expect_of(const Src& src, uint64_t t, uint32_t h, uint32_t lane) {
  uint32_t ev = 0;
  if (FINAL && src.expected_of(h)) {
    bool ok;
    const uint64_t blk = src.block(t, h, block_of_row<KW_LAY>(lane), ok);
    if ((lane & 15) == 0 && ok) ev = src.expected_of(h)[blk];
  }
  return ev;
}


template <bool FINAL, bool SHIFT, class Src>
__device__ __forceinline__ void windows_body(const Src& src, const uint32_t* __restrict__ gtab, uint32_t fin,
                                             uint32_t flags, uint32_t* L, uint32_t* wg_ticket_p, uint32_t nwg = 0) {
  uint32_t& wg_ticket = *wg_ticket_p;
  const uint32_t lane = __lane_id();
  const uint32_t tid = threadIdx.x;
  const uint64_t nreg = src.regions();
  const Share share = make_share(nreg, nwg);  // this workgroup's regions
#ifdef LCRC_PROBE_CLOCK
  const unsigned long long s_entry = __builtin_amdgcn_s_memrealtime();
  unsigned long long s_first = 0;
#endif

  // Prologue. The first region of wave w is region w of the share (static), so its HBM loads go out at
  // once; the tables are then built while they are in flight. Nothing in the build waits behind them: the
  // byte tables are linear maps of their 8-bit index, so every entry is an xor of 8 columns (entries
  // 1, 2, 4, .., 128 of the global image), read with SCALAR loads -- vector-memory returns reach a CU in
  // issue order, and a table read through the vector path would wait for every HBM load issued before it.
  const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t voff_a = lane_voff<KW_LAY>(lane, 0), voff_b = lane_voff<KW_LAY>(lane, 1);
  ShiftCols scols{};
  if (SHIFT) scols = load_shift_cols(gtab, lane);  // issued before the region loads: returns first
  SliceCols slc;
  if (SHIFT) slc = load_slice_cols(gtab, wv);  // scalar: the build then waits on nothing but these
  uint64_t t = share.region(wv);
  uint32_t ht;
  u32x4 va[8], vb[8];
  {
    const __amdgpu_buffer_rsrc_t rs0 = src.first(t, ht);
    __builtin_amdgcn_sched_barrier(0);
    load_half<KW_LAY>(va, rs0, voff_a);
    __builtin_amdgcn_sched_barrier(0);  // issue order va, vb: the loop's vmcnt bookkeeping assumes it
    load_half<KW_LAY>(vb, rs0, voff_b);
    __builtin_amdgcn_sched_barrier(0);
  }
#ifdef LCRC_PROBE_CLOCK
  const unsigned long long s_src = __builtin_amdgcn_s_memrealtime();
#endif
  build_tables<!SHIFT>(L, gtab, wv, lane, SHIFT ? &slc : nullptr);
  if (SHIFT) build_shift_tables(L, scols, wv, lane);
#ifdef LCRC_PROBE_CLOCK
  const unsigned long long s_staged = __builtin_amdgcn_s_memrealtime();
#endif
  if (tid == 0) wg_ticket = A_THREADS / 64;  // tickets 0 .. waves-1 were the static first regions
  lds_barrier();
  const Rot R = make_rot(lane);
  const Rot SR = SHIFT ? make_shift_rot(lane) : R;
#ifdef LCRC_PROBE_CLOCK
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#endif

  uint64_t tn = take_region(&wg_ticket, share, lane);
  uint32_t hn = src.find(tn, ht);
  // tn = the region the refills load (ticket taken after the prologue or in the previous iteration);
  // the ticket for the one after is taken between the two walks.
  // va/vb hold the two halves of region t; walking a half refills it with the same half of region tn.
  // Chain a of the second half continues from the first half's register value, so one Z64 join per
  // half is the only recombination inside a window.
  while (t != NO_REGION) {
    const __amdgpu_buffer_rsrc_t rsn = src.rsrc(tn, hn);
    const uint32_t ev = expect_of<FINAL>(src, t, ht, lane);
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t x = walk_half<true, KW_LAY, false>(L, R, va, 0u, rsn, voff_a);
#ifdef LCRC_PROBE_CLOCK
    if (!s_first) s_first = __builtin_amdgcn_s_memrealtime();
#endif
    __builtin_amdgcn_sched_barrier(0);
    const uint64_t tnn = take_region(&wg_ticket, share, lane);
    const uint32_t p = walk_half<true, KW_LAY>(L, R, vb, x, rsn, voff_b);
    finish_region<FINAL, SHIFT>(L, R, SR, p, t, ht, lane, src, fin, flags, ev);
    t = tn;
    ht = hn;
    tn = tnn;
    hn = src.find(tnn, hn);
  }
#ifdef LCRC_PROBE_CLOCK
  const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x < 1024) {
    lcrc_dbg_clock[blockIdx.x * 4 + 0] = c1 - c0;
    lcrc_dbg_clock[blockIdx.x * 4 + 1] = r1 - r0;
  }
  const uint64_t gw = (uint64_t)blockIdx.x * (A_THREADS / 64) + (threadIdx.x >> 6);
  if (lane == 0 && gw < 4096) {
    lcrc_dbg_stamp[gw * 8 + 0] = s_entry;
    lcrc_dbg_stamp[gw * 8 + 1] = r0;
    lcrc_dbg_stamp[gw * 8 + 2] = s_first;
    lcrc_dbg_stamp[gw * 8 + 3] = r1;
    lcrc_dbg_stamp[gw * 8 + 4] = s_src;
    lcrc_dbg_stamp[gw * 8 + 5] = s_staged;
    // where the wave ran: HW_ID (cu/sh/se fields) and XCC_ID
    lcrc_dbg_stamp[gw * 8 + 6] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    lcrc_dbg_stamp[gw * 8 + 7] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
  }
#endif
}

template <bool FINAL>
__global__ void __launch_bounds__(A_THREADS) k_windows(const uint8_t* __restrict__ base, uint64_t span,
                                                      uint64_t nreg, const uint32_t* __restrict__ gtab,
                                                      uint32_t* __restrict__ out, uint64_t nblk, uint32_t fin,
                                                      uint32_t flags, const uint32_t* __restrict__ expected,
                                                      uint32_t* __restrict__ mismatch) {
  __shared__ __attribute__((aligned(16))) uint32_t L[A_LDS_BYTES / 4];
  __shared__ uint32_t wg_ticket;
  WinOne src{base, span, nreg, out, nblk, expected, mismatch};
  windows_body<FINAL, false>(src, gtab, fin, flags, L, &wg_ticket);
}

// a queue of uniform 4 KiB batches in one launch (final CRCs only)
__global__ void __launch_bounds__(A_THREADS) k_windows_q(const QJobsArg jobs, const uint32_t* __restrict__ gtab,
                                                        uint32_t fin, uint32_t flags) {
  // every argument the prologue needs, loaded in one batch (MAX_QJOBS >= 2: j[1] is in the argument block)
  WinQueue src{jobs.j, jobs.n, jobs.nreg, jobs.j[0].base, jobs.j[0].nblk, jobs.j[1].reg0};
  __asm__ volatile("" ::"s"(src.nj), "s"(src.nreg), "s"(src.b0), "s"(src.n0), "s"(src.r1), "s"(gtab), "s"(fin),
                   "s"(flags), "s"(gridDim.x));
  __shared__ __attribute__((aligned(16))) uint32_t L[AQ_LDS_BYTES / 4];
  __shared__ uint32_t wg_ticket;
  windows_body<true, true>(src, gtab, fin, flags, L, &wg_ticket);
}

// a * b mod P, reflected (bit 31 = x^0): zlib's multmodp recurrence without branches
__device__ __forceinline__ uint32_t gf_mul(uint32_t a, uint32_t b, uint32_t poly) {
  uint32_t p = 0;
#pragma unroll
  for (int i = 31; i >= 0; --i) {
    p ^= b & (0u - ((a >> i) & 1u));
    b = (b >> 1) ^ (poly & (0u - (b & 1u)));
  }
  return p;
}

// ---------------------------------------------------------------------------------------------------
// k_blocks: one 16-lane row per range. LDS (40 KiB): T0..T3 [4 KiB], Z16..Z128 [16 KiB],
// Z256..Z2048 [16 KiB], Z4096 [4 KiB], unreplicated (the hot loop is in k_windows).
// The kernel is latency-bound (a few dependent memory round trips per range), so every load a range
// needs -- head and tail pieces, the first batch of window values -- is issued before any of them is
// used, and 512-thread workgroups (4 per CU by LDS) keep 32 waves per CU in flight.
// ---------------------------------------------------------------------------------------------------
constexpr int B_THREADS = 512;
// k_blocks' LDS image (40 KiB): slice tables T0..T3, the binary row-tree shifts Z16..Z128 and Z256..Z2048, Z4096.
// (4-way two-level row trees -- 8 lookups instead of 16, a 56 KiB image -- measured slower: config 3 3,957 vs
// 4,640 GiB/s, WAL 2,600 vs 3,148; lane-dependent table bases conflict in the banks and only two workgroups fit
// a CU.)
constexpr int KL_Z4096 = TAB_Z4096;
constexpr int B_LDS_DWORDS = TAB_COLS;  // slice and shift tables (not the column block)
constexpr int B_BATCH = 8;  // window values per lane loaded ahead of the fold

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

// Lane g's share of a row walk over [a, e) (0 <= e - a <= 256): the 16 B piece ending at
// e - 16*(15-g). kind 0: empty, 1: whole piece inside [a, e), 2: straddles a (only bytes [first, 16) are
// walked; the piece is read whole when it starts inside the buffer, else bytewise from a on).
struct RowPiece {
  u32x4 w;
  uint32_t kind, first, at_a;
};

__device__ __forceinline__ RowPiece row_load(const uint8_t* __restrict__ base, uint64_t a, uint64_t e, uint32_t g) {
  RowPiece p;
  p.w = u32x4{0, 0, 0, 0};
  p.kind = 0;
  p.first = 0;
  p.at_a = 0;
  const int64_t pe = (int64_t)e - 16 * (15 - (int)g);
  const int64_t ps = pe - 16;
  if (pe > (int64_t)a) {
    if (ps >= (int64_t)a) {
      p.kind = 1;
      p.at_a = ps == (int64_t)a;
      p.w = *(const u32x4_ua*)(base + ps);
    } else {
      p.kind = 2;
      p.first = (uint32_t)((int64_t)a - ps);
      if (ps >= 0) {
        p.w = *(const u32x4_ua*)(base + ps);
      } else {  // the range starts in the buffer's first 16 bytes
        uint32_t b[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) b[i] = (i >= 1 && (uint32_t)i >= p.first) ? base[ps + i] : 0u;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          p.w[q] = b[4 * q] | (b[4 * q + 1] << 8) | (b[4 * q + 2] << 16) | (b[4 * q + 3] << 24);
      }
    }
  }
  return p;
}

// lane g of a 16-lane row <- lane g + 2^m of the same row (0 past the row's end): DPP row_shl
__device__ __forceinline__ uint32_t row_down(uint32_t v, int m) {
  switch (m) {
    case 0: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x101, 0xF, 0xF, false);
    case 1: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x102, 0xF, 0xF, false);
    case 2: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x104, 0xF, 0xF, false);
    default: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x108, 0xF, 0xF, false);
  }
}

// every lane of a 16-lane row <- lane 0 of its row (four scalar reads, no LDS round trip)
__device__ __forceinline__ uint32_t row_bcast0(uint32_t v, uint32_t lane) {
  const uint32_t r0 = __builtin_amdgcn_readlane(v, 0), r1 = __builtin_amdgcn_readlane(v, 16);
  const uint32_t r2 = __builtin_amdgcn_readlane(v, 32), r3 = __builtin_amdgcn_readlane(v, 48);
  return lane < 32 ? (lane < 16 ? r0 : r1) : (lane < 48 ? r2 : r3);
}


// walk(R0, base[a, e)) from the row's loaded pieces, returned to every lane of the row; a == e -> R0.
// Must be called by all 64 lanes (contains cross-lane ops).
__device__ uint32_t row_walk(const uint32_t* L, const RowPiece& p, bool empty_range, uint32_t R0, uint32_t g,
                             uint32_t lane) {
  // Branch-free for every kind: the bytes of the piece before the range are zeroed (a zero prefix walked
  // from register 0 stays 0, so every piece is a whole 16 B unit of the tree), and the register R0 at the
  // range start is injected into the first bytes: walk(R0, M) = walk(0, M ^ LE(R0)[0, k)) ^ (R0 >> 8k)
  // with k = min(|M|, 4) (the high part of R0 just shifts out when fewer than 4 bytes follow).
  const uint32_t f = p.kind == 2 ? p.first : 0u;  // bytes of the piece before the range
  const bool inj = p.kind == 2 || (p.kind == 1 && p.at_a);
  const uint32_t k = 16 - f < 4 ? 16 - f : 4u;
  const uint32_t rl = !inj ? 0u : k == 4 ? R0 : R0 & ((1u << (8 * k)) - 1);
  const uint32_t rh = inj && k < 4 ? R0 >> (8 * k) : 0u;
  const uint64_t sh = (uint64_t)rl << (8 * (f & 3));
  const uint32_t qf = f >> 2;
  uint32_t wq[4];
#pragma unroll
  for (uint32_t q = 0; q < 4; ++q) {
    const uint32_t m = 4 * q + 4 <= f ? 0u : 4 * q >= f ? ~0u : ~0u << (8 * (f - 4 * q));
    wq[q] = (p.w[q] & m) ^ (q == qf ? (uint32_t)sh : q == qf + 1 ? (uint32_t)(sh >> 32) : 0u);
  }
  uint32_t cv = step4(L, 0u, wq[0]);
  cv = step4(L, cv, wq[1]);
  cv = step4(L, cv, wq[2]);
  cv = step4(L, cv, wq[3]) ^ rh;
  // row tree: level m joins lane g with g + 2^m, shifting the left part by 16*2^m bytes
#pragma unroll
  for (int m = 0; m < 4; ++m) {  // only the combining lanes look up (exec-masked: fewer bank conflicts)
    const uint32_t pn = row_down(cv, m);
    if ((g & ((2u << m) - 1)) == 0) cv = zl(L, TAB_ZPIECE + m * 1024, cv) ^ pn;
  }
  const uint32_t res = row_bcast0(cv, lane);
  return empty_range ? R0 : res;
}

__device__ __forceinline__ uint32_t load_le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// range i's mismatch bit. Zeroed bitmap: set the bad ones. LCRC_KFLAG_SETCLR (no fill before the launch):
// every range sets or clears its own bit, and range n - 1 also clears the bits past it in the last word
// (one thread's atomics to one word stay in order).
__device__ __forceinline__ void mismatch_bit(uint32_t* __restrict__ mm, uint64_t i, uint64_t n, bool bad,
                                             uint32_t flags) {
  const uint32_t bit = 1u << (i & 31);
  if (!(flags & LCRC_KFLAG_SETCLR)) {
    if (bad) atomicOr(&mm[i >> 5], bit);
    return;
  }
  if (bad) atomicOr(&mm[i >> 5], bit);
  else atomicAnd(&mm[i >> 5], ~bit);
  if (i + 1 == n && bit != 0x80000000u) atomicAnd(&mm[i >> 5], (bit << 1) - 1u);
}

#ifndef LCRC_KB_WPE
#define LCRC_KB_WPE 8  // k_blocks' waves per SIMD (register budget); measurement builds vary it
#endif
// waves_per_eu(8): 64 VGPRs and few enough SGPRs for 8 waves per SIMD (at 97 SGPRs only 6 fit, so a
// quarter of the 4 x 512-thread workgroups per CU started only when others had finished)
template <bool UNIFORM>
__global__ void __launch_bounds__(B_THREADS) __attribute__((amdgpu_waves_per_eu(LCRC_KB_WPE, 8))) k_blocks(const uint8_t* __restrict__ base, uint64_t base_len,
                                                     const lcrc_desc_dev* __restrict__ descs, uint64_t n,
                                                     uint64_t ustride, uint32_t ulen,
                                                     const uint32_t* __restrict__ uexp,
                                                     const uint32_t* __restrict__ win, const uint32_t* __restrict__ gtab,
                                                     uint32_t init, uint32_t xorout, uint32_t flags,
                                                     uint32_t* __restrict__ out, uint32_t* __restrict__ mismatch,
                                                     const uint64_t* __restrict__ n_dev,
                                                     lcrc_wal_rec_dev* __restrict__ recs) {
  __shared__ __attribute__((aligned(16))) uint32_t L[B_LDS_DWORDS];
#ifdef LCRC_PROBE_CLOCK
  const unsigned long long b_entry = __builtin_amdgcn_s_memrealtime();
  unsigned long long b_it[5] = {0, 0, 0, 0, 0};
  unsigned long long b_ph[4] = {0, 0, 0, 0};  // first iteration: loads landed, head walked, folded, tail walked
  uint32_t b_nit = 0;
#endif
  const uint64_t n_cap = n;  // the descriptor (and WAL record) capacity
  if (n_dev) n = *n_dev < n ? *n_dev : n;  // count produced on the device (WAL scan)
  if ((uint64_t)blockIdx.x * (B_THREADS / 16) >= n) return;  // no range for this workgroup: not even the table load
  const uint32_t lane = __lane_id();
  const uint32_t g = lane & 15, row = lane >> 4;
  const uint64_t wave = (uint64_t)blockIdx.x * (B_THREADS / 64) + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * (B_THREADS / 64);
  const bool use_win = win != nullptr;
  // descriptors are loaded one iteration ahead of their use (the first one before the table fill); the
  // raw words are kept and checked only when the iteration that uses them starts, so the load is not
  // waited for where it is issued.
  // a range outside [0, base_len) is never read: it becomes empty, CRC 0, and is flagged as a mismatch
  auto load_desc = [&](uint64_t i, lcrc_desc_dev& d) {
    d.offset = 0;
    d.length = 0;
    d.expect_rel = LCRC_NO_EXPECT_DEV;
    if (i < n) {
      if (UNIFORM) {
        d.offset = i * ustride;
        d.length = ulen;
      } else {
        d = descs[i];
      }
    }
  };
  lcrc_desc_dev d_nx;
  {
    // every load first, then every store: one L2 round trip for the image instead of one per 8 KiB
    constexpr int PER = (B_LDS_DWORDS / 4 + B_THREADS - 1) / B_THREADS;
    u32x4 t[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const uint32_t i = threadIdx.x + k * B_THREADS;
      if (i < B_LDS_DWORDS / 4) t[k] = ((const u32x4*)gtab)[i];
    }
    load_desc(wave * 4 + row, d_nx);  // the first descriptor in the same round trip
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const uint32_t i = threadIdx.x + k * B_THREADS;
      if (i < B_LDS_DWORDS / 4) ((u32x4*)L)[i] = t[k];
    }
  }
  __syncthreads();
#ifdef LCRC_PROBE_CLOCK
  const unsigned long long b_tab = __builtin_amdgcn_s_memrealtime();
#endif

  for (uint64_t i0 = wave * 4; i0 < n; i0 += nwaves * 4) {
    const uint64_t i = i0 + row;
    const bool valid = i < n;
    const bool oob = !UNIFORM && (d_nx.offset > base_len || (uint64_t)d_nx.length > base_len - d_nx.offset);
    const uint64_t s = oob ? 0 : d_nx.offset;
    const uint32_t len = oob ? 0u : d_nx.length;
    // WAL scan (recs): the descriptor carries the record's file-order index, its expected CRC is at -6
    const uint64_t ridx = recs ? (uint64_t)(uint32_t)d_nx.expect_rel : i;
    const int32_t xrel = recs ? -6 : d_nx.expect_rel;
    load_desc(i + nwaves * 4, d_nx);
    const uint64_t e = s + len;
    // the expected value, loaded with the data (bytewise: any alignment, and checked against the buffer)
    uint32_t expv = 0;
    bool exp_ok = false;
    if (!UNIFORM && valid && g == 0 && xrel != LCRC_NO_EXPECT_DEV) {
      const int64_t xp = (int64_t)s + xrel;
      exp_ok = !(xp < 0 || (uint64_t)xp + 4 > base_len);
      if (exp_ok) expv = load_le32(base + xp);
    }
    uint32_t acc;
    if (use_win) {
      // window indices: head = partial-or-full window ws, full windows (ws, wfull], tail = partial window wl
      const uint64_t ws = s >> 8;
      const uint64_t wl = len ? (e - 1) >> 8 : ws;
      const bool single = (ws == wl);
      const uint64_t head_end = single ? e : (ws + 1) << 8;
      const uint64_t ta = (single || (e & 255) == 0) ? e : (wl << 8);
      const uint64_t wfull = ((e & 255) == 0) ? wl : wl - 1;
      // middle: virtual items [pad zeros..., head, win[ws+1 .. wfull]] folded 16 per round (Horner
      // with Z4096 per lane, then a 4-level tree)
      const uint32_t items = single ? 0u : (uint32_t)(wfull - ws) + 1;  // head + full windows (< 2^24)
      const uint32_t npad = (16 - (items & 15)) & 15;
      const uint32_t rounds = single ? 0u : (npad + items) >> 4;
      const uint32_t rr32 = rounds;
      // lane g's window value of round q is wv[16 q] (the slots before the head are padding)
      const uint32_t* wv = win + ws + g - npad;
      uint32_t rmax = max(max(__builtin_amdgcn_readlane(rr32, 0), __builtin_amdgcn_readlane(rr32, 16)),
                                max(__builtin_amdgcn_readlane(rr32, 32), __builtin_amdgcn_readlane(rr32, 48)));

      // every load this range needs first: head and tail pieces, the first batch of window values
      const RowPiece ph = row_load(base, s, head_end, g);
      const RowPiece pt = row_load(base, ta, e, g);
      uint32_t vals[B_BATCH];
#pragma unroll
      for (int j = 0; j < B_BATCH; ++j) vals[j] = ((uint32_t)j < rounds && 16u * j + g > npad) ? wv[16 * j] : 0u;

#ifdef LCRC_PROBE_PHASES
      if (b_nit == 0) {
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        b_ph[0] = __builtin_amdgcn_s_memrealtime();
      }
#endif
      const uint32_t head = row_walk(L, ph, s == head_end, init, g, lane);
#ifdef LCRC_PROBE_PHASES
      if (b_nit == 0) {
        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::"v"(head) : "memory");
        b_ph[1] = __builtin_amdgcn_s_memrealtime();
      }
#endif
      uint32_t a = 0;
      for (uint32_t q0 = 0; q0 < rmax; q0 += B_BATCH) {
        if (q0) {
#pragma unroll
          for (int j = 0; j < B_BATCH; ++j) {
            const uint32_t q = q0 + j;
            vals[j] = (q < rounds && 16u * q + g > npad) ? wv[16 * q] : 0u;
          }
        }
#pragma unroll
        for (int j = 0; j < B_BATCH; ++j) {
          const uint32_t q = q0 + j;
          if (q < rounds) a = zl(L, KL_Z4096, a) ^ (16u * q + g == npad ? head : vals[j]);
        }
      }
      // (a wave whose four ranges each lie in one window -- short WAL records -- skips the row tree and
      // the tail walk: both are wave-uniform decisions)
      if (rmax) {
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const uint32_t pn = row_down(a, m);
          if ((g & ((2u << m) - 1)) == 0) a = zl(L, TAB_ZWIN + m * 1024, a) ^ pn;
        }
      }
      const uint32_t mid = row_bcast0(a, lane);
#ifdef LCRC_PROBE_PHASES
      if (b_nit == 0) {
        __asm__ volatile("" ::"v"(mid));
        b_ph[2] = __builtin_amdgcn_s_memrealtime();
      }
#endif
      acc = single ? head : mid;
      // tail: the partial last window, walked from the folded value
      if (__builtin_amdgcn_ballot_w64(ta != e)) acc = row_walk(L, pt, ta == e, acc, g, lane);
#ifdef LCRC_PROBE_PHASES
      if (b_nit == 0) {
        __asm__ volatile("" ::"v"(acc));
        b_ph[3] = __builtin_amdgcn_s_memrealtime();
      }
#endif
    } else {
      // direct: walk the whole range in 256 B chunks (sparse batches)
      uint32_t nch = (uint32_t)(((uint64_t)len + 255) >> 8);
      uint32_t cmax = nch;
      cmax = max(cmax, (uint32_t)__shfl_xor((int)cmax, 16, 64));
      cmax = max(cmax, (uint32_t)__shfl_xor((int)cmax, 32, 64));
      acc = init;
      RowPiece pc = row_load(base, s, s + 256 < e ? s + 256 : e, g);
      for (uint32_t k = 0; k < cmax; ++k) {
        uint64_t ca = s + 256 * k;
        uint64_t ce = ca + 256 < e ? ca + 256 : e;
        if (k >= nch) ca = ce = e;
        // next chunk's pieces in flight while this one is walked
        const uint64_t na = ca + 256 < e ? ca + 256 : e, ne = na + 256 < e ? na + 256 : e;
        const RowPiece pn = row_load(base, na, ne, g);
        acc = row_walk(L, pc, ca == ce, acc, g, lane);
        pc = pn;
      }
    }
    if (valid && g == 0) {
      uint32_t crc = acc ^ xorout;
      if (flags & LCRC_FLAG_MASK) crc = mask32c(crc);
      if (oob) crc = 0;
      out[i] = crc;
      bool bad = oob;
      if (UNIFORM) {
        if (uexp) bad = uexp[i] != crc;
      } else if (xrel != LCRC_NO_EXPECT_DEV) {
        bad = bad || !exp_ok || expv != crc;
      }
      if (mismatch) mismatch_bit(mismatch, i, n, bad, flags);
      if (recs && ridx < n_cap) {  // WAL scan: the verdict of read_physical_record's checksum compare (log.rs:260-273)
        recs[ridx].crc = crc;
        recs[ridx].status = bad ? 1 : 0;
      }
    }
#ifdef LCRC_PROBE_CLOCK
    if (b_nit < 5) b_it[b_nit++] = __builtin_amdgcn_s_memrealtime();
#endif
  }
#ifdef LCRC_PROBE_CLOCK
  const uint64_t gw = (uint64_t)blockIdx.x * (B_THREADS / 64) + (threadIdx.x >> 6);
  if (lane == 0 && gw < 8192) {
    lcrc_dbg_bstamp[gw * 8 + 0] = b_entry;
    lcrc_dbg_bstamp[gw * 8 + 1] = b_tab;
    for (int k = 0; k < 5; ++k) lcrc_dbg_bstamp[gw * 8 + 2 + k] = b_it[k];
#ifdef LCRC_PROBE_PHASES
    for (int k = 0; k < 4; ++k) lcrc_dbg_bstamp[gw * 8 + 3 + k] = b_ph[k];  // over it2..it5
#endif
    lcrc_dbg_bstamp[gw * 8 + 7] = __builtin_amdgcn_s_memrealtime();
  }
#endif
}

// ---------------------------------------------------------------------------------------------------
// k_ranges: arbitrary ranges in ONE streaming pass (the general path without k_windows<false> +
// k_blocks). A range is cut into 4 KiB chunks from its start; a wave walks four chunks at a time, one per
// 16-lane row and one 256 B window per lane, with k_windows' coalesced loads (load j covers the windows
// 8j..8j+7, all in row j/2, so each load has a wave-uniform buffer descriptor), transposes, LDS image and
// row tree. Chunks start on the dword at or below the range start (byte-unaligned vector loads are far
// slower); the d4 bytes before the range are zeroed (a zero prefix walked from register 0 stays 0) and the
// start register is injected at byte d4: walk(R0, M) = walk(0, M ^ LE(R0)) for |M| >= 4, which holds for
// the zero-padded message. The buffer descriptor's range check returns a dword only when it lies wholly
// below num_records (tools/probe/probe_oob.hip), so past the last whole dword of a range everything reads
// as zeros and every chunk is a whole 4 KiB unit of M' || 0^z, M' = M without its bytes V in a partial last
// dword:
//   acc = C_0;  acc = Z4096(acc) ^ C_k;  walk(R0, M) = acc * x^(-8 pad) mod P  ^  walk(0, V)
// with pad = nchunks * 4096 - d4 - len (4097 precomputed inverses, one GF(2) multiply) and walk(0, V)
// three independent slice-table lookups (T_{|V|-1-k}[V_k]). Rows take ranges independently from the workgroup's ticket
// counter (ranges dealt round-robin over the workgroups), so a long range only holds its own row.
// ---------------------------------------------------------------------------------------------------
constexpr uint32_t R_SLOTS = 32;    // ranges shared by the rows of a workgroup at a time
constexpr uint32_t R_KMAX = 4096;   // chunks of a shared range (x^(8 * 4096 * k) table); longer: private
constexpr uint32_t R_OVF = 16;      // bytes past one full chunk walked at the end instead of a second chunk


__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}

template <bool UNIFORM>
__global__ void __launch_bounds__(A_THREADS) k_ranges(const uint8_t* __restrict__ base, uint64_t base_len,
                                                     const lcrc_desc_dev* __restrict__ descs, uint64_t n,
                                                     uint64_t ustride, uint32_t ulen,
                                                     const uint32_t* __restrict__ uexp,
                                                     const uint32_t* __restrict__ gtab,
                                                     const uint32_t* __restrict__ inv, uint32_t x4096,
                                                     uint32_t poly, uint32_t init, uint32_t xorout,
                                                     uint32_t flags, uint32_t* __restrict__ out,
                                                     uint32_t* __restrict__ mismatch,
                                                     const uint64_t* __restrict__ n_dev,
                                                     lcrc_wal_rec_dev* __restrict__ recs) {
  __shared__ __attribute__((aligned(16))) uint32_t L[A_LDS_BYTES / 4];
  __shared__ uint32_t ticket, work_mask, free_mask;
  // shared ranges (more than one chunk): chunks claimed by any row of the workgroup, their registers
  // shifted into place and xored into the slot, the row completing the last chunk finishes the range.
  // next / info carry a generation in bits 16+ so a claim that raced with the slot's reuse is recognised.
  __shared__ uint32_t sl_next[R_SLOTS], sl_info[R_SLOTS], sl_left[R_SLOTS], sl_acc[R_SLOTS], sl_gen[R_SLOTS];
  __shared__ uint32_t sl_rng[R_SLOTS], sl_padinv[R_SLOTS], sl_tail[R_SLOTS], sl_meta[R_SLOTS], sl_expv[R_SLOTS];
  __shared__ uint64_t sl_cs0[R_SLOTS], sl_e[R_SLOTS];
  const uint32_t lane = __lane_id(), g = lane & 15;
  const uint32_t tid = threadIdx.x;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t* __restrict__ xch = inv + 4097;  // x^(8 * 4096 * k) mod P, k < R_KMAX
  const uint64_t n_cap = n;  // the descriptor (and WAL record) capacity
  if (n_dev) n = *n_dev < n ? *n_dev : n;  // count produced on the device (WAL scan, async table scan)
  if (blockIdx.x >= n) return;  // a grid sized by a bound: no range is dealt to this workgroup
  // A row's first range is its own ticket (the row index), and rows claim no shared chunk before they have
  // taken it: its descriptor is loaded, and then its first chunk, while the LDS image is built.
  const uint32_t row_wg = tid >> 4;
  const uint64_t i_first = blockIdx.x + (uint64_t)row_wg * gridDim.x;
  lcrc_desc_dev d_first{0, 0, LCRC_NO_EXPECT_DEV};
  if (!UNIFORM && i_first < n) d_first = descs[i_first];
  bool fresh = true, pre = true;
  const uint32_t voff_a = 256u * (lane & 7) + 16u * (lane >> 3), voff_b = voff_a + 128;
  u32x4 va[8], vb[8];
  {
    // the first chunk's start and limit exactly as the loop derives them below
    uint64_t s0 = UNIFORM ? i_first * ustride : d_first.offset;
    uint32_t len0 = UNIFORM ? ulen : d_first.length;
    if (!UNIFORM && (s0 > base_len || len0 > base_len - s0)) s0 = len0 = 0;
    const uint32_t d40 = (uint32_t)(s0 & 3);
    const uint32_t span0 = len0 + d40;
    const bool ovf0 = span0 > 4096 && span0 <= 4096 + R_OVF;
    const uint64_t ce0 = ovf0 ? s0 - d40 + 4096 : s0 + len0;
    const uint64_t lim = i_first < n ? (ce0 < base_len ? ce0 : base_len) : 0;
    const uint64_t csl = i_first < n ? s0 - d40 : 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint64_t B = readlane64(csl, 16 * (j >> 1)) + 2048u * (j & 1);
      const uint64_t lq = readlane64(lim, 16 * (j >> 1));
      const uint32_t nrec = lq > B ? (lq - B < 2048 ? (uint32_t)(lq - B) : 2048u) : 0u;
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void*)(base + (nrec ? B : 0)), (short)0, (int)nrec, 0x00020000);
      va[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff_a, 0, LCRC_LOAD_AUX);
      vb[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff_b, 0, LCRC_LOAD_AUX);
    }
  }
  build_tables(L, gtab, wv, lane);
  if (tid < R_SLOTS) sl_gen[tid] = 0;
  if (tid == 0) {
    ticket = A_THREADS / 16;
    work_mask = 0;
    free_mask = ~0u >> (32 - R_SLOTS);
  }
  lds_barrier();
  const Rot R = make_rot(lane);
  const __amdgpu_buffer_rsrc_t no_rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0, 0x00020000);
  // per-row state, uniform within the 16-lane row. mode 0: looking for work, 1: a private range (chunks
  // walked in order by this row), 2: one chunk of shared range `sl`.
  uint32_t mode = 0, sl = 0, xk = 0;
  uint64_t rng = 0, cs = 0, e = 0, ce = 0;  // range, chunk start, range end, end of its chunked part
  uint32_t acc = 0, padinv = 0, expv = 0, tail = 0, ntail = 0, d4 = 0;  // tail: bytes of a partial last dword
  uint32_t ovn = 0, ov0 = 0, ov1 = 0, ov2 = 0, ov3 = 0;  // whole dwords past a range's one full chunk
  bool ovf = false;  // the range's bytes past its one full chunk are walked on at the end
  bool first = false, has_exp = false, exp_ok = false, done = false, oob = false;
  while (true) {
    // 1. rows without work claim a chunk of a shared range ...
    const bool need = mode == 0 && !done;
    uint32_t got = R_SLOTS, gc = 0;
    if (need && !fresh && g == 0) {
      uint32_t m = *(volatile uint32_t*)&work_mask;
      while (m) {
        const uint32_t s = __builtin_ctz(m);
        m &= m - 1;
        const uint32_t r = atomicAdd(&sl_next[s], 1u);
        const uint32_t info = *(volatile uint32_t*)&sl_info[s];
        if ((r >> 16) == (info >> 16) && (r & 0xFFFFu) < (info & 0xFFFFu)) {
          if ((r & 0xFFFFu) == (info & 0xFFFFu) - 1) atomicAnd(&work_mask, ~(1u << s));  // the last chunk
          got = s;
          gc = r & 0xFFFFu;
          break;
        }
      }
    }
    got = row_bcast0(got, lane);
    gc = row_bcast0(gc, lane);
    if (need && got < R_SLOTS) {
      mode = 2;
      sl = got;
      const uint32_t nch = sl_info[sl] & 0xFFFFu;
      cs = sl_cs0[sl] + 4096ull * gc;
      e = sl_e[sl];
      ce = e;
      first = false;  // chunk 0 is walked by the row that shared the range
      xk = xch[nch - 1 - gc];
    }
    // ... or take the next range
    const bool need2 = need && got >= R_SLOTS;
    uint32_t v = 0;
    const bool use_first = need2 && fresh;
    if (need2 && !fresh && g == 0) v = atomicAdd(&ticket, 1u);
    v = use_first ? row_wg : row_bcast0(v, lane);
    if (need2) fresh = false;
    if (need2) {
      const uint64_t i = blockIdx.x + (uint64_t)v * gridDim.x;
      if (i >= n) {
        done = true;
      } else {
        uint64_t s;
        uint32_t len;
        int32_t xrel = LCRC_NO_EXPECT_DEV;
        uint64_t i_rec = i;  // the output slot (WAL scan: the record's file-order index)
        oob = false;
        if (UNIFORM) {
          s = i * ustride;
          len = ulen;
        } else {
          const lcrc_desc_dev d = use_first ? d_first : descs[i];
          s = d.offset;
          len = d.length;
          xrel = recs ? -6 : d.expect_rel;  // WAL scan: the record's file-order index, its CRC at -6
          if (recs) i_rec = (uint32_t)d.expect_rel;
          if (s > base_len || len > base_len - s) {  // never read: empty, CRC 0, flagged as a mismatch
            oob = true;
            s = 0;
            len = 0;
          }
        }
        rng = i_rec;
        d4 = (uint32_t)(s & 3);  // chunks start on the dword at or below s: aligned loads
        cs = s - d4;
        e = s + len;
        first = true;
        const uint32_t span = len + d4;
        // a range just past one chunk (a 4 KiB block and its type byte): one full chunk, the <= 16 bytes
        // after it walked on from the chunk's register at the end
        ovf = span > 4096 && span <= 4096 + R_OVF;
        const uint32_t nch = ovf ? 1u : span ? ((span - 1) >> 12) + 1 : 1u;
        padinv = inv[ovf ? 0 : (uint64_t)nch * 4096 - span];  // pad in [0, 4096]
        ce = ovf ? cs + 4096 : e;
        ovn = ovf ? (span - 4096) >> 2 : 0u;
        ov0 = ov1 = ov2 = ov3 = 0;
        if (ovn && g == 0) {
          const uint32_t* ow = (const uint32_t*)(base + cs + 4096);  // dword-aligned like cs
          ov0 = ow[0];
          if (ovn > 1) ov1 = ow[1];
          if (ovn > 2) ov2 = ow[2];
          if (ovn > 3) ov3 = ow[3];
        }
        // the range's bytes in a last dword that is not whole read as zeros: walked separately
        const uint64_t e4 = e & ~3ull;
        ntail = (uint32_t)(e - (e4 > s ? e4 : s));
        tail = 0;
        if (g == 0)
          for (uint32_t k = 0; k < ntail; ++k)
            if (e - ntail + k < base_len) tail |= (uint32_t)base[e - ntail + k] << (8 * k);
        has_exp = false;
        exp_ok = false;
        expv = 0;
        if (UNIFORM) {
          if (uexp) {
            has_exp = exp_ok = true;
            expv = uexp[i];
          }
        } else if (xrel != LCRC_NO_EXPECT_DEV && g == 0) {
          has_exp = true;
          const int64_t xp = (int64_t)s + xrel;
          exp_ok = !(xp < 0 || (uint64_t)xp + 4 > base_len);
          if (exp_ok) expv = load_le32(base + xp);
        }
        mode = 1;
        // share a range of several chunks through a free slot (a range past R_KMAX chunks stays private)
        uint32_t slot = R_SLOTS;
        if (g == 0 && nch > 1 && nch <= R_KMAX) {
          uint32_t fm = *(volatile uint32_t*)&free_mask;
          while (fm) {
            const uint32_t b = __builtin_ctz(fm);
            const uint32_t old = atomicAnd(&free_mask, ~(1u << b));
            if (old & (1u << b)) {
              slot = b;
              break;
            }
            fm = old & ~(1u << b);
          }
          if (slot < R_SLOTS) {
            const uint32_t gen = (sl_gen[slot] + 1) & 0xFFFFu;
            sl_gen[slot] = gen;
            sl_rng[slot] = (uint32_t)rng;  // the output slot (a WAL record: its file-order index)
            sl_cs0[slot] = cs;
            sl_e[slot] = e;
            sl_padinv[slot] = padinv;
            sl_tail[slot] = tail;
            sl_expv[slot] = expv;
            sl_meta[slot] = ntail | (has_exp ? 0x100u : 0u) | (exp_ok ? 0x200u : 0u) | (oob ? 0x400u : 0u);
            sl_acc[slot] = 0;
            sl_left[slot] = nch;
            sl_info[slot] = (gen << 16) | nch;
            __builtin_amdgcn_s_waitcnt(0xC07F);  // fields before the claim counter, counter before the bit
            sl_next[slot] = (gen << 16) | 1u;  // chunk 0 is this row's
            __builtin_amdgcn_s_waitcnt(0xC07F);
            atomicOr(&work_mask, 1u << slot);
          }
        }
        slot = row_bcast0(slot, lane);
        if (slot < R_SLOTS) {
          mode = 2;
          sl = slot;
          xk = xch[nch - 1];
        }
      }
    }
    const bool act = mode != 0;
    if (__builtin_amdgcn_ballot_w64(act) == 0) break;
    // 2. the rows' chunks; bytes past the range (or the buffer) end read as zeros
    const uint64_t lim = act ? (ce < base_len ? ce : base_len) : 0;
    const uint64_t csl = act ? cs : 0;
    if (!pre)  // (the first iteration's chunks were loaded before the tables)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint64_t B = readlane64(csl, 16 * (j >> 1)) + 2048u * (j & 1);
      const uint64_t lq = readlane64(lim, 16 * (j >> 1));
      const uint32_t nrec = lq > B ? (lq - B < 2048 ? (uint32_t)(lq - B) : 2048u) : 0u;
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void*)(base + (nrec ? B : 0)), (short)0, (int)nrec, 0x00020000);
      va[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff_a, 0, LCRC_LOAD_AUX);
      vb[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff_b, 0, LCRC_LOAD_AUX);
    }
    // a range's first chunk: zero the d4 bytes before the range and inject the start register at byte
    // d4. Before the transpose, window 0 of row q starts with register va[2q] of lane 0.
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t f = (uint32_t)__builtin_amdgcn_readlane((int)(first && act ? 1u : 0u), 16 * q);
      if (f) {
        const uint32_t dq = (uint32_t)__builtin_amdgcn_readlane((int)d4, 16 * q);
        const uint64_t sh = (uint64_t)init << (8 * dq);
        if (lane == 0) {
          va[2 * q].x = (va[2 * q].x & (~0u << (8 * dq))) ^ (uint32_t)sh;
          va[2 * q].y ^= (uint32_t)(sh >> 32);
        }
      }
    }
    pre = false;
    const uint32_t x = walk_half<false, false, false>(L, R, va, 0u, no_rs, voff_a);
    uint32_t p = walk_half<false>(L, R, vb, x, no_rs, voff_b);
    p = tree_level<0>(L, R, p, lane);
    p = tree_level<1>(L, R, p, lane);
    p = tree_level<2>(L, R, p, lane);
    p = tree_level<3>(L, R, p, lane);  // lane 0 of a row: the chunk's register
    // 3. combine. Private: acc = Z4096(acc) ^ C. Shared: slot ^= Z_{4096 (nch - 1 - c)}(C).
    const bool more = mode == 1 && !first;
    const bool shr = mode == 2;
    if (__builtin_amdgcn_ballot_w64((more || shr) && g == 0)) {
      const uint32_t z = gf_mul(shr ? xk : x4096, shr ? p : acc, poly);
      if (more) acc = z ^ p;
      if (shr) p = z;
    }
    if (mode == 1 && first) acc = p;
    first = false;
    bool fin = false;
    if (mode == 1) {
      cs += 4096;
      fin = cs >= ce;
    }
    uint32_t fin_slot = R_SLOTS;
    if (shr && g == 0) {
      atomicXor(&sl_acc[sl], p);
      if (atomicSub(&sl_left[sl], 1u) == 1u) fin_slot = sl;  // the range's last chunk: finish it here
    }
    fin_slot = row_bcast0(fin_slot, lane);
    if (shr && fin_slot < R_SLOTS) {
      fin = true;
      acc = *(volatile uint32_t*)&sl_acc[fin_slot];
      rng = sl_rng[fin_slot];
      padinv = sl_padinv[fin_slot];
      tail = sl_tail[fin_slot];
      expv = sl_expv[fin_slot];
      const uint32_t meta = sl_meta[fin_slot];
      ntail = meta & 0xFFu;
      has_exp = meta & 0x100u;
      exp_ok = meta & 0x200u;
      oob = meta & 0x400u;
      ovn = 0;
      ovf = false;
    }
    if (shr) mode = 0;
    // 4. finish: register = acc * x^(-8 pad) ^ walk(0, V)
    if (__builtin_amdgcn_ballot_w64(fin && g == 0)) {
      uint32_t raw = acc;
      // x^0 (reflected: bit 31) when the range fills its chunks exactly or runs on past one full chunk
      if (__builtin_amdgcn_ballot_w64(fin && g == 0 && padinv != 0x80000000u)) raw = gf_mul(padinv, acc, poly);
      // slice table T_t at LDS byte 256 * entry + 32 * t (set S0, replica 0)
      if (ovf) {  // walk on over the dwords and bytes past the full chunk
        for (uint32_t k = 0; k < ovn; ++k) {
          const uint32_t xw = raw ^ (k == 0 ? ov0 : k == 1 ? ov1 : k == 2 ? ov2 : ov3);
          raw = lds_u32(L, (xw & 255u) * 256u + 96u) ^ lds_u32(L, ((xw >> 8) & 255u) * 256u + 64u) ^
                lds_u32(L, ((xw >> 16) & 255u) * 256u + 32u) ^ lds_u32(L, (xw >> 24) * 256u);
        }
        for (uint32_t k = 0; k < ntail; ++k)
          raw = (raw >> 8) ^ lds_u32(L, ((raw ^ (tail >> (8 * k))) & 255u) * 256u);
      } else {  // + walk(0, V)
        for (uint32_t k = 0; k < ntail; ++k)
          raw ^= lds_u32(L, ((tail >> (8 * k)) & 255u) * 256u + 32u * (ntail - 1 - k));
      }
      if (fin && g == 0) {
        uint32_t crc = raw ^ xorout;
        if (flags & LCRC_FLAG_MASK) crc = mask32c(crc);
        if (oob) crc = 0;
        out[rng] = crc;
        const bool bad = oob || (has_exp && (!exp_ok || expv != crc));
        if (mismatch) mismatch_bit(mismatch, rng, n, bad, flags);
        if (recs && rng < n_cap) {  // WAL scan: the verdict of read_physical_record's checksum compare (log.rs:260-273)
          recs[rng].crc = crc;
          recs[rng].status = bad ? 1 : 0;
        }
        if (fin_slot < R_SLOTS) atomicOr(&free_mask, 1u << fin_slot);  // the slot's fields are read
      }
    }
    if (fin) mode = 0;
  }
}

// ---------------------------------------------------------------------------------------------------
// WAL scan: k_wal_parse walks the record headers of every 32 KiB log block exactly as
// LogReader::read_physical_record (src/db/log.rs:204-279) does, minus the checksum (k_blocks computes it,
// in parallel over all records, and stores it with the verdict in the record); k_wal_emit writes the
// records and their descriptors at their file-order positions. Nothing returns to the host in between.
// (Several logs, lcrc_wal_scan_queue: k_wal_parse_q walks every log's blocks in one launch, k_wal_emit_q emits.)
// ---------------------------------------------------------------------------------------------------
constexpr uint32_t WAL_SLOTS = 64;  // records per block kept by the parse (a block with more is re-walked)

// header of the record at in-block offset `at`: length (bytes 4..5) and type (byte 6), three independent
// byte loads in ONE memory round trip per hop of the walk (left alone, the compiler sinks the type load
// below the length check: two dependent round trips per record)
__device__ __forceinline__ void wal_header(const uint8_t* __restrict__ blk, uint32_t at, uint32_t& length,
                                           uint32_t& type) {
  uint32_t l0 = blk[at + 4], l1 = blk[at + 5], ty = blk[at + 6];
  __asm__ volatile("" : "+v"(l0), "+v"(l1), "+v"(ty));
  length = l0 | (l1 << 8);
  type = ty;
}

// one lane per block: record count, stop reason and the first WAL_SLOTS records as (offset | length << 16,
// type), and the wave's exclusive scan of the counts: local[b] (u32) and part[wave] (the total). One wave
// per workgroup, so the waves spread over the CUs instead of sharing one CU's address units four apiece.
// The walk is one dependent memory round trip per record, so the block with the most records sets the
// kernel's time.
constexpr uint32_t WAL_PARTB = 64;  // blocks per parse workgroup (= per part total)

// The WAL scan orders its record descriptors for k_blocks with the records whose covered bytes
// [h + 6, h + 7 + len) lie in one 256 B window of the file first (about half of the reference's random-read
// length mix): waves of them alone take the head walk only (k_blocks skips the row tree and the tail walk).
__device__ __forceinline__ uint32_t wal_single(uint64_t b, uint32_t at, uint32_t length) {
  const uint64_t s = b * 32768ull + at + 6;
  return (s >> 8) == ((s + length) >> 8) ? 1u : 0u;  // last covered byte s + length
}

__device__ __forceinline__ void wal_parse_body(const uint8_t* __restrict__ file, uint64_t file_len,
                                               uint64_t nblocks, uint32_t* __restrict__ counts,
                                               uint2* __restrict__ slots, uint8_t* __restrict__ stops,
                                               uint64_t* __restrict__ local, uint64_t* __restrict__ part,
                                               uint32_t bx) {
  const uint64_t b = (uint64_t)bx * 64 + threadIdx.x;
  const uint32_t lane = threadIdx.x;
  const uint8_t* blk = file + b * 32768ull;
  const uint64_t rem = b < nblocks ? file_len - b * 32768ull : 0;
  const uint32_t cap = rem < 32768ull ? (uint32_t)rem : 32768u;
  uint32_t consumed = 0, nrec = 0, nsingle = 0, stop = LCRC_WAL_STOP_TRAILER_DEV;
  while (cap - consumed >= 7) {
    uint32_t length, type;
    // bytes 4..7 at the header inside the block: ONE dword load per hop (the length and type bytes), instead of
    // three byte loads -- beside another scan's window pass a CU's address units are shared, and every lane's
    // hop is its own cache line (measured: WAL on two streams 3,494 vs 3,469 GiB/s, 6 alternated runs)
    if (cap - consumed >= 8) {
      typedef uint32_t u32_ua __attribute__((aligned(1)));
      const uint32_t v = *(const u32_ua*)(blk + consumed + 4);
      length = v & 0xFFFFu;
      type = (v >> 16) & 0xFFu;
    } else {
      wal_header(blk, consumed, length, type);
    }
    if (7 + length > cap - consumed) {
      stop = LCRC_WAL_STOP_BAD_LENGTH_DEV;
      break;
    }
    if (type == 0 && length == 0) {
      stop = LCRC_WAL_STOP_ZERO_DEV;
      break;
    }
    const uint32_t one = wal_single(b, consumed, length);  // the high count: one-window records
    const uint32_t tag = one << 8;
    if (nrec < WAL_SLOTS) slots[b * WAL_SLOTS + nrec] = make_uint2(consumed | (length << 16), type | tag);
    ++nrec;
    nsingle += one;
    consumed += 7 + length;
  }
  // wave exclusive scan by shuffles of (records | one-window records << 32)
  const uint64_t mine = (uint64_t)nrec | ((uint64_t)nsingle << 32);
  uint64_t inc = mine;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t v = __shfl_up(inc, d, 64);
    if (lane >= (uint32_t)d) inc += v;
  }
  if (b < nblocks) {
    counts[b] = nrec;
    stops[b] = (uint8_t)stop;
    local[b] = inc - mine;
  }
  if (lane == 63) part[bx] = inc;
}

__global__ void __launch_bounds__(64) k_wal_parse(const uint8_t* __restrict__ file, uint64_t file_len,
                                                  uint64_t nblocks, uint32_t* __restrict__ counts,
                                                  uint2* __restrict__ slots, uint8_t* __restrict__ stops,
                                                  uint64_t* __restrict__ local, uint64_t* __restrict__ part) {
  wal_parse_body(file, file_len, nblocks, counts, slots, stops, local, part, blockIdx.x);
}

// several logs in one launch (lcrc_wal_scan_queue): log blockIdx.y, its parse workgroups blockIdx.x
struct WalJobDev {
  const uint8_t* file;
  uint64_t file_len, nblocks;
  uint32_t* counts;
  uint2* slots;
  uint8_t* stops;
  uint64_t* local;
  uint64_t* part;
  lcrc_wal_rec_dev* recs;
  lcrc_desc_dev* descs;
  uint64_t max_recs;
  uint64_t* n_total;
  uint64_t* n_out;
};
constexpr int MAX_WJOBS = 16;  // logs per launch (kernel-argument space: 16 x 104 B)
struct WalJobsArg {
  WalJobDev j[MAX_WJOBS];
};

__global__ void __launch_bounds__(64) k_wal_parse_q(const WalJobsArg jobs) {
  const WalJobDev& J = jobs.j[blockIdx.y];
  if ((uint64_t)blockIdx.x * WAL_PARTB >= J.nblocks) return;  // past this log's blocks (workgroup-uniform)
  wal_parse_body(J.file, J.file_len, J.nblocks, J.counts, J.slots, J.stops, J.local, J.part, blockIdx.x);
}

// record o (file order) and its verify descriptor at position pos of k_blocks' order. The descriptor's
// expect_rel carries o (the expected CRC of a WAL record is always at -6: k_blocks and k_ranges read it there
// and store the crc and verdict in recs[o]).
__device__ __forceinline__ void wal_put(lcrc_wal_rec_dev* __restrict__ recs, lcrc_desc_dev* __restrict__ descs,
                                        uint64_t o, uint64_t pos, uint64_t max_recs, uint64_t header, uint32_t length,
                                        uint32_t type, bool last, uint32_t stop) {
  if (o < max_recs) {
    lcrc_wal_rec_dev rr;
    rr.header = header;
    rr.length = length;
    rr.type = (uint8_t)type;
    rr.status = 0;
    rr.block_end = last ? 1 : 0;
    rr.crc = 0;
    rr.stop = last ? stop : 0;
    recs[o] = rr;
  }
  if (pos < max_recs) {
    lcrc_desc_dev d;
    d.offset = header + 6;
    d.length = 1 + length;
    d.expect_rel = (int32_t)(uint32_t)o;
    descs[pos] = d;
  }
}

// one thread per (block, slot), one wave per block: records in file order at first(b) + i (those below
// max_recs); the thread of the last slot re-walks a block that has more records than slots. Packed counts
// (records | one-window records << 32): first(b) = the parse workgroups' totals before b's workgroup (summed
// by each emit workgroup) + local[b]. Descriptors: the one-window records first, then the others, each in file
// order (both only when every record fits max_recs; else in file order). Workgroup 0 also writes the total
// record count to n_total (device) and n_out (device or pinned host memory).
__device__ __forceinline__ void wal_emit_body(const uint8_t* __restrict__ file, uint64_t nblocks,
                                              const uint32_t* __restrict__ counts,
                                              const uint2* __restrict__ slots, const uint8_t* __restrict__ stops,
                                              const uint64_t* __restrict__ local,
                                              const uint64_t* __restrict__ part,
                                              lcrc_wal_rec_dev* __restrict__ recs,
                                              lcrc_desc_dev* __restrict__ descs, uint64_t max_recs,
                                              uint64_t* __restrict__ n_total, uint64_t* __restrict__ n_out,
                                              uint32_t bx) {
  const uint64_t g = (uint64_t)bx * blockDim.x + threadIdx.x;
  const uint64_t b = g / WAL_SLOTS;
  const uint32_t i = (uint32_t)(g % WAL_SLOTS);
  const uint64_t nparts = (nblocks + WAL_PARTB - 1) / WAL_PARTB;
  // the totals of all parse workgroups, and of those before this wave's block: one wave per block (64 slots),
  // each wave sums the parts itself (lane-strided loads and a butterfly: no barrier, no LDS)
  static_assert(WAL_SLOTS == 64, "one wave per block");
  const uint64_t mine = b / WAL_PARTB;
  uint64_t total = 0, before = 0;
  for (uint64_t w = i; w < nparts; w += 64) {
    const uint64_t v = part[w];
    total += v;
    if (w < mine) before += v;
  }
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    total += __shfl_xor(total, d, 64);
    before += __shfl_xor(before, d, 64);
  }
  const uint64_t tot_r = (uint32_t)total, tot_s = total >> 32;
  if (bx == 0 && threadIdx.x == 0) {
    *n_total = tot_r;
    if (n_out) *n_out = tot_r;
  }
  if (b >= nblocks || max_recs == 0) return;  // wave-uniform
  const bool split = tot_r <= max_recs;
  const uint32_t cnt = counts[b];
  const uint64_t loc = local[b];
  const uint64_t first = (uint32_t)before + (uint32_t)loc;           // file order
  const uint64_t first_s = (before >> 32) + (loc >> 32);             // one-window records before b
  const uint64_t first_m = tot_s + first - first_s;                  // the others, after every one-window one
  uint2 sl = make_uint2(0, 0);
  if (i < cnt) sl = slots[g];
  const uint32_t one = (sl.y >> 8) & 1u;
  const uint64_t ones = __builtin_amdgcn_ballot_w64(i < cnt && one);
  const uint32_t rank_s = __builtin_popcountll(ones & ((1ull << i) - 1));
  if (i >= cnt) return;
  uint32_t at = sl.x & 0xFFFFu, length = sl.x >> 16;
  const uint64_t o = first + i;
  uint64_t pos = !split ? o : one ? first_s + rank_s : first_m + (i - rank_s);
  wal_put(recs, descs, o, pos, max_recs, b * 32768ull + at, length, sl.y & 0xFFu, i + 1 == cnt, stops[b]);
  if (i == WAL_SLOTS - 1 && cnt > WAL_SLOTS) {
    const uint8_t* blk = file + b * 32768ull;
    uint64_t ns = __builtin_popcountll(ones), nm = WAL_SLOTS - ns;
    for (uint32_t j = WAL_SLOTS; j < cnt; ++j) {  // the parse already validated every header up to cnt
      at += 7 + length;
      uint32_t type;
      wal_header(blk, at, length, type);
      const uint32_t one_j = wal_single(b, at, length);
      const uint64_t oj = first + j;
      pos = !split ? oj : one_j ? first_s + ns : first_m + nm;
      ns += one_j;
      nm += 1 - one_j;
      wal_put(recs, descs, oj, pos, max_recs, b * 32768ull + at, length, type, j + 1 == cnt, stops[b]);
    }
  }
}

__global__ void __launch_bounds__(256) k_wal_emit(const uint8_t* __restrict__ file, uint64_t nblocks,
                                                  const uint32_t* __restrict__ counts,
                                                  const uint2* __restrict__ slots, const uint8_t* __restrict__ stops,
                                                  const uint64_t* __restrict__ local,
                                                  const uint64_t* __restrict__ part,
                                                  lcrc_wal_rec_dev* __restrict__ recs,
                                                  lcrc_desc_dev* __restrict__ descs, uint64_t max_recs,
                                                  uint64_t* __restrict__ n_total, uint64_t* __restrict__ n_out) {
  wal_emit_body(file, nblocks, counts, slots, stops, local, part, recs, descs, max_recs, n_total, n_out,
                       blockIdx.x);
}

__global__ void __launch_bounds__(256) k_wal_emit_q(const WalJobsArg jobs) {
  const WalJobDev& J = jobs.j[blockIdx.y];
  // past this log's (block, slot) threads: workgroup 0 always runs (it writes the total)
  if (blockIdx.x && (uint64_t)blockIdx.x * 256 >= J.nblocks * WAL_SLOTS) return;
  wal_emit_body(J.file, J.nblocks, J.counts, J.slots, J.stops, J.local, J.part, J.recs, J.descs, J.max_recs,
                       J.n_total, J.n_out, blockIdx.x);
}

// ---------------------------------------------------------------------------------------------------
// Snappy framing (the `snap` crate's FrameEncoder / FrameDecoder used for compressed SSTable blocks,
// src/sstable/table.rs:481-497, src/sstable/format.rs:194-206; framing format: stream identifier
// ff 06 00 00 "sNaPpY", chunks [type u8][length u24 LE][body]; data chunks 0x00 (Snappy-compressed) and
// 0x01 (uncompressed) start with the masked CRC-32C of their uncompressed bytes, at most 65,536 of them;
// 0xfe padding and 0x80..0xfd are skipped, 0x02..0x7f are fatal). One lane per frame walks its chunks;
// the chunk CRCs are computed by the general path over the decoded bytes.
// ---------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ld_u8(const uint8_t* p) { return *p; }

// The Snappy raw-format length preamble of a compressed chunk's data, as the snap crate (Cargo.toml:15, "1") reads it
// for FrameDecoder (format.rs:196): bytes::read_varu64 -- up to 10 bytes, the value taken mod 2^64 (a byte's bits
// shifted past bit 63 are dropped, an 11th byte is an error) -- and the frame decoder then rejects a decoded length
// over MAX_BLOCK_SIZE (65,536). byte(i) reads preamble byte i (i < n). True with ulen (<= 65,536) and used (the
// preamble's bytes) when the chunk's length is acceptable; a 5-byte preamble of 2^32 is NOT a zero length.
template <class ByteAt>
__device__ __forceinline__ bool snappy_preamble(ByteAt byte, uint32_t n, uint32_t& ulen, uint32_t& used) {
  uint64_t v = 0;
  ulen = 0;
  used = 0;
  for (uint32_t i = 0; i < 10 && i < n; ++i) {
    const uint32_t b = byte(i);
    v |= (uint64_t)(b & 127u) << (7 * i);
    if (!(b & 128)) {
      used = i + 1;
      ulen = v <= 65536 ? (uint32_t)v : 0u;
      return v <= 65536;
    }
  }
  return false;
}
// snap's FrameDecoder reads a chunk body into a buffer of MAX_COMPRESS_BLOCK_SIZE = 76,490 bytes (the worst-case
// compressed size of a 64 KiB block): any chunk longer than that, of any type, is an error
constexpr uint32_t SN_MAX_CHUNK = 76490;

// the framing walk of one frame p[0, len): decoded size, data-chunk count, largest compressed data (after the
// crc) and decoded chunk; false when the framing is malformed
// padded: the bytes the table scan's decode takes, each chunk 16-aligned with its stored CRC in the 16 B after it
// LDS staging of the wave decoders: compressed bytes + SN_SLACK for the parse windows' header reads, then the decoded
// bytes, each at most SN_MAX (k_snappy_decode_wave sizes them from the batch's largest chunk)
constexpr uint32_t SN_SLACK = 128;
constexpr uint32_t SN_MAX = 16384;
// k_ts_decode (the whole-table scan's decode): TD_WAVES waves per 256-block tile. Each wave decodes 64 / TD_RL frames
// at once, one per TD_RL-lane row. A row (TR_ROW bytes of LDS) decodes IN PLACE: the frame is staged at the row's end
// and the chunk decoded from the row's start, the output growing towards the unread input. Round 6: the chunk CRC
// masks the bytes past the chunk's end instead of zero-filling the row to whole 1 KiB passes, so a row holds the chunk
// itself (a db_bench-style 4 KiB block decodes to ~4,125 B and needs at most 4,132 B of row with its frame staged
// behind the output), and only the row path's CRC tables stay in LDS; and rows are 8 lanes, not 16: a Snappy element
// of the bench's blocks is 39 B on average (41 literals of ~50 B and 65 copies a 4 KiB block), so a 16-lane row moved
// it with half its lanes idle while the element loop's ~110 instructions served four frames. With eight frames a wave
// the loop's instructions per frame halve; LDS (32 rows a CU) then holds four waves, one a SIMD. A frame of over TR_IN
// bytes (the register staging), a chunk of over TR_OUT, or one whose output would reach its own unread input goes
// through the whole-wave decoder afterwards, in its wave's row area (TD_IN + TD_OUT); a chunk too large for that,
// lane-serially to the workspace.
#ifndef LCRC_TD_RL
#define LCRC_TD_RL 8  // lanes a row (measurement builds: 16, with eight waves of four rows)
#endif
constexpr uint32_t TD_RL = LCRC_TD_RL;
static_assert(TD_RL == 8 || TD_RL == 16, "rows of 8 or 16 lanes");
constexpr uint32_t TD_RPW = 64 / TD_RL;     // rows (frames in flight) a wave
constexpr uint32_t TD_PASS = 8 * TD_RL;     // bytes a row moves per pass (8 a lane)
constexpr uint32_t TD_WAVES = 32 / TD_RPW;  // 32 rows a workgroup (one a CU: the LDS)
constexpr uint32_t TD_TAB_WORDS = TAB_ZWIN + 3 * 1024;  // T0..T3, Z16..Z128, Z256, Z512, Z1024 (at their TAB_* offsets)
// k_ts_decode's LDS table image (words): T0..T3, then the table image's Z_(1024 / TD_RL) .. Z1024 (the row tree's
// joins of lane pieces of 1024 / TD_RL bytes, Z1024 chaining the passes); the shorter shifts stay in global memory
constexpr uint32_t TDL_ZSRC = TD_RL == 16 ? TAB_ZPIECE + 2 * 1024 : TAB_ZPIECE + 3 * 1024;  // Z64 or Z128
constexpr uint32_t TDL_Z64 = 1024;  // (TD_RL = 16 only)
constexpr uint32_t TDL_Z128 = 1024 + (TAB_ZPIECE + 3 * 1024 - TDL_ZSRC), TDL_Z256 = TDL_Z128 + 1024;
constexpr uint32_t TDL_Z512 = TDL_Z256 + 1024, TDL_Z1024 = TDL_Z512 + 1024, TDL_WORDS = TDL_Z1024 + 1024;
static_assert(TAB_SLICE == 0 && TAB_ZWIN == TAB_ZPIECE + 4 * 1024 && TD_TAB_WORDS == TAB_ZWIN + 3 * 1024,
              "k_ts_decode's image: the slice tables, then the table image's Z64 or Z128 .. Z1024 in order");
// a row's frame (+ the slack of its element-header reads): frames up to 2,701 B (db_bench-style 4 KiB blocks: <= 2,298)
constexpr uint32_t TR_IN = 2704 + 16;
#ifndef LCRC_TD_ROW
#define LCRC_TD_ROW (LCRC_TD_RL == 8 ? 4320 : 4192)
#endif
constexpr uint32_t TR_ROW = LCRC_TD_ROW;  // the row's decoded chunk + 16 B of slack (header reads past the input,
constexpr uint32_t TR_OUT = TR_ROW - 16;  // the dump dword)
constexpr uint32_t TD_WAVE_LDS = TD_RPW * TR_ROW;
constexpr uint32_t TD_IN = 12288 + 16;   // the whole-wave decoder's staging: compressed bytes (+ 4 for the tail dword)
constexpr uint32_t TD_OUT = 16384;       // decoded bytes (a multiple of 1 KiB: V fits as is)
static_assert(TD_OUT % 1024 == 0, "the chunk CRC reads V in whole 1 KiB passes");
static_assert(TR_ROW % 16 == 0 && TR_IN + 16 <= TR_ROW && TR_OUT >= 4096, "row staging");
// the whole-wave decoder's staging: one wave's row area, or two (TD_WW waves then share one decoder)
constexpr uint32_t TD_WW = TD_IN + SN_SLACK + TD_OUT <= TD_WAVE_LDS ? 1 : 2;
static_assert(TD_WAVES % TD_WW == 0 && TD_IN + SN_SLACK + TD_OUT <= TD_WW * TD_WAVE_LDS,
              "the whole-wave decoder's staging is one or two waves' row areas");
constexpr uint32_t TD_LDS = TDL_WORDS * 4 + TD_WAVES * TD_WAVE_LDS + 256 + 16 + 16;  // + the rows' zero piece
static_assert(TD_LDS + 4160 + 344 <= 163840, "k_ts_decode's LDS leaves room for k_ts_finish");
// workgroups per 256-block tile of k_ts_finish: each takes TD_SUBN = 256 / TD_SUB frames (round 6: two, so that the
// decode's work is dealt in ~200 us pieces -- with one workgroup a tile, all 256 resident at once, a CU held by the
// other stream's index decode (k_ts_open2, ~210 us, a whole CU's LDS too) delayed its tile's whole decode by that
// much; four sub-tiles cost 26 us more alone: each workgroup's table image, gate and slowest-wave barrier)
#ifndef LCRC_TD_SUB
#define LCRC_TD_SUB 2
#endif
constexpr uint32_t TD_SUB = LCRC_TD_SUB, TD_SUBN = 256 / TD_SUB;
static_assert(TD_SUBN * TD_SUB == 256 && TD_SUBN % (TD_RPW * TD_WAVES) == 0, "whole groups a wave");

// `slow`: the decoded bytes (16-aligned) of the compressed chunks too large for k_ts_decode's LDS staging (TD_IN
// compressed, TD_OUT decoded), which it decodes lane-serially into the table scan's workspace
__device__ __forceinline__ bool snappy_frame_size(const uint8_t* __restrict__ p, uint32_t len, uint64_t& total,
                                                  uint64_t& chunks, uint32_t& max_in, uint32_t& max_out,
                                                  uint64_t& padded, uint64_t* slow = nullptr) {
  total = 0;
  padded = 0;
  if (slow) *slow = 0;
  chunks = 0;
  max_in = 0;
  max_out = 0;
  bool ok = true, seen_id = false;
  uint32_t at = 0;
  while (ok && at < len) {
    if (len - at < 4) {
      ok = false;
      break;
    }
    const uint32_t type = ld_u8(p + at);
    const uint32_t cl = ld_u8(p + at + 1) | (ld_u8(p + at + 2) << 8) | (ld_u8(p + at + 3) << 16);
    at += 4;
    if (len - at < cl || cl > SN_MAX_CHUNK) {
      ok = false;
      break;
    }
    if (type == 0xff) {
      ok = cl == 6 && ld_u8(p + at) == 's' && ld_u8(p + at + 1) == 'N' && ld_u8(p + at + 2) == 'a' &&
           ld_u8(p + at + 3) == 'P' && ld_u8(p + at + 4) == 'p' && ld_u8(p + at + 5) == 'Y';
      seen_id = true;
    } else if (!seen_id) {
      ok = false;
    } else if (type <= 1) {
      uint32_t ulen = cl >= 4 ? cl - 4 : 0, used = 0;
      if (cl < 4) ok = false;
      else if (type == 0) ok = snappy_preamble([&](uint32_t i) { return ld_u8(p + at + 4 + i); }, cl - 4, ulen, used);
      if (ulen > 65536) ok = false;
      if (type == 0 && cl - 4 > max_in) max_in = cl - 4;
      if (ulen > max_out) max_out = ulen;
      total += ulen;
      padded += ((ulen + 15) & ~15u) + 16;
      if (slow && type == 0 && (ulen > TD_OUT || cl - used + 4 > TD_IN + 4)) *slow += (ulen + 15) & ~15u;
      ++chunks;
    } else if (type <= 0x7f) {
      ok = false;  // reserved unskippable
    }
    at += cl;
  }
  return ok;
}

// pass 1: decoded size, data-chunk count and framing verdict of every frame
__global__ void __launch_bounds__(256) k_snappy_size(const uint8_t* __restrict__ base,
                                                     const lcrc_desc_dev* __restrict__ frames, uint64_t n,
                                                     uint64_t* __restrict__ size, uint64_t* __restrict__ nchunks,
                                                     uint8_t* __restrict__ status, uint32_t* __restrict__ maxes,
                                                     const uint64_t* __restrict__ n_dev) {
  if (n_dev) n = *n_dev < n ? *n_dev : n;  // the count produced on the device
  const uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint8_t* p = f < n ? base + frames[f].offset : base;
  const uint32_t len = f < n ? frames[f].length : 0u;
  uint64_t total, chunks;
  uint32_t max_in, max_out;
  uint64_t padded;
  const bool ok = snappy_frame_size(p, len, total, chunks, max_in, max_out, padded);
  if (f < n) {
    size[f] = ok ? total : 0;
    nchunks[f] = ok ? chunks : 0;
    status[f] = ok ? 0 : 1;
  }
  // one atomic per wave (the build turns the compiler's atomic combining off for the hot kernels)
  uint32_t mi = ok ? max_in : 0u, mo = ok ? max_out : 0u;
  for (int d = 1; d < 64; d <<= 1) {
    mi = max(mi, (uint32_t)__shfl_xor((int)mi, d, 64));
    mo = max(mo, (uint32_t)__shfl_xor((int)mo, d, 64));
  }
  if (__lane_id() == 0) {
    if (mi) atomicMax(&maxes[0], mi);
    if (mo) atomicMax(&maxes[1], mo);
  }
}

// exclusive scans of two u64 arrays (n entries): per-workgroup part, then every element adds the totals
// of the workgroups before it; out_a[n], out_b[n] = the totals
__global__ void __launch_bounds__(256) k_scan2_local(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b,
                                                     uint64_t n, uint64_t* __restrict__ out_a,
                                                     uint64_t* __restrict__ out_b, uint64_t* __restrict__ part,
                                                     const uint64_t* __restrict__ n_dev) {
  __shared__ uint64_t sa[256], sb[256];
  if (n_dev) n = *n_dev < n ? *n_dev : n;
  if ((uint64_t)blockIdx.x * 256 > n) return;  // past the device count (the grid is sized by a bound)
  const uint32_t t = threadIdx.x;
  const uint64_t i = (uint64_t)blockIdx.x * 256 + t;
  const uint64_t va = i < n ? a[i] : 0, vb = i < n ? b[i] : 0;
  sa[t] = va;
  sb[t] = vb;
  __syncthreads();
  for (uint32_t d = 1; d < 256; d <<= 1) {
    const uint64_t xa = t >= d ? sa[t - d] : 0, xb = t >= d ? sb[t - d] : 0;
    __syncthreads();
    sa[t] += xa;
    sb[t] += xb;
    __syncthreads();
  }
  if (i < n) {
    out_a[i] = sa[t] - va;
    out_b[i] = sb[t] - vb;
  }
  if (t == 255) {
    part[2 * blockIdx.x] = sa[255];
    part[2 * blockIdx.x + 1] = sb[255];
  }
}

__global__ void __launch_bounds__(256) k_scan2_add(uint64_t n, uint64_t* __restrict__ out_a,
                                                   uint64_t* __restrict__ out_b, const uint64_t* __restrict__ part,
                                                   const uint64_t* __restrict__ n_dev) {
  __shared__ uint64_t ra[256], rb[256];
  const uint32_t t = threadIdx.x;
  if (n_dev) n = *n_dev < n ? *n_dev : n;
  const uint64_t nparts = (n + 255) / 256;
  const uint64_t last = nparts ? nparts - 1 : 0;  // the workgroup that also writes the totals
  if (blockIdx.x > last) return;
  const uint64_t upto = blockIdx.x == last ? nparts : blockIdx.x;
  uint64_t xa = 0, xb = 0, ma = 0, mb = 0;
  for (uint64_t w = t; w < upto; w += 256) {
    xa += part[2 * w];
    xb += part[2 * w + 1];
    if (w < blockIdx.x) {
      ma += part[2 * w];
      mb += part[2 * w + 1];
    }
  }
  ra[t] = ma;
  rb[t] = mb;
  __syncthreads();
  for (uint32_t d = 128; d; d >>= 1) {
    if (t < d) {
      ra[t] += ra[t + d];
      rb[t] += rb[t + d];
    }
    __syncthreads();
  }
  const uint64_t ba = ra[0], bb = rb[0];
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * 256 + t;
  if (i < n) {
    out_a[i] += ba;
    out_b[i] += bb;
  }
  if (blockIdx.x == last) {
    ra[t] = xa;
    rb[t] = xb;
    __syncthreads();
    for (uint32_t d = 128; d; d >>= 1) {
      if (t < d) {
        ra[t] += ra[t + d];
        rb[t] += rb[t + d];
      }
      __syncthreads();
    }
    if (t == 0) {
      out_a[n] = ra[0];
      out_b[n] = rb[0];
    }
  }
}

// pass 2, one wave per frame: decode frame f into out[out_off[f] ..) and describe its data chunks for the
// CRC pass -- cdesc (offset into out, length), cexp (stored masked CRC-32C), cframe (frame index).
// Chunk headers are read through two 256 B register windows (lane j holds dword j; a byte is one
// v_readlane with a scalar index). A compressed chunk is staged into LDS with dword loads, decoded in LDS
// (snappy_wave_decode) and leaves LDS with 16 B per lane. Chunks over the LDS staging take a lane-serial
// path from and to global memory.

__device__ __forceinline__ uint32_t bcast(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

struct sn_reader {
  const uint8_t* a;  // 4-byte aligned start (positions are relative to it)
  uint32_t lim;      // readable bytes from a
  uint32_t k;        // cur covers [256 k, 256 k + 256), nxt the next 256 B
  uint32_t cur, nxt;

  __device__ __forceinline__ uint32_t load(uint32_t w, uint32_t lane) const {
    const uint32_t i = 256u * w + 4u * lane;
    return i < lim ? *(const uint32_t*)(a + i) : 0u;  // the aligned dword of a readable byte is mapped
  }
  __device__ __forceinline__ void init(const uint8_t* p, uint32_t len, uint32_t lane) {
    a = p - ((uintptr_t)p & 3);  // pointer arithmetic keeps the global address space (no flat loads)
    lim = (uint32_t)(p - a) + len;
    k = 0;
    cur = load(0, lane);
    nxt = load(1, lane);
  }
  __device__ __forceinline__ void ensure(uint32_t i, uint32_t lane) {  // cur covers i (i never decreases)
    const uint32_t w = i >> 8;
    if (w == k + 1) {
      cur = nxt;
      k = w;
      nxt = load(w + 1, lane);
    } else if (w != k) {
      k = w;
      cur = load(w, lane);
      nxt = load(w + 1, lane);
    }
  }
  __device__ __forceinline__ uint32_t byte(uint32_t i) const {  // i in [256 k, 256 k + 512)
    const uint32_t dw = (uint32_t)__builtin_amdgcn_readlane((int)((i >> 8) == k ? cur : nxt), (int)((i >> 2) & 63));
    return (dw >> ((i & 3) * 8)) & 255u;
  }
  __device__ __forceinline__ uint32_t le(uint32_t i, uint32_t nb) const {  // nb <= 4 bytes little-endian
    uint32_t v = 0;
    for (uint32_t t = 0; t < nb; ++t) v |= byte(i + t) << (8 * t);
    return v;
  }
};

// Decode the Snappy elements staged at in[q, qe) (LDS) into o[0, ulen) (LDS); false when malformed.
// Parsing is data-parallel: for a window of 64 candidate start positions base + lane, every lane decodes
// the element that WOULD start at its byte (tag, header size, output length, offset or literal source)
// and where the next one would start; the real starts are then the chain from lane 0, followed with one
// v_readlane per element. A masked wave scan gives every element its output position, one ballot
// validates the window, and the elements are executed in order: a literal is an LDS -> LDS copy, a copy
// moves up to 64 bytes in one pass (a copy whose offset is shorter than its length repeats the last `off`
// bytes: lane k takes byte k mod off of them). The next window starts where the chain left this one.
// (Executing several elements per LDS round trip when their sources are outside the batch's output was
// tried: the hazard bookkeeping is scalar work per element and lost 2.5x on chained copies.)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, uint32_t lane) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);  // row_shr:8
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
  const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
  const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 47);
  return v + (lane >= 16 ? r0 : 0u) + (lane >= 32 ? r1 : 0u) + (lane >= 48 ? r2 : 0u);
}

// x mod a for x < 64, 1 <= a <= 64: (x + 1/2) / a is at least 1/(2a) away from an integer, far beyond
// the error of v_rcp_f32, so the floored quotient is exact
__device__ __forceinline__ uint32_t small_mod(uint32_t x, uint32_t a) {
  const float q = __builtin_floorf(((float)x + 0.5f) * __builtin_amdgcn_rcpf((float)a));
  return x - (uint32_t)q * a;
}

typedef __attribute__((address_space(3))) uint8_t lds_u8;
// ndw dwords from global za (4-byte aligned) to LDS dst (16-byte aligned) by nl lanes (li: the lane's index among
// them): whole 16 B units, eight per lane loaded before any is stored -- one memory latency per group, not one per
// dword as a plain copy loop waits -- then the last 0..3 dwords (no read beyond the dword holding the last byte)
__device__ __forceinline__ void stage_to_lds(const uint32_t* za, lds_u8* dst, uint32_t ndw, uint32_t li, uint32_t nl) {
  typedef __attribute__((address_space(3))) u32x4 lds_u32x4_t;
  typedef __attribute__((address_space(3))) uint32_t lds_u32_t;
  const uint32_t units = ndw >> 2;
  for (uint32_t b = 0; b < units; b += 8 * nl) {
    u32x4 t[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t u = b + li + nl * i;
      if (u < units) t[i] = *(const u32x4_ua*)(za + 4 * u);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t u = b + li + nl * i;
      if (u < units) *(lds_u32x4_t*)(dst + 16 * u) = t[i];
    }
  }
  if (li < (ndw & 3)) ((lds_u32_t*)dst)[4 * units + li] = za[4 * units + li];
}
__device__ bool snappy_wave_decode(const uint8_t* in_g, uint32_t q, uint32_t qe, uint8_t* o_g, uint32_t ulen,
                                   uint32_t lane) {
  // both staging buffers are LDS: say so, so that every access is a ds_ op (a generic pointer picked between them at
  // run time would become a flat access waiting on the vector memory counter too)
  const lds_u8* const in = (const lds_u8*)in_g;
  lds_u8* const o = (lds_u8*)o_g;
  uint32_t w0 = 0;  // bytes written before this window
  for (uint32_t base = q; base < qe;) {
    const uint32_t i = base + lane;  // candidate start (reads stay inside the staging's slack)
    const uint32_t t = in[i], b1 = in[i + 1], b2 = in[i + 2], b3 = in[i + 3], b4 = in[i + 4];
    const uint32_t typ = t & 3;
    const uint32_t room = qe > i ? qe - i : 0;  // input bytes from the candidate start
    uint32_t hdr, outlen, a;                     // a: copy offset, or the literal's source position
    bool good;
    if (typ == 0) {
      const uint32_t L = t >> 2;
      const uint32_t nb = L >= 60 ? L - 59 : 0;
      const uint32_t ext = b1 | (b2 << 8) | (b3 << 16) | (b4 << 24);
      const uint32_t lm1 = nb ? (nb == 4 ? ext : ext & ((1u << (8 * nb)) - 1)) : L;
      hdr = 1 + nb;
      outlen = lm1 + 1;
      a = i + hdr;
      good = room >= hdr && lm1 < room - hdr && (nb == 0 || room >= 5);  // bytes inside the input (no u32 wrap);
      // an extended length needs 4 bytes after the tag whatever nb is (snap's read_literal reads one 4-byte word)
    } else {
      hdr = typ == 1 ? 2 : typ == 2 ? 3 : 5;
      outlen = typ == 1 ? 4 + ((t >> 2) & 7) : 1 + (t >> 2);
      a = typ == 1 ? ((t >> 5) << 8) | b1 : typ == 2 ? b1 | (b2 << 8) : b1 | (b2 << 8) | (b3 << 16) | (b4 << 24);
      good = room >= hdr;
    }
    const uint32_t size = typ == 0 ? hdr + outlen : hdr;
    const uint32_t nxt = good ? lane + size : 0x7FFFFFFFu;
    // the chain of real element starts in this window
    const uint32_t lim = qe - base < 64 ? qe - base : 64;
    uint64_t mask = 0;
    uint32_t cur = 0;
    while (cur < lim) {
      mask |= 1ull << cur;
      cur = (uint32_t)__builtin_amdgcn_readlane((int)nxt, (int)cur);
    }
    const bool sel = (mask >> lane) & 1;
    const uint32_t v = sel ? outlen : 0u;
    const uint32_t incl = wave_incl_scan(v, lane);
    const uint32_t w = w0 + incl - v;
    const bool bad = sel && (!good || w > ulen || outlen > ulen - w || (typ != 0 && (a == 0 || a > w)));
    if (__builtin_amdgcn_ballot_w64(bad)) return false;
    // Each element's source: in[sa + f(i)] (a literal's bytes, or a copy whose whole source lies in the literal just
    // before it -- the usual Snappy shape of repeated text -- read from that literal's input bytes instead), or
    // o[sa + f(i)]; f(i) = i, or i mod `per` for a copy shorter-offset than it is long (it repeats its last `per` bytes).
    const int pj = 63 - __builtin_clzll((mask & ((1ull << lane) - 1)) | 1ull);  // the previous element's lane
    const bool has_prev = (mask & ((1ull << lane) - 1)) != 0;
    const uint32_t pw_ = (uint32_t)__builtin_amdgcn_ds_bpermute(pj * 4, (int)w);
    const uint32_t pl_ = (uint32_t)__builtin_amdgcn_ds_bpermute(pj * 4, (int)(typ == 0 ? outlen : 0u));  // 0: not a literal
    const uint32_t pa_ = (uint32_t)__builtin_amdgcn_ds_bpermute(pj * 4, (int)a);
    uint32_t sa = a, per = 0, from_in = 1;
    if (typ != 0) {
      per = a < outlen ? a : 0u;
      sa = w - a;
      from_in = 0;
      const uint32_t s_hi = per ? w : w - a + outlen;  // end of the output bytes the copy reads
      if (has_prev && pl_ && sa >= pw_ && s_hi <= pw_ + pl_) {
        sa = pa_ + (sa - pw_);
        from_in = 1;
      }
    }
    const uint32_t pw = (w & 0xFFFFu) | ((outlen - 1) << 16);  // w < ulen <= SN_MAX, outlen <= SN_MAX
    const uint32_t ps = sa | (from_in << 31);
    // Execute in order, in batches of up to four elements: the batch's bytes are all read, then all written (one LDS
    // round trip per batch instead of one per element). An element joins the batch only when its source lies outside
    // the batch's own output (a literal, a copy resolved to its literal's input bytes, or a copy of earlier output);
    // a literal over 64 bytes runs alone, pass by pass.
    uint64_t m = mask;
    while (m) {
      // the batch, chosen with scalar work only (no loaded value crosses a branch: the reads below are unconditional)
      uint32_t eo[4], eln[4], esa[4], eper[4];
      bool ein[4];
      uint32_t cnt = 0, bo = 0;
      bool long_lit = false;
      uint64_t mm = m;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        eo[k] = 0;
        eln[k] = 0;
        esa[k] = 0;
        eper[k] = 0;
        ein[k] = true;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (mm == 0 || cnt < (uint32_t)k) continue;
        const int j = (int)__builtin_ctzll(mm);
        const uint32_t ew = (uint32_t)__builtin_amdgcn_readlane((int)pw, j);
        const uint32_t es = (uint32_t)__builtin_amdgcn_readlane((int)ps, j);
        const uint32_t ep = (uint32_t)__builtin_amdgcn_readlane((int)per, j);
        const uint32_t o_ = ew & 0xFFFFu, n_ = (ew >> 16) + 1;
        const bool in_ = (es >> 31) != 0;
        const uint32_t sa_ = es & 0x7FFFFFFFu;
        if (n_ > 64) {  // a long literal (a copy is at most 64 bytes) runs alone
          if (k == 0) {
            long_lit = true;
            eo[0] = o_;
            eln[0] = n_;
            esa[0] = sa_;
          }
          continue;
        }
        if (k > 0 && !in_ && (ep ? o_ : sa_ + n_) > bo) continue;  // reads this batch's output: the next batch
        if (k == 0) bo = o_;
        mm &= mm - 1;
        eo[k] = o_;
        eln[k] = n_;
        esa[k] = sa_;
        eper[k] = ep;
        ein[k] = in_;
        cnt = k + 1;
      }
      if (long_lit) {
        m &= m - 1;
        for (uint32_t q2 = lane; q2 < eln[0]; q2 += 64) o[eo[0] + q2] = in[esa[0] + q2];
        continue;
      }
      m = mm;
      uint32_t v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t idx = lane < eln[k] ? esa[k] + small_mod(lane, eper[k] ? eper[k] : 64u) : esa[k];
        v[k] = ein[k] ? in[idx] : o[idx];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (lane < eln[k]) o[eo[k] + lane] = (uint8_t)v[k];
    }
    __builtin_amdgcn_wave_barrier();
    w0 += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    base += cur;
  }
  return w0 == ulen;
}

// One Snappy chunk's elements qp[0, qe - qp) decoded lane-serially into out[o, lim) (global memory; chunks too large
// for the LDS staging); o advances. False when malformed or the output does not end exactly at lim.
__device__ bool sn_serial_decode(const uint8_t* qp, const uint8_t* qe, uint8_t* __restrict__ out, uint64_t& o,
                                 uint64_t lim) {
  const uint64_t start = o;
  bool ok = true;
  while (ok && qp < qe) {
    const uint32_t tag = *qp++;
    uint32_t ln, off;
    if ((tag & 3) == 0) {
      ln = tag >> 2;
      if (ln >= 60) {
        const uint32_t nb = ln - 59;
        if ((uint64_t)(qe - qp) < 4) { ok = false; break; }  // snap: 4 bytes after the tag whatever nb is
        ln = 0;
        for (uint32_t k = 0; k < nb; ++k) ln |= (uint32_t)qp[k] << (8 * k);
        qp += nb;
      }
      ln += 1;
      if ((uint64_t)(qe - qp) < ln || o + ln > lim) { ok = false; break; }
      for (uint32_t k = 0; k < ln; ++k) out[o + k] = qp[k];
      o += ln;
      qp += ln;
      continue;
    }
    if ((tag & 3) == 1) {
      if (qp >= qe) { ok = false; break; }
      ln = 4 + ((tag >> 2) & 7);
      off = ((tag >> 5) << 8) | *qp++;
    } else if ((tag & 3) == 2) {
      if (qe - qp < 2) { ok = false; break; }
      ln = 1 + (tag >> 2);
      off = qp[0] | ((uint32_t)qp[1] << 8);
      qp += 2;
    } else {
      if (qe - qp < 4) { ok = false; break; }
      ln = 1 + (tag >> 2);
      off = qp[0] | ((uint32_t)qp[1] << 8) | ((uint32_t)qp[2] << 16) | ((uint32_t)qp[3] << 24);
      qp += 4;
    }
    if (off == 0 || off > o - start || o + ln > lim) { ok = false; break; }
    for (uint32_t k = 0; k < ln; ++k, ++o) out[o] = out[o - off];
  }
  return ok && o == lim;
}

// One wave per frame (lcrc_snappy_frames), grid-stride; each chunk's descriptor for the CRC pass over the decoded
// bytes (the whole-table scan decodes and checks its frames in k_ts_decode instead).
__global__ void __launch_bounds__(64) k_snappy_decode_wave(const uint8_t* __restrict__ base,
                                                           const lcrc_desc_dev* __restrict__ frames, uint64_t n,
                                                           const uint64_t* __restrict__ out_off,
                                                           const uint64_t* __restrict__ chunk_off,
                                                           uint8_t* __restrict__ out, uint8_t* __restrict__ status,
                                                           lcrc_desc_dev* __restrict__ cdesc,
                                                           uint32_t* __restrict__ cexp, uint32_t* __restrict__ cframe,
                                                           uint32_t in_lim, uint32_t out_cap) {
  extern __shared__ __attribute__((aligned(16))) uint8_t sn_lds[];
  const uint32_t lane = __lane_id();
  uint8_t* const lin = sn_lds;
  uint8_t* const lout = sn_lds + in_lim + SN_SLACK;
  for (uint64_t f = blockIdx.x; f < n; f += gridDim.x) {
    if (status[f]) continue;
    const uint8_t* p = base + frames[f].offset;
    const uint32_t len = frames[f].length;
    uint64_t o = out_off[f];
    uint64_t c = chunk_off[f];
    const uint64_t c_end = chunk_off[f + 1];
    sn_reader rd;
    rd.init(p, len, lane);
    const uint32_t end = rd.lim;
    bool ok = true;
    uint32_t at = (uint32_t)(p - rd.a);
    // the framing was validated by pass 1: chunk headers and lengths are in bounds, preambles are sane
    while (ok && at < end) {
      rd.ensure(at, lane);
      const uint32_t type = rd.byte(at);
      const uint32_t cl = rd.le(at + 1, 3);
      const uint32_t body = at + 4;
      at = body + cl;
      if (type > 1) continue;  // stream identifiers and skippable chunks
      rd.ensure(body, lane);
      const uint32_t want = rd.le(body, 4);
      const uint64_t start = o;
      if (type == 1) {
        const uint8_t* src = rd.a + body + 4;
        for (uint32_t k = lane; k < cl - 4; k += 64) out[o + k] = src[k];
        o += cl - 4;
      } else {
        uint32_t ulen = 0, q = body + 4, used = 0;  // preamble = uncompressed length (valid: pass 1)
        snappy_preamble([&](uint32_t i) { return rd.byte(q + i); }, at - q, ulen, used);
        q += used;
        if (ulen <= out_cap && at - q + 4 <= in_lim) {
          // stage the elements: aligned dwords from the one holding the first byte
          const uint8_t* zs = rd.a + q;
          const uint32_t d = (uint32_t)((uintptr_t)zs & 3);
          const uint32_t* za = (const uint32_t*)(zs - d);
          const uint32_t ndw = (d + (at - q) + 3) >> 2;
          stage_to_lds(za, (lds_u8*)lin, ndw, lane, 64);
          __builtin_amdgcn_s_waitcnt(0);
          __builtin_amdgcn_wave_barrier();
          ok = snappy_wave_decode(lin, d, d + (at - q), lout, ulen, lane);
          __builtin_amdgcn_wave_barrier();
          if (ok) {
            if ((o & 15) == 0) {
              uint32_t k = 16 * lane;
              for (; k + 16 <= ulen; k += 1024)
                *(uint4*)(out + o + k) = *(const uint4*)(lout + k);
              for (; k < ulen; ++k) out[o + k] = lout[k];  // the lane holding the tail (< 16 B)
            } else {
              for (uint32_t k = lane; k < ulen; k += 64) out[o + k] = lout[k];
            }
            o += ulen;
          }
        } else if (lane == 0) {  // too large for the staging: lane-serial, from and to global memory
          ok = sn_serial_decode(rd.a + q, rd.a + at, out, o, start + ulen);
        }
        ok = bcast(ok ? 1u : 0u) != 0;
        o = ((uint64_t)bcast((uint32_t)(o >> 32)) << 32) | bcast((uint32_t)o);
      }
      if (!ok) break;
      if (lane == 0) {
        lcrc_desc_dev d;
        d.offset = start;
        d.length = (uint32_t)(o - start);
        d.expect_rel = LCRC_NO_EXPECT_DEV;
        cdesc[c] = d;
        cexp[c] = want;
        cframe[c] = (uint32_t)f;
      }
      ++c;
    }
    if (!ok && lane == 0) {
      status[f] = 1;
      // the chunk slots this frame did not fill: empty ranges that match by construction
      for (const uint64_t ce = c_end; c < ce; ++c) {
        lcrc_desc_dev d;
        d.offset = 0;
        d.length = 0;
        d.expect_rel = LCRC_NO_EXPECT_DEV;
        cdesc[c] = d;
        cexp[c] = 0;
        cframe[c] = (uint32_t)f;
      }
    }
  }
}

// a chunk whose masked CRC-32C differs from the stored one marks its frame corrupt (frames already
// marked corrupt by the decode are skipped: their empty placeholder chunks carry no CRC)
__global__ void __launch_bounds__(256) k_snappy_check(const uint32_t* __restrict__ crc,
                                                      const uint32_t* __restrict__ cexp,
                                                      const uint32_t* __restrict__ cframe,
                                                      const uint64_t* __restrict__ nch, uint8_t* __restrict__ status) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= *nch) return;
  const uint32_t f = cframe[c];
  if (status[f] == 1) return;
  if (crc[c] != cexp[c]) status[f] = 2;  // 2: CRC mismatch (reported like 1)
}

// ---------------------------------------------------------------------------------------------------
// SSTable index block on the device (lcrc_table_scan): one thread per restart segment walks its entries
// (src/sstable/block.rs: entry = varint32 shared, non_shared, value_len, key delta, value; the value is a
// BlockHandle = varint64 offset, size, src/sstable/format.rs:24-61). Anything the segmented walk cannot
// vouch for -- a restart entry with shared != 0, an entry crossing the next restart, a malformed varint
// or handle -- sets the segment's fallback flag and the host repeats the walk sequentially (for the
// reference's exact error message).
// ---------------------------------------------------------------------------------------------------
// varint32 (BITS 32: shifts 0..28) / varint64 (BITS 64: shifts 0..63), as the host's get_varint32/64.
// Returns the position after it, or ~0u when it is malformed or runs past lim.
template <int BITS>
__device__ __forceinline__ uint32_t dev_varint(const uint8_t* __restrict__ d, uint32_t p, uint32_t lim,
                                               uint64_t* __restrict__ out) {
  uint64_t result = 0;
  for (int shift = 0; shift <= (BITS == 32 ? 28 : 63); shift += 7) {
    if (p >= lim) return ~0u;
    const uint64_t b = d[p];
    p += 1;
    result |= (b & 127) << shift;
    if (!(b & 128)) {
      *out = BITS == 32 ? (uint64_t)(uint32_t)result : result;  // the host decoder keeps 32 bits
      return p;
    }
  }
  return ~0u;
}

// PASS 1: count[i] = entries of segment i, flag[i] = 1 if the host must walk. PASS 2: writes the handles
// (tblk offset/size, kind DATA) at pos[i] .. and their verify descriptors; a handle past the end of the file
// gets an empty descriptor and status TRUNCATED.
template <bool PASS2>
__device__ __forceinline__ uint64_t idx_segment(const uint8_t* __restrict__ d, uint32_t len, uint32_t nres,
                                                uint64_t file_len, uint64_t o0, lcrc_tblk_dev* __restrict__ out,
                                                lcrc_desc_dev* __restrict__ descs, uint64_t i, bool& bad,
                                                uint64_t ocap = ~0ull);

template <bool PASS2>
__global__ void __launch_bounds__(256) k_idx_parse(const uint8_t* __restrict__ d, uint32_t len, uint32_t nres,
                                                   uint64_t file_len, uint64_t* __restrict__ count,
                                                   uint64_t* __restrict__ flag, const uint64_t* __restrict__ pos,
                                                   lcrc_tblk_dev* __restrict__ out, lcrc_desc_dev* __restrict__ descs) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nres) return;
  bool bad;
  const uint64_t n = idx_segment<PASS2>(d, len, nres, file_len, PASS2 ? pos[i] : 0, out, descs, i, bad);
  if (!PASS2) {
    count[i] = bad ? 0 : n;
    flag[i] = bad ? 1 : 0;
  }
}

// PASS 1: returns the entries of segment i (bad: the host must walk it). PASS 2: writes them from slot o0 on (the
// slots below ocap).
template <bool PASS2>
__device__ __forceinline__ uint64_t idx_segment(const uint8_t* __restrict__ d, uint32_t len, uint32_t nres,
                                                uint64_t file_len, uint64_t o0, lcrc_tblk_dev* __restrict__ out,
                                                lcrc_desc_dev* __restrict__ descs, uint64_t i, bool& bad,
                                                uint64_t ocap) {
  const uint32_t restarts = len - (1 + nres) * 4;
  auto rst = [&](uint32_t k) { return load_le32(d + restarts + 4 * k); };
  const uint32_t start = rst((uint32_t)i);
  const uint32_t end = i + 1 < nres ? rst((uint32_t)i + 1) : restarts;
  bad = (i == 0 && start != 0) || start > end || end > restarts;
  uint64_t n = 0;
  uint32_t off = start;
  for (uint32_t guard = 0; !bad && off < end; ++guard) {
    if (guard > len || restarts - off < 3) {  // an entry takes >= 3 bytes: at most len of them
      bad = true;
      break;
    }
    uint64_t shared = 0, non_shared = 0, vlen = 0;
    uint32_t p = dev_varint<32>(d, off, restarts, &shared);
    if (p != ~0u) p = dev_varint<32>(d, p, restarts, &non_shared);
    if (p != ~0u) p = dev_varint<32>(d, p, restarts, &vlen);
    if (p == ~0u || (uint64_t)restarts - p < non_shared + vlen || (off == start && shared != 0) ||
        p + non_shared + vlen > end) {
      bad = true;
      break;
    }
    const uint32_t qe = (uint32_t)(p + non_shared + vlen);
    uint64_t hoff = 0, hsize = 0;
    uint32_t q = dev_varint<64>(d, (uint32_t)(p + non_shared), qe, &hoff);
    if (q != ~0u) q = dev_varint<64>(d, q, qe, &hsize);
    if (q == ~0u) {
      bad = true;
      break;
    }
    if (PASS2) {
      const uint64_t o = o0 + n;
      lcrc_tblk_dev b;
      b.offset = hoff;
      b.size = hsize;
      b.crc = 0;
      b.kind = 0;
      b.type = 0;
      b.status = 0;
      b.reserved = 0;
      lcrc_desc_dev dd;
      const bool in = hoff <= file_len && hsize + 5 <= file_len - hoff && hsize + 1 <= 0x7FFFFFFFull;
      dd.offset = in ? hoff : 0;
      dd.length = in ? (uint32_t)(hsize + 1) : 0;
      dd.expect_rel = in ? (int32_t)(hsize + 1) : LCRC_NO_EXPECT_DEV;
      if (!in) {
        b.status = 2;  // LCRC_TBLK_TRUNCATED
        b.type = 0xFF;
      }
      if (o < ocap) {  // (k_ts_windows: slots past the result capacity are never written)
        out[o] = b;
        descs[o] = dd;
      }
    }
    ++n;
    off = (uint32_t)(p + non_shared + vlen);
  }
  return n;
}

// per block: computed crc, stored type, status (mismatch / bad type), and the Snappy frame to check when
// the checksum holds and the type is 1 (length 0 otherwise)
__global__ void __launch_bounds__(256) k_tbl_finish(lcrc_tblk_dev* blk, uint64_t n,
                                                    const uint32_t* __restrict__ crc,
                                                    const uint32_t* __restrict__ mismatch,
                                                    const uint8_t* __restrict__ file,
                                                    lcrc_desc_dev* __restrict__ frames,
                                                    const uint64_t* __restrict__ n_dev) {
  if (n_dev) n = *n_dev < n ? *n_dev : n;
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  lcrc_tblk_dev b = blk[i];
  lcrc_desc_dev f;
  f.offset = 0;
  f.length = 0;
  f.expect_rel = LCRC_NO_EXPECT_DEV;
  if (b.status != 2) {
    b.crc = crc[i];
    b.type = file[b.offset + b.size];
    b.status = (mismatch[i >> 5] >> (i & 31)) & 1;
    if (b.status == 0 && b.type > 1) b.status = 4;  // LCRC_TBLK_BAD_TYPE
    if (b.status == 0 && b.type == 1) {
      f.offset = b.offset;
      f.length = (uint32_t)b.size;
    }
  }
  blk[i] = b;
  frames[i] = f;
}

// the Snappy frames' verdicts into the blocks' status; *unsorted = gen when a block starts before its
// predecessor (the host then sorts the result: a well-formed table never needs it). Only the status byte
// is written here, so the offsets every thread compares are read-only in this kernel.
__global__ void __launch_bounds__(256) k_tbl_content(lcrc_tblk_dev* __restrict__ blk, uint64_t n,
                                                     const uint8_t* __restrict__ fstatus,
                                                     uint32_t* __restrict__ unsorted, uint32_t gen,
                                                     const uint64_t* __restrict__ n_dev) {
  if (n_dev) n = *n_dev < n ? *n_dev : n;
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (unsorted && i > 0 && blk[i - 1].offset > blk[i].offset) *unsorted = gen;
  if (fstatus[i]) blk[i].status = 3;  // LCRC_TBLK_BAD_CONTENT
}

// ---------------------------------------------------------------------------------------------------
// Asynchronous whole-table scan (lcrc_table_scan_async): Table::open + read_meta + one verify of every block
// (table.rs:39-146, format.rs:146-213) with no host round trip. The index and metaindex are walked
// OPTIMISTICALLY, before their own checksums are known: both are verified in the same batch as the data
// blocks, and k_ts_close applies the reference's order afterwards (index checksum before any index-contents
// error; the filter block named by a metaindex that does not verify is dropped, as read_meta swallows it).
// Whatever the device walk cannot vouch for sets status 2 and the synchronous wrapper walks on the host.
// ---------------------------------------------------------------------------------------------------
enum { TS_OK = 0, TS_CORRUPT = 1, TS_HOST = 2, TS_CAPACITY = 3 };
enum { TSM_SHORT = 1, TSM_MAGIC = 2, TSM_VARINT = 3, TSM_CHECKSUM = 4, TSM_TYPE = 5, TSM_SMALL = 6, TSM_CONTENTS = 7 };

// footer, index block header and (meta) the metaindex filter entry, by one thread; key: 256 B of LDS
// idec / iopen: k_ts_open2's decoded index and its verdict (nullptr when the scan has no LCRC_TSCAN_SNAPPY_INDEX)
// pre (k_ts_windows, nullable): every value this walk loads, loaded beforehand by the workgroup in parallel rounds
// (a chain of dependent loads costs ~5 us a link under the window stream), each under the condition its use here has
struct TsPre {
  const uint8_t* foot;       // the file's last 48 bytes (LDS)
  const uint8_t* meta_copy;  // the metaindex block with its type byte (LDS), or nullptr: read from the file
  uint64_t io[3];            // iopen[0..2] (when iopen is given)
  uint32_t itype, nres_raw, nres_dec;  // the index block's type byte; the restart count of its raw / decoded contents
};
__device__ __forceinline__ void ts_open_state(const uint8_t* __restrict__ file, uint64_t file_len, const lcrc_tscan_key& fkey,
                              uint64_t seg_cap, uint8_t* __restrict__ key, bool meta, const uint8_t* __restrict__ idec,
                              const uint64_t* __restrict__ iopen, lcrc_tscan_dev& s, const TsPre* pre = nullptr) {
  s = {};
  if (file_len < 48) {
    s.status = TS_CORRUPT;
    s.code = TSM_SHORT;
    return;
  }
  const uint8_t* f = pre ? pre->foot : file + file_len - 48;
  const uint64_t magic = (uint64_t)load_le32(f + 40) | ((uint64_t)load_le32(f + 44) << 32);
  if (magic != 0xdb4775248b80fb57ull) {
    s.status = TS_CORRUPT;
    s.code = TSM_MAGIC;
    return;
  }
  uint32_t p = dev_varint<64>(f, 0, 48, &s.meta_off);
  if (p != ~0u) p = dev_varint<64>(f, p, 48, &s.meta_size);
  if (p != ~0u) p = dev_varint<64>(f, p, 48, &s.idx_off);
  if (p != ~0u) p = dev_varint<64>(f, p, 48, &s.idx_size);
  if (p == ~0u) {
    s.status = TS_CORRUPT;
    s.code = TSM_VARINT;
    return;
  }
  // Table::open reads the index block (verified: paranoid_checks); its checksum comes with the batch
  if (s.idx_off > file_len || s.idx_size + 5 > file_len - s.idx_off || s.idx_size + 1 > 0x7FFFFFFFull) {
    s.status = TS_HOST;  // "truncated block read" and its kin: the host walk
    return;
  }
  const uint8_t itype = pre ? (uint8_t)pre->itype : file[s.idx_off + s.idx_size];
  const uint8_t* ic = file + s.idx_off;  // the index block's contents
  uint64_t clen = s.idx_size;
  if (itype == 1) {
    // a Snappy-framed index block: its contents are what k_ts_open2 decoded, when it decoded them all; otherwise the
    // host path decodes it (and gives the reference's message) -- after the workspace grows, when that was the reason
    const uint64_t o0 = iopen ? (pre ? pre->io[0] : iopen[0]) : 0;
    const uint64_t o1 = o0 ? (pre ? pre->io[1] : iopen[1]) : 0, o2 = o0 ? (pre ? pre->io[2] : iopen[2]) : 0;
    if (!(o0 & 2) || o2 || o1 > 0x7FFFFFFFull) {
      if (o0 & 4) {
        s.gate = 1;
        s.need_out = o1;
      }
      s.status = TS_HOST;
      return;
    }
    s.idx_dec = 1;
    ic = idec;
    clen = o1;
  }
  s.idx_clen = clen;
  if (itype > 1) {
    s.pcode = TSM_TYPE;
  } else if (clen < 4) {
    s.pcode = TSM_SMALL;
  } else {
    const uint32_t nres = pre ? (s.idx_dec ? pre->nres_dec : pre->nres_raw) : load_le32(ic + clen - 4);
    if ((uint64_t)nres > (clen - 4) / 4) {
      s.pcode = TSM_CONTENTS;
    } else if (nres == 0 || (clen - 4) / nres > 4096) {
      s.status = TS_HOST;  // no restart points / long segments: the sequential host walk
      return;
    } else if (nres + 2 > seg_cap) {
      s.status = TS_CAPACITY;  // at least one block per segment: more than the result can hold
      s.n_data = nres + 2;
      return;
    } else {
      s.nres = nres;
    }
  }
  // read_meta (only with a filter policy): the first metaindex key >= "filter" + name; a malformed
  // metaindex yields no filter, as the reference swallows read_meta's errors
  if (meta && fkey.len && s.meta_off <= file_len && s.meta_size + 5 <= file_len - s.meta_off && s.meta_size <= 0xFFFFFFFFull) {
    const uint8_t* d = pre && pre->meta_copy ? pre->meta_copy : file + s.meta_off;
    const uint64_t n = s.meta_size;
    const uint8_t mtype = d[n];
    if (mtype == 1) {
      s.status = TS_HOST;  // compressed metaindex: the host path decodes it
      return;
    }
    if (mtype == 0 && n >= 4) {
      const uint32_t nr = load_le32(d + n - 4);
      if ((uint64_t)nr <= (n - 4) / 4) {
        const uint32_t restarts = (uint32_t)(n - (1 + (uint64_t)nr) * 4);
        uint32_t off = 0, klen = 0;
        while (off < restarts) {
          if (restarts - off < 3) break;
          uint64_t shared, non_shared, vlen;
          uint32_t q = dev_varint<32>(d, off, restarts, &shared);
          if (q != ~0u) q = dev_varint<32>(d, q, restarts, &non_shared);
          if (q != ~0u) q = dev_varint<32>(d, q, restarts, &vlen);
          if (q == ~0u || (uint64_t)restarts - q < non_shared + vlen || klen < shared) break;
          if (shared + non_shared > 256) {  // the LDS key buffer
            s.status = TS_HOST;  // a key longer than the walk's buffer
            return;
          }
          for (uint32_t i = 0; i < non_shared; ++i) key[shared + i] = d[q + i];
          klen = (uint32_t)(shared + non_shared);
          int c = 0;  // compare key with the wanted key (bytewise, then length)
          const uint32_t m = klen < fkey.len ? klen : fkey.len;
          for (uint32_t i = 0; i < m && !c; ++i) c = (int)key[i] - (int)fkey.key[i];
          if (!c) c = klen < fkey.len ? -1 : klen > fkey.len ? 1 : 0;
          if (c >= 0) {
            if (c == 0) {
              const uint32_t ve = (uint32_t)(q + non_shared + vlen);
              uint64_t fo, fs;
              uint32_t r = dev_varint<64>(d, (uint32_t)(q + non_shared), ve, &fo);
              if (r != ~0u) r = dev_varint<64>(d, r, ve, &fs);
              if (r != ~0u) {
                s.has_filter = 1;
                s.filt_off = fo;
                s.filt_size = fs;
              }
            }
            break;
          }
          off = (uint32_t)(q + non_shared + vlen);
        }
      }
    }
  }
}

// Workgroup-wide exclusive scan of two u64 values per thread (NWAVE waves): e* = the sums over the threads
// before this one, t* = the workgroup's totals. s*: NWAVE words of LDS each.
template <int NWAVE = 4>
__device__ __forceinline__ void wg_scan2(uint64_t va, uint64_t vb, uint64_t* sa, uint64_t* sb, uint64_t& ea,
                                         uint64_t& eb, uint64_t& ta, uint64_t& tb) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned long long ia = va, ib = vb;
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long xa = __shfl_up(ia, d, 64), xb = __shfl_up(ib, d, 64);
    if (lane >= (uint32_t)d) {
      ia += xa;
      ib += xb;
    }
  }
  if (lane == 63) {
    sa[w] = ia;
    sb[w] = ib;
  }
  __syncthreads();
  uint64_t pa = 0, pb = 0;
  ta = tb = 0;
  for (uint32_t k = 0; k < NWAVE; ++k) {
    if (k < w) {
      pa += sa[k];
      pb += sb[k];
    }
    ta += sa[k];
    tb += sb[k];
  }
  __syncthreads();  // the caller may reuse sa / sb
  ea = pa + ia - va;
  eb = pb + ib - vb;
}

// After pass 1, from the totals (nd: the data blocks the index names, nflag: segments the device walk cannot vouch
// for): the capacity check and the fallback flags (decided alike by every workgroup; `lead` records them), then
// pass 2 writes the handles (seg(d, len, nres): this workgroup's segments at their slots) and, in workgroup 0
// (wg0), threads 0..2 append the filter, metaindex and index blocks with their descriptors. s: the state
// ts_open_state left (the last index ticket's own).
template <class Seg>
__device__ void ts_emit_body(const lcrc_tscan_dev& s, lcrc_tscan_dev* __restrict__ st, bool lead, bool wg0,
                             uint64_t nd, uint64_t nflag, const uint8_t* __restrict__ file, uint64_t file_len,
                             lcrc_tblk_dev* __restrict__ out, lcrc_desc_dev* __restrict__ descs, uint64_t cap,
                             uint64_t vcap, const uint8_t* __restrict__ idec, Seg seg) {
  if (s.status != TS_OK) {
    if (lead) st->n_total = 0;
    return;
  }
  const uint64_t nres = s.nres;
  const bool hf = s.has_filter;
  const uint64_t ntot = nd + (hf ? 3 : 2);
  if (nres && nflag) {
    // a segment the device walk cannot vouch for. The reference checks the index block's checksum before its
    // contents: verify it alone, and let the host walk give the contents' message only if it holds
    if (lead) {
      st->n_total = cap ? 1 : 0;
      st->n_verify = st->n_total;
      if (!cap) {
        st->status = TS_HOST;
        return;
      }
      st->idx_only = 1;
      lcrc_tblk_dev b = {};
      b.offset = s.idx_off;
      b.size = s.idx_size;
      b.kind = 3;  // LCRC_TBLK_INDEX
      lcrc_desc_dev dd;
      dd.offset = s.idx_off;
      dd.length = (uint32_t)(s.idx_size + 1);  // in the file: checked by ts_open_state
      dd.expect_rel = (int32_t)(s.idx_size + 1);
      out[0] = b;
      descs[0] = dd;
    }
    return;
  }
  if (ntot > cap) {
    if (lead) {
      st->status = TS_CAPACITY;
      st->n_data = ntot;  // the capacity needed (reported); n_total stays 0: nothing is verified
      st->n_total = 0;
    }
    return;
  }
  // the filter, metaindex and index blocks (k = 0, 1, 2): in the file, and split into pieces when long
  uint64_t offk[3], sizek[3], npk[3];
  bool ink[3];
  uint64_t npieces = 0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    offk[k] = k == 0 ? s.filt_off : k == 1 ? s.meta_off : s.idx_off;
    sizek[k] = k == 0 ? s.filt_size : k == 1 ? s.meta_size : s.idx_size;
    ink[k] = (k > 0 || hf) && offk[k] <= file_len && sizek[k] + 5 <= file_len - offk[k] && sizek[k] + 1 <= 0x7FFFFFFFull;
    npk[k] = ink[k] && sizek[k] + 1 > LCRC_TS_PIECE ? (sizek[k] + LCRC_TS_PIECE) / LCRC_TS_PIECE : 0;
    npieces += npk[k];
  }
  const bool split = ntot + npieces <= vcap;
  if (lead) {
    st->n_data = nd;
    st->n_total = ntot;
    st->n_verify = ntot + (split ? npieces : 0);
  }
  seg(s.idx_dec ? idec : file + s.idx_off, (uint32_t)s.idx_clen, nres);
  if (wg0 && threadIdx.x < 3) {
    const uint32_t k = threadIdx.x;  // 0 filter (if any), then metaindex, index
    if (k == 0 && !hf) return;
    const uint64_t at = nd + (hf ? k : k - 1);
    // (selects, not a runtime index into the arrays: those would live in scratch)
    const uint64_t off = k == 0 ? offk[0] : k == 1 ? offk[1] : offk[2];
    const uint64_t size = k == 0 ? sizek[0] : k == 1 ? sizek[1] : sizek[2];
    const uint64_t np = k == 0 ? npk[0] : k == 1 ? npk[1] : npk[2];
    const bool in = k == 0 ? ink[0] : k == 1 ? ink[1] : ink[2];
    if (split && np) {
      // the first piece takes the remainder, so that every later piece is joined by the same Z65536
      const uint64_t first = ntot + (k > 0 ? npk[0] : 0) + (k > 1 ? npk[1] : 0);
      const uint64_t r = size + 1 - (np - 1) * LCRC_TS_PIECE;
      st->pbase[k] = (uint32_t)first;
      st->pcnt[k] = (uint32_t)np;
      for (uint64_t q = 0; q < np; ++q) {
        lcrc_desc_dev pd;
        pd.offset = q ? off + r + (q - 1) * LCRC_TS_PIECE : off;
        pd.length = (uint32_t)(q ? LCRC_TS_PIECE : r);
        pd.expect_rel = LCRC_NO_EXPECT_DEV;
        descs[first + q] = pd;
      }
    }
    lcrc_tblk_dev b;
    b.offset = off;
    b.size = size;
    b.crc = 0;
    b.kind = (uint8_t)(k + 1);  // LCRC_TBLK_FILTER, _METAINDEX, _INDEX
    b.type = 0;
    b.status = 0;
    b.reserved = 0;
    lcrc_desc_dev dd;
    const bool whole = in && !(split && np);  // a split block's own descriptor is empty
    dd.offset = in ? off : 0;
    dd.length = whole ? (uint32_t)(size + 1) : 0;
    dd.expect_rel = whole ? (int32_t)(size + 1) : LCRC_NO_EXPECT_DEV;
    if (!in) {
      b.status = 2;  // LCRC_TBLK_TRUNCATED
      b.type = 0xFF;
    }
    out[at] = b;
    descs[at] = dd;
  }
}

// The table scan's first launch (lcrc_table_scan_async_ex): the file's window pass (k_windows<false>: its values do
// not depend on the index) in workgroups [0, nwg), and Table::open's index walk with the handles in the nidx
// workgroups after them, which run beside the window stream instead of before it (nwg = 0: the index walk alone).
// Progress without co-residency (several scans may share the chip, one per stream): an index workgroup first takes a
// TICKET j from agg[TSA_TICKET_AT] and walks the j-th contiguous range of the restart segments; the ranges' entry
// counts meet through agg[j] (a ready bit, a fallback bit, the count), which ticket j publishes before it waits on
// anything. Ticket j then waits only on the words of tickets below j (decoupled look-back, without the shortcut:
// at most 256 words, one polling thread each). A lower ticket was taken by a workgroup that has started, so it is
// resident or done, and it publishes without waiting: every wait ends whatever else occupies the CUs. Each ticket
// writes its handles at its offset (slots bounded by the capacity, since only the last ticket knows the total) and
// then sets the done bit of its word; the last ticket (nidx - 1) waits for every done bit -- its lower tickets
// again --, then alone writes the state, the filter / metaindex / index entries after the data blocks, and when a range is
// bad the index block's entry at slot 0 (the one slot another range may have written: that range releases its
// stores before counting itself, the last ticket acquires), and zeroes the words for the next scan. Each index
// workgroup computes the footer state itself (the metaindex walk included), so that none reads another's. The
// totals travel inside the atomic words themselves, so the polls are relaxed: an acquire/release at agent scope
// writes back / invalidates the XCD's L2, under the window stream, and is paid once, by the two workgroups above.
constexpr uint64_t TSA_READY = 1ull << 63, TSA_BAD = 1ull << 62, TSA_DONE = 1ull << 61, TSA_COUNT = TSA_DONE - 1;
constexpr uint32_t TSA_MAX = 256, TSA_TICKET_AT = TSA_MAX;  // agg: 257 words
static_assert(A_THREADS >= TSA_MAX, "a thread per lower ticket's word");
struct TsIdxArgs {
  const uint8_t* file;
  uint64_t file_len;
  uint64_t seg_cap, cap, vcap, nzero;
  lcrc_tscan_dev* st;
  uint64_t* local_c;
  uint32_t* zero;  // the batch's mismatch bitmap (nzero words)
  const uint8_t* idec;
  const uint64_t* iopen_r;  // k_ts_open2's verdict (nullptr: no Snappy-framed index)
  uint64_t* iopen;          // its failure mark is cleared once every workgroup has read it
  lcrc_tblk_dev* out;
  lcrc_desc_dev* descs;
  uint64_t* agg;  // nidx words, then the arrival count
};

// bytes [src1, src1 + n1) and [src2, src2 + n2) of global memory into dst1[0, n1) and dst2[0, n2) (LDS), by the
// whole workgroup: aligned dword loads (the dwords holding a range's first and last bytes stay inside its
// allocation), up to 8 a thread issued before any of its stores, so that up to 16 KiB of both is one load round trip
__device__ __forceinline__ void wg_copy_bytes(uint8_t* dst1, const uint8_t* __restrict__ src1, uint32_t n1,
                                              uint8_t* dst2 = nullptr, const uint8_t* __restrict__ src2 = nullptr,
                                              uint32_t n2 = 0) {
  const uint32_t mis1 = (uint32_t)((uintptr_t)src1 & 3), mis2 = (uint32_t)((uintptr_t)src2 & 3);
  const uint32_t* __restrict__ w1 = (const uint32_t*)(src1 - mis1);
  const uint32_t* __restrict__ w2 = (const uint32_t*)(src2 - mis2);
  const uint32_t nd1 = n1 ? (mis1 + n1 + 3) / 4 : 0, nd2 = n2 ? (mis2 + n2 + 3) / 4 : 0, nd = nd1 + nd2;
  for (uint32_t base = 0; base < nd; base += 8 * A_THREADS) {
    uint32_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t k = base + u * A_THREADS + threadIdx.x;
      v[u] = k < nd1 ? w1[k] : k < nd ? w2[k - nd1] : 0u;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t k = base + u * A_THREADS + threadIdx.x;
      const bool first = k < nd1;
      const uint32_t kk = first ? k : k - nd1, mis = first ? mis1 : mis2, n = first ? n1 : n2;
      uint8_t* dst = first ? dst1 : dst2;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t o = 4 * kk + q - mis;  // (wraps below 0: out of range)
        if (k < nd && o < n) dst[o] = (uint8_t)(v[u] >> (8 * q));
      }
    }
  }
}

#ifdef LCRC_PROBE_CLOCK  // diagnostic build: index workgroup j's phase stamps in lcrc_dbg_stamp row 2048 + j
#define TSI_STAMP(k)                                                                       \
  if (threadIdx.x == 0 && j < 2048) lcrc_dbg_stamp[(2048 + j) * 8 + (k)] = __builtin_amdgcn_s_memrealtime()
#else
#define TSI_STAMP(k)
#endif
// Index workgroup j of k_ts_windows. Under the window stream a load takes ~5 us, so every value the walk needs is
// loaded in four parallel rounds instead of chains: (1) the footer and k_ts_open2's verdict words; (2) the metaindex
// block, the index block's type byte and its restart count (raw and decoded: the type picks); (3) the workgroup's
// slice of the restart array; (4) the bytes of its segments. Its restart segments [lo, hi) are then a block of their
// own in LDS (stage): the bytes [s0, E) -- s0 = the first segment's start (0 in workgroup 0, so that segment 0 must
// start at 0), E = the next range's start or the restart array -- followed by the range's offsets minus s0 and
// their count, so that idx_segment reads it as it reads the whole block, with local segment numbers. Rebasing is
// exact once the offsets are non-decreasing, within the restart array and rst(0) = 0; a violation is a segment the
// whole-block walk finds bad too (start > end, or end past the restarts), so it only raises the fallback bit. A
// range too long for the LDS is walked in place.
__device__ void ts_index_wg(const TsIdxArgs& a, const lcrc_tscan_key& fkey, uint32_t nidx, uint32_t* L,
                            uint32_t* ticket) {
  if (threadIdx.x == 0)
    *ticket = __hip_atomic_fetch_add((uint32_t*)(a.agg + TSA_TICKET_AT), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const uint32_t j = *ticket;  // this workgroup's range (the order in which the index workgroups started)
  if (j >= nidx) return;       // (never: the counter is zero at every launch; no store past the words if it were not)
  TSI_STAMP(0);
#ifndef LCRC_TSI_PRIO
#define LCRC_TSI_PRIO 3
#endif
  if (LCRC_TSI_PRIO) __builtin_amdgcn_s_setprio(LCRC_TSI_PRIO);  // issue ahead of the window waves on the CU: this
                                                                // walk is the launch's critical path
  constexpr int NT = A_THREADS, NWAVE = A_THREADS / 64;
  constexpr uint32_t META_STAGE = 4096, RSL_AT = 6144, RSL_CAP = 16384, STAGE_AT = RSL_AT + RSL_CAP;
  constexpr uint32_t STAGE_CAP = A_LDS_BYTES - STAGE_AT;
  uint8_t* key = (uint8_t*)L;  // 256 B
  lcrc_tscan_dev* S = (lcrc_tscan_dev*)(L + 64);
  static_assert(sizeof(lcrc_tscan_dev) <= 256, "state slot");
  uint64_t* sa = (uint64_t*)(L + 128);
  uint64_t* sb = sa + NWAVE;
  uint64_t* tot = sb + NWAVE;
  uint64_t* io_l = tot + 4;                     // iopen[0..2]
  uint32_t* pre_l = (uint32_t*)(io_l + 3);      // type byte, restart counts
  uint32_t* flags = pre_l + 4;
  uint8_t* foot = (uint8_t*)(L + 256);          // 48 B
  uint8_t* mcopy = (uint8_t*)(L + 272);         // META_STAGE + 1 B
  uint8_t* rsl = (uint8_t*)L + RSL_AT;          // the restart array slice
  uint8_t* stage = (uint8_t*)L + STAGE_AT;
  static_assert(512 + 16 * 8 + 8 * 7 + 4 * 5 <= 1024 && 1088 + META_STAGE + 1 <= RSL_AT && STAGE_CAP >= 32768,
                "index workgroup LDS");
  const uint32_t tid = threadIdx.x;
  const uint64_t file_len = a.file_len;
  for (uint64_t i = (uint64_t)j * NT + tid; i < a.nzero; i += (uint64_t)nidx * NT) a.zero[i] = 0;
  // round 1
  if (tid < 48 && file_len >= 48) foot[tid] = a.file[file_len - 48 + tid];
  if (a.iopen_r && tid >= 64 && tid < 67) io_l[tid - 64] = a.iopen_r[tid - 64];
  if (tid == 0) *flags = 0;
  __syncthreads();
  TSI_STAMP(1);
  // round 2, each load under the condition of its use in ts_open_state
  uint64_t mo = 0, ms = 0, io = 0, is = 0;
  uint32_t p = file_len >= 48 ? dev_varint<64>(foot, 0, 48, &mo) : ~0u;
  if (p != ~0u) p = dev_varint<64>(foot, p, 48, &ms);
  if (p != ~0u) p = dev_varint<64>(foot, p, 48, &io);
  if (p != ~0u) p = dev_varint<64>(foot, p, 48, &is);
  const bool iin = p != ~0u && io <= file_len && is + 5 <= file_len - io && is + 1 <= 0x7FFFFFFFull;
  const bool mstage = p != ~0u && mo <= file_len && ms + 5 <= file_len - mo && ms + 1 <= META_STAGE;
  uint32_t pv = 0;
  if (tid == 0 && iin) pv = a.file[io + is];
  if (tid == 1 && iin && is >= 4) pv = load_le32(a.file + io + is - 4);
  if (tid == 2 && a.iopen_r && (io_l[0] & 2) && !io_l[2] && io_l[1] >= 4 && io_l[1] <= 0x7FFFFFFFull)
    pv = load_le32(a.idec + io_l[1] - 4);
  if (mstage) wg_copy_bytes(mcopy, a.file + mo, (uint32_t)ms + 1);
  if (tid < 3) pre_l[tid] = pv;
  __syncthreads();
  TSI_STAMP(2);
  if (tid == 0) {
    const TsPre pre{foot, mstage ? mcopy : nullptr, {io_l[0], io_l[1], io_l[2]}, pre_l[0], pre_l[1], pre_l[2]};
    lcrc_tscan_dev st0;
    ts_open_state(a.file, file_len, fkey, a.seg_cap, key, true, a.idec, a.iopen_r, st0, &pre);
    *S = st0;
  }
  __syncthreads();
  const lcrc_tscan_dev& s = *S;  // (read in place: a private copy would go to scratch)
  const uint64_t nres = s.nres;  // 0 unless the index block can be walked
  const uint8_t* d = s.idx_dec ? a.idec : a.file + s.idx_off;
  const uint32_t len = (uint32_t)s.idx_clen;
  const uint64_t per = (nres + nidx - 1) / nidx;
  const uint64_t lo = min(nres, (uint64_t)j * per), hi = min(nres, lo + per);
  const uint64_t m = hi - lo;
  const uint32_t restarts = len - (uint32_t)(1 + nres) * 4;
  // round 3: the offsets rst(lo .. min(hi, nres - 1)) (rst(nres) is the restart array's offset) and, speculatively,
  // the bytes around restarts * [lo, hi) / nres (where index entries of even size put the range)
  const bool rstage = nres && 4 * (m + 1) <= RSL_CAP;
  const uint32_t nrs = hi < nres ? (uint32_t)m + 1 : (uint32_t)m;
  uint64_t sp_lo = 0, sp_n = 0;
  if (rstage && m) {
    const uint64_t e0 = (uint64_t)restarts * lo / nres, e1 = (uint64_t)restarts * hi / nres;
    const uint64_t mg = (e1 - e0) / 8 + 64;
    sp_lo = e0 > mg ? e0 - mg : 0;
    sp_n = min((uint64_t)restarts, e1 + mg) - sp_lo;
    if (sp_n + 4 * (m + 1) > STAGE_CAP) sp_n = 0;
  }
  if (rstage) wg_copy_bytes(rsl, d + restarts + 4 * lo, 4 * nrs, stage, d + sp_lo, (uint32_t)sp_n);
  __syncthreads();
  auto rs = [&](uint64_t k) {  // rst(lo + k), k <= m
    return lo + k < nres ? (rstage ? load_le32(rsl + 4 * k) : load_le32(d + restarts + 4 * (lo + k))) : restarts;
  };
  const uint32_t s0 = lo == 0 ? 0u : rs(0), E = rs(m);
  const uint64_t bytes = (uint64_t)E - s0;
  const bool rbad = nres && (s0 > E || E > restarts);
  const bool staged = rstage && !rbad && bytes + 4 * (m + 1) <= STAGE_CAP;
  const bool covered = staged && sp_n && s0 >= sp_lo && E <= sp_lo + sp_n;
  const uint32_t voff = covered ? (uint32_t)(s0 - sp_lo) : 0u;  // the range's first byte in stage
  TSI_STAMP(7);
  // round 4 (unless the speculative bytes cover the range): the segments' bytes, then the rebased offsets after them
  // (idx_segment reads bytes; past E the speculative bytes are not needed)
  if (staged) {
    if (!covered) wg_copy_bytes(stage, d + s0, (uint32_t)bytes);
    uint8_t* sr = stage + voff + bytes;
    auto put = [&](uint64_t k, uint32_t v) {
      sr[4 * k] = (uint8_t)v;
      sr[4 * k + 1] = (uint8_t)(v >> 8);
      sr[4 * k + 2] = (uint8_t)(v >> 16);
      sr[4 * k + 3] = (uint8_t)(v >> 24);
    };
    uint32_t mybad = 0;
    for (uint64_t k = tid; k < m; k += NT) {
      const uint32_t x = rs(k), y = rs(k + 1);
      mybad |= (x > y || y > restarts || (lo + k == 0 && x != 0) || x < s0) ? 1u : 0u;
      put(k, x - s0);
    }
    if (tid == 0) put(m, (uint32_t)m);
    if (mybad) *flags = 1;
  }
  __syncthreads();
  const bool vbad = rbad || (staged && *flags);
  TSI_STAMP(3);
  // pass 1 over the walk's view: the staged range (an LDS pointer, local numbering; the entry offsets within the range
  // kept in the dead restart slice) or the block in place (global numbering, offsets in local_c). Two call sites, so
  // that the staged one reads LDS directly and neither waits on global stores
  uint32_t* loc = (uint32_t*)rsl;
  uint64_t run = 0, nbad = vbad ? 1 : 0;
  auto pass1 = [&](const uint8_t* vd, uint32_t vlen, uint64_t vn, uint64_t v0, bool inl) {
    for (uint64_t t0 = lo; t0 < hi; t0 += NT) {
      const uint64_t i = t0 + tid;
      uint64_t c = 0, f = 0;
      if (i < hi) {
        bool bad;
        const uint64_t n = idx_segment<false>(vd, vlen, (uint32_t)vn, file_len, 0, nullptr, nullptr, i - v0, bad);
        c = bad ? 0 : n;
        f = bad ? 1 : 0;
      }
      uint64_t ec, ef, tc, tf;
      wg_scan2<NWAVE>(c, f, sa, sb, ec, ef, tc, tf);
      if (i < hi) {
        if (inl)
          loc[i - lo] = (uint32_t)(run + ec);
        else
          a.local_c[i] = run + ec;
      }
      run += tc;
      nbad += tf;
    }
  };
  if (staged)
    pass1(stage + voff, (uint32_t)(bytes + 4 * (m + 1)), m, lo, true);
  else
    pass1(d, len, nres, 0, false);
  TSI_STAMP(4);
  // publish this range's count (never waiting on anything first), then look back at the ranges BEFORE it only: one
  // thread per lower ticket polls that ticket's word (one load round trip per poll, all in flight together)
  if (tid == 0)
    __hip_atomic_store(a.agg + j, TSA_READY | (nbad ? TSA_BAD : 0) | run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint64_t v = 0;
  if (tid < j) {
    do {
      v = __hip_atomic_load(a.agg + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } while (!(v & TSA_READY));
  }
  const uint64_t cnt = v & TSA_COUNT;
  uint64_t e1, e2, before, unused;
  wg_scan2<NWAVE>(cnt, 0, sa, sb, e1, e2, before, unused);
  const bool badb = __syncthreads_or((v & TSA_BAD) != 0) != 0;  // a range before this one the walk cannot vouch for
  TSI_STAMP(5);
  // this range's handles at their slots, unless a range up to this one is bad (the scan is then the index block's
  // checksum alone). Whether the whole index fits the result is known to the last ticket only: every slot is bounded
  // by the capacity instead, and the last ticket reports TS_CAPACITY (nothing the caller reads) when it does not fit
  const bool write = s.status == TS_OK && nres && !badb && !nbad;
  if (write) {
    bool bad;
    if (staged) {
      for (uint64_t i = lo + tid; i < hi; i += NT)
        idx_segment<true>(stage + voff, (uint32_t)(bytes + 4 * (m + 1)), (uint32_t)m, file_len, before + loc[i - lo],
                          a.out, a.descs, i - lo, bad, a.cap);
    } else {
      for (uint64_t i = lo + tid; i < hi; i += NT)
        idx_segment<true>(d, len, (uint32_t)nres, file_len, before + a.local_c[i], a.out, a.descs, i, bad, a.cap);
    }
  }
  __syncthreads();
  const bool last = j == nidx - 1;
  if (!last) {
    if (tid == 0) {
      // slot 0 is the one the last ticket may overwrite (the index block alone): a range that wrote it makes its
      // stores visible across the XCDs' L2s before it marks itself done
      if (write && before == 0 && run) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      // done: on its own word, so that the last ticket's reset of that word is ordered after both of its stores
      __hip_atomic_fetch_or(a.agg + j, TSA_DONE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    TSI_STAMP(6);
    return;
  }
  // the last ticket: every other range has published, read what it needed and written its handles once its word
  // says done. It alone writes the state, the tail entries (the filter, metaindex and index blocks after the data
  // blocks) and, when a range is bad, the index block's entry at slot 0; then it resets the words for the next scan
  // (nobody reads them any more)
  if (tid < j)
    while (!(__hip_atomic_load(a.agg + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & TSA_DONE))
      __builtin_amdgcn_s_sleep(2);
  __syncthreads();
  if (tid == 0) {
    if (nres && (badb || nbad)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    *a.st = s;
    a.iopen[2] = 0;  // k_ts_open2's failure mark (every workgroup read it before publishing): clear for the next scan
  }
  __syncthreads();
  ts_emit_body(s, a.st, tid == 0, true, before + run, (badb || nbad) ? 1 : 0, a.file, a.file_len, a.out, a.descs,
               a.cap, a.vcap, a.idec, [&](const uint8_t*, uint32_t, uint64_t) {});
  if (tid < nidx) __hip_atomic_store(a.agg + tid, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // (every ticket was taken before this one's: the count is nidx)
  if (tid == 0) __hip_atomic_store((uint32_t*)(a.agg + TSA_TICKET_AT), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  TSI_STAMP(6);
}

__global__ void __launch_bounds__(A_THREADS) k_ts_windows(const uint8_t* __restrict__ base, uint64_t span,
                                                         uint64_t nreg, const uint32_t* __restrict__ gtab,
                                                         uint32_t* __restrict__ out, uint32_t nwg,
                                                         const lcrc_tscan_key fkey, const TsIdxArgs ia) {
  __shared__ __attribute__((aligned(16))) uint32_t L[A_LDS_BYTES / 4];
  __shared__ uint32_t wg_ticket;
  if (blockIdx.x >= nwg) {
    ts_index_wg(ia, fkey, gridDim.x - nwg, L, &wg_ticket);
    return;
  }
  WinOne src{base, span, nreg, out, 0, nullptr, nullptr};
  windows_body<false, false>(src, gtab, 0, 0, L, &wg_ticket, nwg);
}

// read_block_from_file's type dispatch for every block (k_tbl_finish) and, in the same thread, the framing
// walk of the block's Snappy frame (k_snappy_size), for tile t (blocks [256 t, 256 t + 256)) by a workgroup of NWAVE
// waves (threads past 256 take part in the scan with nothing). The frames' workspace sizes (the decoded bytes of
// chunks too large for k_ts_decode's LDS staging, see snappy_frame_size) and chunk counts are scanned within the tile
// (out_off, choff) with the tile totals in part[2 t], part[2 t + 1] and returned (to, tc). z64k: 1024 words of LDS;
// sa, sb: NWAVE words each.
template <int NWAVE>
__device__ void ts_finish_tile(uint64_t t, lcrc_tblk_dev* __restrict__ blk, uint64_t n, const uint32_t* __restrict__ crc,
                               const uint32_t* __restrict__ mismatch, const uint8_t* __restrict__ file,
                               lcrc_desc_dev* __restrict__ frames, uint64_t* __restrict__ out_off,
                               uint64_t* __restrict__ choff, uint64_t* __restrict__ part, uint64_t* __restrict__ nchunks,
                               uint8_t* __restrict__ fstatus, lcrc_tscan_dev* __restrict__ st,
                               const uint32_t* __restrict__ gtab, uint32_t flags, uint32_t* z64k, uint64_t* sa,
                               uint64_t* sb, uint64_t& to, uint64_t& tc, const lcrc_tblk_dev& b0, uint32_t c0,
                               uint32_t m0) {
  // b0, c0, m0: this thread's block record, CRC and mismatch word, loaded by the caller before the state
  const uint64_t i = t * 256 + threadIdx.x;
  const uint64_t nd = st->n_data;
  const bool hf = st->has_filter;
  // the workgroup holding a split block's entry stages Z65536 in LDS (uniform decision)
  bool stage = false;
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k) {
    const uint64_t e = nd + k - (hf ? 0 : 1);
    stage |= st->pcnt[k] && (k > 0 || hf) && e < n && e / 256 == t;
  }
  if (stage) {
    for (uint32_t j = threadIdx.x; j < 1024; j += 64 * NWAVE) z64k[j] = gtab[TAB_Z64K + j];
    __syncthreads();
  }
  const bool mine = threadIdx.x < 256 && i < n;
  uint64_t fsize = 0, fch = 0;
  if (mine) {
    lcrc_tblk_dev b = b0;
    uint32_t flen = 0;
    if (b.status != 2) {
      b.crc = c0;
      b.type = file[b.offset + b.size];
      b.status = (m0 >> (i & 31)) & 1;
      const uint32_t k = i < nd ? 3u : (uint32_t)(i - nd) + (hf ? 0u : 1u);
      if (k < 3 && st->pcnt[k]) {
        // a block verified as pieces: crc(A || B) = Z_|B|(crc(A)) ^ crc(B) (init = xorout = ~0); every piece
        // after the first is 64 KiB long
        const uint32_t* pc = crc + st->pbase[k];
        const uint32_t np = st->pcnt[k];
        const bool masked = flags & LCRC_FLAG_MASK;
        auto unmask = [&](uint32_t v) {
          if (!masked) return v;
          const uint32_t r = v - 0xa282ead8u;
          return (r >> 17) | (r << 15);
        };
        uint32_t c = unmask(pc[0]);
        for (uint32_t q = 1; q < np; ++q)
          c = z64k[c & 0xff] ^ z64k[256 + ((c >> 8) & 0xff)] ^ z64k[512 + ((c >> 16) & 0xff)] ^ z64k[768 + (c >> 24)] ^
              unmask(pc[q]);
        if (masked) c = mask32c(c);
        b.crc = c;
        b.status = c != load_le32(file + b.offset + b.size + 1);
      }
      if (b.status == 0 && b.type > 1) b.status = 4;  // LCRC_TBLK_BAD_TYPE
      if (b.status == 0 && b.type == 1 && !(k == 2 && st->idx_dec)) flen = (uint32_t)b.size;  // (k_ts_open2 decoded
      // and checked a Snappy-framed index already)
    }
    lcrc_desc_dev f;
    f.offset = flen ? b.offset : 0;
    f.length = flen;
    f.expect_rel = LCRC_NO_EXPECT_DEV;
    blk[i] = b;
    frames[i] = f;
    uint64_t total, chunks, padded, slow;
    uint32_t mi, mo;
    const bool ok = snappy_frame_size(file + f.offset, flen, total, chunks, mi, mo, padded, &slow);
    fsize = ok ? slow : 0;  // k_ts_decode's workspace: only the chunks it cannot decode in LDS
    fch = ok ? chunks : 0;
    nchunks[i] = fch;
    fstatus[i] = ok ? 0 : 1;
  }
  uint64_t eo, ec;
  wg_scan2<NWAVE>(fsize, fch, sa, sb, eo, ec, to, tc);
  if (mine) {
    out_off[i] = eo;
    choff[i] = ec;
  }
  if (threadIdx.x == 0) {
    part[2 * t] = to;
    part[2 * t + 1] = tc;
    if (to | tc) st->any_frame = 1u;  // tiles with frames only (every writer stores the same 1: no atomic)
  }
}

// The table scan's finish: one workgroup per tile; k_ts_decode's workgroup of a tile adds the totals of the tiles
// before it (no scan launch between), and sums them all for its gate only when a tile had frames (any_frame).
// (Run as k_ts_decode's first phase instead, with the tiles' totals met by a decoupled look-back: 81.2 against
// 78.6-79.4 us per raw scan alone -- the last tile's workgroup waits for every other tile's finish either way.)
__global__ void __launch_bounds__(256) k_ts_finish(lcrc_tblk_dev* __restrict__ blk, uint64_t n,
                                                   const uint32_t* __restrict__ crc,
                                                   const uint32_t* __restrict__ mismatch,
                                                   const uint8_t* __restrict__ file, lcrc_desc_dev* __restrict__ frames,
                                                   uint64_t* __restrict__ out_off, uint64_t* __restrict__ choff,
                                                   uint64_t* __restrict__ part, uint64_t* __restrict__ nchunks,
                                                   uint8_t* __restrict__ fstatus, lcrc_tscan_dev* __restrict__ st,
                                                   const uint32_t* __restrict__ gtab, uint32_t flags) {
  __shared__ uint32_t z64k[1024];
  __shared__ uint64_t sa[4], sb[4];
  // the block's record, CRC and mismatch word loaded before the state (the count) is known, in the same round trip
  // (every index below n, the arrays' length, may be read)
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  lcrc_tblk_dev b0 = {};
  uint32_t c0 = 0, m0 = 0;
  if (i < n) {
    b0 = blk[i];
    c0 = crc[i];
    m0 = mismatch[i >> 5];
  }
  n = st->n_total < n ? st->n_total : n;
  if ((uint64_t)blockIdx.x * 256 >= n) return;  // a whole workgroup past the count (uniform)
  uint64_t to, tc;
  ts_finish_tile<4>(blockIdx.x, blk, n, crc, mismatch, file, frames, out_off, choff, part, nchunks, fstatus, st, gtab,
                    flags, z64k, sa, sb, to, tc, b0, c0, m0);
}

// the reference's order of outcomes, once every checksum is known; the count and the status for the caller
__device__ void ts_final(lcrc_tscan_dev* __restrict__ st, lcrc_tblk_dev* __restrict__ blk, uint64_t* __restrict__ n_out,
                         uint32_t* __restrict__ status_out) {
  lcrc_tscan_dev s = *st;
  if (s.status == TS_OK && s.idx_only) {
    if (blk[0].status == 1) {
      s.status = TS_CORRUPT;
      s.code = TSM_CHECKSUM;
    } else {
      s.status = TS_HOST;
    }
    s.n_total = 0;
  } else if (s.status == TS_OK) {
    const uint64_t n = s.n_total;
    const lcrc_tblk_dev ix = blk[n - 1];  // the index block, last
    if (ix.status == 1) {
      s.status = TS_CORRUPT;
      s.code = TSM_CHECKSUM;  // Table::open: "block checksum mismatch"
    } else if (s.pcode) {
      s.status = TS_CORRUPT;
      s.code = s.pcode;
    } else if (s.has_filter && blk[n - 2].status != 0) {
      // read_meta: a metaindex that does not read cleanly names no filter -- drop the filter block
      blk[n - 3] = blk[n - 2];
      blk[n - 2] = blk[n - 1];
      s.n_total = n - 1;
    }
  }
  // only the fields decided here (k_ts_decode's other workgroups may be setting st->unsorted)
  st->status = s.status;
  st->code = s.code;
  st->n_total = s.n_total;
  *n_out = s.status == TS_OK ? s.n_total : s.status == TS_CAPACITY ? s.n_data : 0;
  status_out[0] = s.status;
  status_out[1] = s.code;
}

// The table scan's last launch. Every block's content verdict -- its Snappy frame failed the framing walk or
// the decode (fstatus), or one of its chunks' masked CRC-32C differs from the stored one (the CRC pass's
// mismatch bits cmm; not read when the gate sent the frames to the host) -- and the order check of the
// offsets, then the reference's order of outcomes (ts_final). The last three blocks (filter, metaindex,
// index), which ts_final may move, are thread 0 of workgroup 0's alone.

// ---------------------------------------------------------------------------------------------------
// small helpers of the table scan and the writer-side seal
// ---------------------------------------------------------------------------------------------------
// out[i] = base[pos[i]] (the type bytes of a table's blocks)
__global__ void __launch_bounds__(256) k_gather_u8(const uint8_t* __restrict__ base, const uint64_t* __restrict__ pos,
                                                   uint64_t n, uint8_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = base[pos[i]];
}

// base[offset_i + expect_rel_i .. +4) = crc_i, little-endian: the trailer of write_raw_block
// (table.rs:519-527) or the header checksum of emit_physical_record (log.rs:61-70), in place
__global__ void __launch_bounds__(256) k_store_crc(uint8_t* __restrict__ base, uint64_t base_len,
                                                   const lcrc_desc_dev* __restrict__ descs,
                                                   const uint32_t* __restrict__ crc, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const lcrc_desc_dev d = descs[i];
  if (d.expect_rel == LCRC_NO_EXPECT_DEV) return;
  const int64_t at = (int64_t)d.offset + d.expect_rel;
  if (d.offset > base_len || at < 0 || (uint64_t)at + 4 > base_len) return;  // never written outside the buffer
  uint8_t* p = base + at;
  const uint32_t c = crc[i];
  p[0] = (uint8_t)c;
  p[1] = (uint8_t)(c >> 8);
  p[2] = (uint8_t)(c >> 16);
  p[3] = (uint8_t)(c >> 24);
}

// ---------------------------------------------------------------------------------------------------
// k_ts_decode: the table scan's last launch -- the Snappy frames decoded, every chunk's masked CRC-32C computed in
// the decoding wave and compared with the stored one, every block's content verdict, and the reference's order of
// outcomes (ts_final). It replaces three launches (the decode, a CRC pass over the decoded bytes, the close) and the
// decoded bytes' round trip through HBM: a chunk decoded in LDS is checksummed there and never written out
// (format.rs:194-206; the snap crate's FrameDecoder checks each chunk's masked CRC-32C).
//
// TD_SUB workgroups of TD_WAVES waves per 256-block tile of k_ts_finish (its in-tile scans of the frames' padded
// decoded sizes give each frame's global-memory workspace for the lane-serial path; each workgroup adds the tiles
// before its own once). A wave decodes 64 / TD_RL frames at a time, one per TD_RL-lane row (row_frame); a frame the
// row staging cannot hold goes through the whole wave (td_frame). The last three blocks (filter, metaindex, index:
// whatever ts_final may move) are the last workgroup's.
//
// Whole-wave chunk CRC (td_chunk_crc): the chunk M is read as V = 0^pad || M, |V| = 1024 np (leading zeros walked from
// register 0 stay 0, so walk(0, V) = walk(0, M)); per 1 KiB pass each lane walks 16 B (slice-by-4), the 16-lane rows
// join with Z16..Z128, the four rows with Z256 / Z512, the passes with Z1024 -- T0..T3 and Z64 or Z128 .. Z1024 from
// k_ts_decode's LDS image (TDL_*), the shorter shifts (used by this path only) from the table image in global memory.
// The init register is injected into the first min(4, |M|) bytes: walk(R, M) = walk(0, M ^ LE(R)) ^ (R >> 8 |M|) for
// |M| < 4.
// ---------------------------------------------------------------------------------------------------

// the piece of pass k of lane `lane`: V[1024 k + 16 lane, +16), init injected into V[pad, pad + q)
__device__ __forceinline__ u32x4 td_inject(u32x4 w, uint32_t x0, uint32_t pad, uint32_t q) {
  if (x0 < pad + q && x0 + 16 > pad) {
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t x = x0 + 4 * d + b;
        if (x >= pad && x < pad + q) w[d] ^= 0xFFu << (8 * b);  // CRC-32C init 0xFFFFFFFF
      }
  }
  return w;
}

template <bool FROM_LDS>
__device__ uint32_t td_chunk_crc(const uint32_t* T, const uint32_t* __restrict__ G, const uint8_t* src, uint32_t len,
                                 uint32_t lane) {
  const uint32_t np = (len + 1023) >> 10, pad = (np << 10) - len, q = len < 4 ? len : 4u;
  const uint32_t g = lane & 15;
  uint32_t acc = 0;
  for (uint32_t k = 0; k < np; ++k) {
    const uint32_t x0 = 1024 * k + 16 * lane;
    u32x4 w;
    if constexpr (FROM_LDS) {
      w = *(const u32x4*)(src + x0);  // src = V (the chunk decoded at V + pad, V[0, pad) zeroed)
    } else {  // src = M in global memory, any alignment
      if (x0 >= pad) {
        w = *(const u32x4_ua*)(src + (x0 - pad));
      } else {
        w = u32x4{0, 0, 0, 0};
        if (x0 + 16 > pad)
          for (uint32_t b = pad - x0; b < 16; ++b) w[b >> 2] |= (uint32_t)src[x0 + b - pad] << (8 * (b & 3));
      }
    }
    w = td_inject(w, x0, pad, q);
    uint32_t cv = step4(T, 0u, w.x);
    cv = step4(T, cv, w.y);
    cv = step4(T, cv, w.z);
    cv = step4(T, cv, w.w);
#pragma unroll
    for (int m = 0; m < 4; ++m) {  // row tree: 16 pieces of 16 B -> one 256 B value in lane 0 of the row
      const uint32_t pn = row_down(cv, m);
      if ((g & ((2u << m) - 1)) == 0)
        cv = (m == 3 ? zl(T, TDL_Z128, cv) : m == 2 && TD_RL == 16 ? zl(T, TDL_Z64, cv)
                                                                  : zl(G, TAB_ZPIECE + m * 1024, cv)) ^ pn;
    }
    const uint32_t r0 = __builtin_amdgcn_readlane(cv, 0), r1 = __builtin_amdgcn_readlane(cv, 16);
    const uint32_t r2 = __builtin_amdgcn_readlane(cv, 32), r3 = __builtin_amdgcn_readlane(cv, 48);
    const uint32_t a = zl(T, TDL_Z256, r0) ^ r1, b = zl(T, TDL_Z256, r2) ^ r3;
    const uint32_t pass = zl(T, TDL_Z512, a) ^ b;
    acc = k ? zl(T, TDL_Z1024, acc) ^ pass : pass;
  }
  if (len < 4) acc ^= len ? 0xFFFFFFFFu >> (8 * len) : 0xFFFFFFFFu;
  return __builtin_amdgcn_readfirstlane(acc ^ 0xFFFFFFFFu);  // raw CRC-32C (xorout)
}

// frame f decoded chunk by chunk, every chunk's masked CRC-32C checked: true when the frame is good (format.rs:194-206)
__device__ bool td_frame(const uint8_t* __restrict__ p, uint32_t len, const uint32_t* T, const uint32_t* __restrict__ G,
                         uint8_t* lin, uint8_t* lout, uint8_t* __restrict__ out, uint64_t o, uint32_t lane) {
  sn_reader rd;
  rd.init(p, len, lane);
  const uint32_t end = rd.lim;
  bool ok = true;
  uint32_t at = (uint32_t)(p - rd.a);
  // the framing was validated by k_ts_finish: chunk headers and lengths are in bounds, preambles are sane
  while (ok && at < end) {
    rd.ensure(at, lane);
    const uint32_t type = rd.byte(at);
    const uint32_t cl = rd.le(at + 1, 3);
    const uint32_t body = at + 4;
    at = body + cl;
    if (type > 1) continue;  // stream identifiers and skippable chunks
    rd.ensure(body, lane);
    const uint32_t want = rd.le(body, 4);
    uint32_t crc;
    if (type == 1) {  // uncompressed: checksummed where it lies
      crc = td_chunk_crc<false>(T, G, rd.a + body + 4, cl - 4, lane);
    } else {
      uint32_t ulen = 0, q = body + 4, used = 0;  // preamble = uncompressed length (valid: k_ts_finish)
      snappy_preamble([&](uint32_t i) { return rd.byte(q + i); }, at - q, ulen, used);
      q += used;
      if (ulen <= TD_OUT && at - q + 4 <= TD_IN) {
        // decoded at V + pad of the output staging, V[0, pad) zeroed: the CRC reads whole aligned 16 B pieces
        const uint32_t pad = ((ulen + 1023) & ~1023u) - ulen;
        for (uint32_t k = 16 * lane; k < pad; k += 1024) *(u32x4*)(lout + k) = u32x4{0, 0, 0, 0};
        const uint8_t* zs = rd.a + q;
        const uint32_t d = (uint32_t)((uintptr_t)zs & 3);
        const uint32_t* za = (const uint32_t*)(zs - d);
        const uint32_t ndw = (d + (at - q) + 3) >> 2;
        stage_to_lds(za, (lds_u8*)lin, ndw, lane, 64);
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
        ok = snappy_wave_decode(lin, d, d + (at - q), lout + pad, ulen, lane);
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
        crc = ok ? td_chunk_crc<true>(T, G, lout, ulen, lane) : 0u;
      } else {  // too large for the staging: lane-serial into this frame's workspace, checksummed there
        uint64_t oo = o;
        if (lane == 0) ok = sn_serial_decode(rd.a + q, rd.a + at, out, oo, o + ulen);
        ok = bcast(ok ? 1u : 0u) != 0;
        __threadfence_block();
        crc = ok ? td_chunk_crc<false>(T, G, out + o, ulen, lane) : 0u;
        o += (ulen + 15) & ~15u;
      }
    }
    ok = ok && mask32c(crc) == want;
  }
  return ok;
}

// ---- 64 / TD_RL frames per wave: one per TD_RL-lane row (lane g = lane % TD_RL of row lane / TD_RL) ----
typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
typedef __attribute__((address_space(3))) const u32x4 lds_cu32x4;

// a select of two computed values (clang emits `c ? a : b` with non-trivial arms as a branch, which the optimiser
// then keeps, sinking the arms' work into it: exec-mask juggling in a divergent loop)
__device__ __forceinline__ uint32_t sel(bool c, uint32_t a, uint32_t b) { return c ? a : b; }

// An element's bytes moved within a row's staging: m bytes to D from S = Sl (a literal, the input) or D - off (a copy,
// earlier output); the pass layout and the repeat as row_snappy_decode describes. Two halves: the loads of pass 0
// (row_move_load, issued as soon as the element's header is decoded) and the rest (row_move_store, once the element is
// validated: m = 0 for an element that is not moved).
struct RowMoveLd {
  uint32_t S, old, d0, d1, d2;
};
__device__ __forceinline__ RowMoveLd row_move_load(const lds_u8* B, uint32_t D, uint32_t Sl, uint32_t off, bool lit,
                                                   uint32_t g) {
  RowMoveLd l;
  l.S = sel(lit, Sl, D - min(off, D));  // (an offset past the output is refused later: clamped, the reads stay in the row)
  const uint32_t Da = D & ~3u, sh = D & 3u;
  l.old = *(lds_cu32*)(B + Da);
  const uint32_t A = (l.S + 8 * g - sh) & ~3u;
  l.d0 = *(lds_cu32*)(B + A);
  l.d1 = *(lds_cu32*)(B + A + 4);
  l.d2 = *(lds_cu32*)(B + A + 8);
  return l;
}
__device__ __forceinline__ void row_move_store(lds_u8* B, const RowMoveLd& l, uint32_t D, uint32_t m, uint32_t off,
                                               bool lit, uint32_t gmask, uint32_t g, uint32_t dump) {
  typedef __attribute__((address_space(3))) uint32_t lds_w32;
  const uint32_t S = l.S;
  const bool pat = !lit & (off < m) & (off < 128);
  const uint32_t mm = sel(pat, 0u, m), Da = D & ~3u, sh = D & 3u;
  // pass 0 (every row; a row with nothing to move -- finished, inactive, or a repeat, which goes bytewise below --
  // writes nothing: its first lane's merged dword would carry garbage past D into bytes the row's uncompressed-chunk
  // copy has written)
  const int r0 = (int)(8 * g) - (int)sh;  // element-relative offset of the lane's first dword
  const uint32_t al = (S + (uint32_t)r0) & 3u;
  const uint32_t keep = ((1u << (8 * sh)) - 1) & gmask;  // (sh = 0: nothing kept)
  const uint32_t v0 = (__builtin_amdgcn_alignbyte(l.d1, l.d0, al) & ~keep) | (l.old & keep);
  const uint32_t v1 = __builtin_amdgcn_alignbyte(l.d2, l.d1, al);
  const uint32_t a0 = Da + 8 * g;
  *(lds_w32*)(B + sel((mm != 0) & (r0 < (int)mm), a0, dump)) = v0;
  *(lds_w32*)(B + sel(r0 + 4 < (int)mm, a0 + 4, dump)) = v1;
  // elements longer than a pass: literals (and with 8-lane rows copies of over 61 B; a copy that is not a repeat
  // reads only output written before it)
  if (__builtin_amdgcn_ballot_w64(sh + mm > TD_PASS)) {
    for (uint32_t b = TD_PASS; __builtin_amdgcn_ballot_w64(b < sh + mm); b += TD_PASS) {
      const int r = (int)(b + 8 * g) - (int)sh;
      const uint32_t sb = S + (uint32_t)r, Ab = sb & ~3u, ab = sb & 3u;
      const uint32_t e0 = *(lds_cu32*)(B + Ab), e1 = *(lds_cu32*)(B + Ab + 4), e2 = *(lds_cu32*)(B + Ab + 8);
      *(lds_w32*)(B + sel(r < (int)mm, Da + b + 8 * g, dump)) = __builtin_amdgcn_alignbyte(e1, e0, ab);
      *(lds_w32*)(B + sel(r + 4 < (int)mm, Da + b + 8 * g + 4, dump)) = __builtin_amdgcn_alignbyte(e2, e1, ab);
    }
  }
  if (__builtin_amdgcn_ballot_w64(pat)) {  // (pat: a copy, m <= 64: 64 / TD_RL bytes a lane)
    constexpr int PB = 64 / TD_RL;
    uint32_t v[PB];
#pragma unroll
    for (int k = 0; k < PB; ++k) {
      const uint32_t j = PB * g + k;
      v[k] = pat ? B[S + small_mod(j, off)] : 0u;
    }
#pragma unroll
    for (int k = 0; k < PB; ++k) {
      const uint32_t j = PB * g + k;
      B[pat && j < m ? D + j : dump] = (uint8_t)v[k];
    }
  }
}

// One Snappy chunk per row: the elements B[q, qe) decoded into B[OB, OB + ulen) (both in the row's LDS staging, B
// its base). Every row walks its own chain -- one element per iteration, its header two dwords of the row's staging
// read one element ahead (its position is known once the previous header is decoded; the input is never written) --
// and decodes the header without branches (selects only: the round-4 decoder's divergent if/else cost more SALU exec
// juggling than VALU work). An element is moved in destination-aligned dwords, 8 B per lane and TD_PASS per row pass:
// each lane reads the three aligned dwords holding its 8 source bytes and funnel-shifts them (v_alignbyte); the row's
// first dword keeps the bytes before the element from the dword already there; the bytes a row's last dword writes
// past the element are overwritten by the next element's (in order: a wave's LDS operations execute in issue order),
// and V's end is dword-aligned, so nothing past it is touched. A copy whose source overlaps its own destination
// closer than a pass (offset < length, offset < 128: the Snappy repeat) goes bytewise, j mod offset. Validation as
// the wave decoder's. Rows with active = false only ride along. Returns the row's verdict: 0 good (output ends at
// ulen), 1 malformed, 2 given up (the in-place output would reach unread input).
__device__ __forceinline__ uint32_t row_snappy_decode(lds_u8* B, uint32_t q, uint32_t qe, uint32_t OB, uint32_t ulen,
                                                      bool active, uint32_t g, uint32_t dump) {
  uint32_t w = 0, res = 0;  // res: 1 malformed, 2 given up in place (the row stops at either)
  uint32_t h0, h1, hs;
  auto fetch = [&](uint32_t at) {
    const uint32_t ba = at & ~3u;
    h0 = *(lds_cu32*)(B + ba);
    h1 = *(lds_cu32*)(B + ba + 4);
    hs = at & 3;
  };
  fetch(active && q < qe ? q : 0u);
  // (the loop state in VGPRs: a bool carried around a divergent loop costs lane-mask merges every iteration)
  uint32_t livef = active && q < qe ? 1u : 0u;
  const uint32_t gmask = g == 0 ? ~0u : 0u;  // the row's first lane merges the element's first dword
  // the first header waited for here, so the loop's own wait (for the next header, issued with the element's
  // source reads) is the only one per element: never one for the writes of the element before
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  // one LDS round trip per element: the next header, the dword the element's first write merges with and the pass-0
  // source dwords are issued together and waited for together; the writes are never waited for (only ordered)
  while (__builtin_amdgcn_ballot_w64(livef != 0)) {
    const bool live = livef != 0;
    const uint32_t lo = __builtin_amdgcn_alignbyte(h1, h0, hs);                         // bytes q .. q + 3
    const uint32_t ext = sel(hs == 3, h1, __builtin_amdgcn_alignbyte(h1, h0, hs + 1));  // bytes q + 1 .. q + 4
    const uint32_t t = lo & 0xFFu, typ = t & 3, L = t >> 2;
    const uint32_t room = qe - q;  // (q >= qe: live = false, nothing below counts)
    // (bitwise & | on the conditions and selects of computed values: no short-circuit branches)
    const bool lit = typ == 0, c1 = typ == 1, c2 = typ == 2;
    // literal: L < 60: length L + 1; else L - 59 little-endian bytes of length - 1 follow the tag
    const uint32_t nb = sel(L >= 60, L - 59, 0u);
    const uint32_t lbits = __builtin_amdgcn_ubfe(ext, 0, 8 * nb);  // (nb = 4: width 32 reads as 0, selected away)
    const uint32_t lm1 = sel(nb == 4, ext, sel(nb == 0, L, lbits));
    // copies: 1-byte offset (tag bits 5..7 = offset bits 8..10, length 4..11), 2-byte, 4-byte offset
    const uint32_t o1 = ((t >> 5) << 8) | (ext & 0xFFu), o2 = ext & 0xFFFFu;
    const uint32_t off = sel(c1, o1, sel(c2, o2, ext));
    const uint32_t hdr = sel(lit, 1 + nb, (0x5320u >> (4 * typ)) & 0xFu);  // 1 + nb | 2 | 3 | 5
    const uint32_t n = sel(lit, lm1 + 1, sel(c1, 4 + (L & 7), L + 1));
    const uint32_t qn0 = q + hdr + sel(lit, n, 0u);
    // the next header and the element's pass-0 source read before the element's verdict is known (a row whose element
    // fails stops: what it read is never used), so their LDS round trip runs beside the validation; min: qn0 <= qe,
    // the 8 bytes from qe & ~3 lie in the row's input staging and its slack
    const uint32_t qh = q + hdr;
    fetch(min(qn0, qe));
    const RowMoveLd ld = row_move_load(B, OB + w, qh, off, lit, g);
    __builtin_amdgcn_sched_barrier(0);  // (the scheduler would otherwise sink the loads below the validation)
    const bool good = (room >= hdr) & (!lit | ((lm1 < room - hdr) & ((nb == 0) | (room >= 5))));
    // (w <= ulen holds; off - 1 >= w: a copy's offset 0 or past the output)
    const bool bad = live & (!good | (n > ulen - w) | (!lit & (off - 1u >= w)));
    // in place (output and input in one row area, the output from its start): every dword this element writes lies
    // before the input not yet read -- from the next element on (its header is read before these writes), and for a
    // literal longer than a pass, before its own bytes' later passes. Else the row gives the frame up (spill)
    const bool sp = live & !bad & ((((OB + w + n + 3) & ~3u) > qn0) | (lit & (OB + w + 8 > qh)));
    res = sel(bad, 1u, sel(sp, 2u, res));
    const bool ex = live & !bad & !sp;
    const uint32_t m = sel(ex, n, 0u);
    const uint32_t qn = sel(ex, qn0, q);
    row_move_store(B, ld, OB + w, m, off, lit, gmask, g, dump);
    q = qn;
    w += m;
    livef = sel(ex & (qn < qe), 1u, 0u);
  }
  return res ? res : w == ulen ? 0u : 1u;
}

// every lane of a k_ts_decode row <- the row's first lane (8-lane rows: ds_swizzle in bit-mask mode, source lane
// = lane & 0x18 within each 32)
__device__ __forceinline__ uint32_t td_row_bcast0(uint32_t v, uint32_t lane) {
  if constexpr (TD_RL == 16) return row_bcast0(v, lane);
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x18);
}

// The CRC-32C of M = V[0, len) per row, walked as M || 0^z to whole 1 KiB passes (z = 1024 np - len, undone at the end
// by one GF(2) multiply with invz = x^(-8z)), the init register already XORed into the first min(4, len) bytes of M by
// the caller (the decoded bytes are not kept): per 1 KiB pass each lane walks 1024 / TD_RL B (slice-by-4), the row tree
// joins the lanes with Z64, Z128, Z256, Z512 (8-lane rows: 128 B a lane, Z128 .. Z512), and the passes chain with
// Z1024. The zeros are not in the row (round 6): the caller zeroes M's bytes up to the next 16 B boundary, and a piece
// wholly past M is read from Z0, 16 zero bytes. A lane's walk over a pass is one dependent chain of LDS lookups (32 of
// them for 128 B), so the passes -- independent until the Z1024 chaining -- are walked at once, TR_NP chains a lane,
// when a row of the wave has that many (every chunk that fills a row: a 4 KiB block); else one pass after the other.
constexpr uint32_t TR_NP = (TR_OUT + 1023) / 1024;  // a row chunk's passes at most
__device__ __forceinline__ uint32_t row_tree(const uint32_t* T, uint32_t cv, uint32_t g, uint32_t lane) {
  // level m joins lane g with g + 2^m, shifting the left part by (1024 / TD_RL) * 2^m bytes (Z64 .. Z512 for 16
  // lanes, Z128 .. Z512 for 8)
#pragma unroll
  for (int m = 0; (1u << m) < TD_RL; ++m) {
    const uint32_t pn = row_down(cv, m);
    const int zt = TD_RL == 16 ? (m == 0 ? TDL_Z64 : m == 1 ? TDL_Z128 : m == 2 ? TDL_Z256 : TDL_Z512)
                               : (m == 0 ? TDL_Z128 : m == 1 ? TDL_Z256 : TDL_Z512);
    if ((g & ((2u << m) - 1)) == 0) cv = zl(T, zt, cv) ^ pn;
  }
  return td_row_bcast0(cv, lane);
}
__device__ __forceinline__ uint32_t row_chunk_crc(const uint32_t* T, const lds_u8* V, const lds_u8* Z0, uint32_t len,
                                                  bool active, uint32_t g, uint32_t lane, uint32_t invz) {
  constexpr uint32_t LB = 1024 / TD_RL, SP = LB / 16;  // bytes a lane walks per pass, in 16 B pieces
  const uint32_t np = active ? (len + 1023) >> 10 : 0u;
  uint32_t acc = 0;
  if (__builtin_amdgcn_ballot_w64(np == TR_NP)) {
    uint32_t cv[TR_NP];
#pragma unroll
    for (uint32_t j = 0; j < TR_NP; ++j) cv[j] = 0;
#pragma unroll
    for (uint32_t sp = 0; sp < SP; ++sp) {
      u32x4 w[TR_NP];
#pragma unroll
      for (uint32_t j = 0; j < TR_NP; ++j) {
        const uint32_t x0 = 1024 * j + LB * g + 16 * sp;
        w[j] = *(lds_cu32x4*)(x0 < len ? V + x0 : Z0);
      }
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (uint32_t j = 0; j < TR_NP; ++j) cv[j] = step4(T, cv[j], w[j][d]);
    }
    uint32_t pass[TR_NP];
#pragma unroll
    for (uint32_t j = 0; j < TR_NP; ++j) pass[j] = row_tree(T, cv[j], g, lane);
#pragma unroll
    for (uint32_t j = 0; j < TR_NP; ++j)
      if (j < np) acc = j ? zl(T, TDL_Z1024, acc) ^ pass[j] : pass[j];
  } else {
    for (uint32_t k = 0; __builtin_amdgcn_ballot_w64(k < np); ++k) {
      uint32_t cv = 0;
#pragma unroll
      for (uint32_t sp = 0; sp < SP; ++sp) {
        const uint32_t x0 = 1024 * k + LB * g + 16 * sp;
        const u32x4 w = *(lds_cu32x4*)(x0 < len ? V + x0 : Z0);
        cv = step4(T, cv, w.x);
        cv = step4(T, cv, w.y);
        cv = step4(T, cv, w.z);
        cv = step4(T, cv, w.w);
      }
      const uint32_t pass = row_tree(T, cv, g, lane);
      if (k < np) acc = k ? zl(T, TDL_Z1024, acc) ^ pass : pass;
    }
  }
  // walk(M || 0^z) = Z_z(walk(M)), undone by x^(-8z)
  if (__builtin_amdgcn_ballot_w64(active && (len & 1023) != 0)) acc = (len & 1023) ? gf_mul(invz, acc, 0x82F63B78u) : acc;
  if (len < 4) acc ^= len ? 0xFFFFFFFFu >> (8 * len) : 0xFFFFFFFFu;
  return acc ^ 0xFFFFFFFFu;
}

// A row's frame staging through registers: the next group's frames are loaded (row_stage_load, 16 B units, lane g of
// the row taking units g, g + TD_RL, ...) while this group decodes, and stored to the row's input area when its turn
// comes (row_stage_store) -- the global-memory latency of the staging off the decode's path
constexpr int TR_UNITS = (TR_IN + 16 * TD_RL - 1) / (16 * TD_RL);  // TD_RL lanes x TR_UNITS x 16 B >= the row's input
static_assert(TD_RL * TR_UNITS * 16 >= TR_IN, "row staging units");
struct RowStage {
  u32x4 t[TR_UNITS];
  uint32_t tail;
};
__device__ __forceinline__ void row_stage_load(RowStage& s, const uint32_t* za, uint32_t ndw, uint32_t g) {
  const uint32_t units = ndw >> 2;
#pragma unroll
  for (int i = 0; i < TR_UNITS; ++i) {
    const uint32_t u = g + TD_RL * i;
    if (u < units) s.t[i] = *(const u32x4_ua*)(za + 4 * u);
  }
  // (unconditional: a select or an exec-masked load into the register would make the compiler wait for every load
  // in flight here; a frame's last dword +12 B stays inside the file, the data blocks being followed by the index
  // block and the footer)
  s.tail = za[4 * units + (g & 3)];
}
__device__ __forceinline__ void row_stage_store(const RowStage& s, lds_u8* dst, uint32_t ndw, uint32_t g) {
  typedef __attribute__((address_space(3))) u32x4 lds_u32x4_t;
  typedef __attribute__((address_space(3))) uint32_t lds_u32_t;
  const uint32_t units = ndw >> 2;
#pragma unroll
  for (int i = 0; i < TR_UNITS; ++i) {
    const uint32_t u = g + TD_RL * i;
    if (u < units) *(lds_u32x4_t*)(dst + 16 * u) = s.t[i];
  }
  if (g < (ndw & 3)) ((lds_u32_t*)dst)[4 * units + g] = s.tail;
}

// One frame per row (`elig` rows only), staged by the caller at B[ib + d, ib + d + len) (row_stage_load / _store), its
// chunks walked there, each data chunk decoded in place (or, uncompressed, copied forward) to B[0, ulen) and
// checksummed. Returns 0 good, 1 bad, 2 deferred to the whole-wave decoder (a chunk over TR_OUT, or an in-place decode
// that would reach unread input).
__device__ __forceinline__ uint32_t row_frame(uint32_t d, uint32_t len, bool elig, const uint32_t* T, lds_u8* B,
                                              const lds_u8* Z0, uint32_t ib, uint32_t g, uint32_t lane,
                                              const uint32_t* __restrict__ inv) {
  lds_u8* const in = B + ib;
  // the framing was validated by k_ts_finish: headers and lengths are in bounds, preambles are sane
  uint32_t pos = d, res = 0;
  const uint32_t end = d + (elig ? len : 0u);
  while (true) {
    bool have = false;
    uint32_t type = 0, cl = 0;
    while (elig && res == 0 && pos < end) {  // the next data chunk (stream identifier, skippable chunks passed)
      type = in[pos];
      cl = in[pos + 1] | ((uint32_t)in[pos + 2] << 8) | ((uint32_t)in[pos + 3] << 16);
      if (type <= 1) {
        have = true;
        break;
      }
      pos += 4 + cl;
    }
    if (!__builtin_amdgcn_ballot_w64(have)) break;
    const uint32_t body = pos + 4, next = body + cl;
    uint32_t want = 0, ulen = 0, q = body + 4;
    if (have) {
      want = in[body] | ((uint32_t)in[body + 1] << 8) | ((uint32_t)in[body + 2] << 16) | ((uint32_t)in[body + 3] << 24);
      if (type == 1) {
        ulen = cl - 4;
      } else {  // preamble = uncompressed length (valid: k_ts_finish)
        uint32_t used = 0;
        snappy_preamble([&](uint32_t i) { return (uint32_t)in[q + i]; }, next - q, ulen, used);
        q += used;
      }
      // too large for the row, or M's zeroed bytes up to the next 16 B boundary would reach a later chunk's input:
      // the whole wave
      if (ulen > TR_OUT || (next < end && ((ulen + 15) & ~15u) > ib + next)) {
        res = 2;
        have = false;
      }
    }
    const uint32_t z = have ? ((ulen + 1023) & ~1023u) - ulen : 0u;
    const uint32_t invz = inv[z];  // x^(-8z) (loaded now, used after the decode)
    if (__builtin_amdgcn_ballot_w64(have && type == 1))  // uncompressed: copied forward to B[0, ulen) (in place: the
      // destination is below the source, and each byte is read before anything is stored at or above it)
      for (uint32_t k = g; k < (have && type == 1 ? ulen : 0u); k += TD_RL) B[k] = in[q + k];
    const bool dec = have && type == 0;
    const uint32_t rd = row_snappy_decode(B, ib + q, ib + next, 0u, ulen, dec, g, TR_ROW - 4);
    const bool ok = !dec || rd == 0;
    if (dec && rd == 2) {
      res = 2;  // given up in place: the whole wave decodes the frame from the file
      have = false;
    }
    // B[ulen, ulen rounded up to 16) zeroed (the CRC reads whole 16 B pieces up to there, Z0 past it), then the init
    // register injected into M's first bytes
    const uint32_t u4 = (ulen + 3) & ~3u, u16 = (ulen + 15) & ~15u;
    if (have && ulen + g < u4) B[ulen + g] = 0;
    if (have && u4 + 4 * g < u16) *(__attribute__((address_space(3))) uint32_t*)(B + u4 + 4 * g) = 0;
    if (have && g < (ulen < 4 ? ulen : 4u)) B[g] ^= 0xFFu;
    const uint32_t crc = row_chunk_crc(T, B, Z0, ulen, have, g, lane, invz);
    if (have) {
      if (!ok || mask32c(crc) != want) res = 1;
      pos = next;
    }
  }
  return res;
}

__global__ void __launch_bounds__(64 * TD_WAVES) k_ts_decode(const uint8_t* __restrict__ file,
                                                            const lcrc_desc_dev* __restrict__ frames,
                                                            const uint64_t* __restrict__ out_off, uint8_t* __restrict__ out,
                                                            const uint8_t* __restrict__ fstatus,
                                                            lcrc_tscan_dev* __restrict__ st, lcrc_tblk_dev* __restrict__ blk,
                                                            const uint32_t* __restrict__ tab_c, uint64_t ts_out_cap,
                                                            const uint64_t* __restrict__ tparts,
                                                            uint64_t* __restrict__ n_out, uint32_t* __restrict__ status_out,
                                                            uint64_t bound) {
  extern __shared__ __attribute__((aligned(16))) uint8_t td_lds[];
  uint32_t* const T = (uint32_t*)td_lds;
  // workgroup b: sub-tile b % TD_SUB of tile t = b / TD_SUB, the frames lo .. lo + TD_SUBN
  const uint64_t t = blockIdx.x / TD_SUB, lo = t * 256 + (blockIdx.x % TD_SUB) * TD_SUBN;
  // the content verdict's inputs for this thread's block, loaded with the state (bound: the arrays' length)
  const uint64_t j = lo + threadIdx.x;
  uint8_t fs_j = 0;
  uint64_t off_j = 0, off_p = 0;
  if (threadIdx.x < TD_SUBN && j < bound) {
    fs_j = fstatus[j];
    off_j = blk[j].offset;
    off_p = j ? blk[j - 1].offset : 0;
  }
  uint8_t* const bad = td_lds + TDL_WORDS * 4 + TD_WAVES * TD_WAVE_LDS;  // the sub-tile's flags (256) + the meta blocks
  const uint32_t lane = __lane_id(), wv = threadIdx.x >> 6;
  // the block count from fields ts_final leaves alone (it may shrink n_total while later workgroups start)
  const bool live = st->status == TS_OK && !st->idx_only;
  const uint64_t n = live ? st->n_data + (st->has_filter ? 3 : 2) : 0;
  // TD_SUB workgroups per 256 data blocks; the meta blocks after them (filter, metaindex, index) are the last
  // workgroup's (its wave 0, after the rows): a table of 65,536 data blocks is 256 tiles, not 257; and a table without
  // a filter keeps its last data block in the rows (as one of "the last three" it went through the whole-wave decoder
  // alone, after the rows: ~35 us of the scan's tail)
  const uint64_t tail = live ? st->n_data : 0, tiles = n ? (tail + 255) / 256 + (tail ? 0 : 1) : 0;
  const bool last = n && t == tiles - 1 && blockIdx.x % TD_SUB == TD_SUB - 1;
  // (workgroup 0 runs ts_final when nothing is live; a sub-tile past the data blocks has nothing else to do)
  if ((t >= tiles || lo >= tail) && blockIdx.x != 0 && !last) return;
#ifdef LCRC_PROBE_CLOCK  // diagnostic build: phase stamps of workgroup b in lcrc_dbg_stamp row 2304 + b
#define TD_STAMP(k) \
  if (threadIdx.x == 0 && blockIdx.x < 768) lcrc_dbg_stamp[(2304 + blockIdx.x) * 8 + (k)] = __builtin_amdgcn_s_memrealtime()
#else
#define TD_STAMP(k)
#endif
  TD_STAMP(0);
  uint64_t before = 0, total = 0, chunks = 0;
  bool over = false;
  // the gate: the decoded total and the chunk count the frames need against the workspace (decided alike by every
  // workgroup from the tile totals; workgroup 0 records it -- over: the host path). No frames: no sums.
  if (n && st->any_frame) {
    unsigned long long xb = 0, xo = 0, xc = 0;
    for (uint64_t w = lane; w < (n + 255) / 256; w += 64) {  // (k_ts_finish's tiles: the last may hold only some
      // of the meta blocks)
      const uint64_t v = tparts[2 * w];
      xo += v;
      xc += tparts[2 * w + 1];
      if (w < t) xb += v;
    }
    for (int d = 1; d < 64; d <<= 1) {
      xo += __shfl_xor(xo, d, 64);
      xc += __shfl_xor(xc, d, 64);
      xb += __shfl_xor(xb, d, 64);
    }
    before = xb;
    total = xo;
    chunks = xc;
  }
  over = total > ts_out_cap;
  // recorded by workgroup 0 and by the last tile's workgroup (the same values): the last one runs ts_final and is the
  // only one that changes st->status, so its `live` is always the scan's own; workgroup 0 may read a status the last
  // one has already set to TS_HOST (frames over the workspace) and skip the record
  if (threadIdx.x == 0 && live && (blockIdx.x == 0 || last)) {
    st->need_out = total;
    st->need_chunks = chunks;
    st->gate = over ? 1u : chunks == 0 ? 2u : 0u;
    st->n_chunks = over ? 0 : chunks;
  }
  TD_STAMP(3);
  const bool dec = !over && chunks;
  for (uint32_t i = threadIdx.x; i < 256 + 16 + 16; i += blockDim.x) bad[i] = 0;  // (+ the zero piece)
  if (dec)  // the LDS image (TDL_*): the table image's T0..T3, then its Z64 or Z128 .. Z1024
    for (uint32_t i = threadIdx.x; i < TDL_WORDS / 4; i += blockDim.x)
      ((u32x4*)T)[i] = ((const u32x4*)tab_c)[i < 256 ? i : i + (TDL_ZSRC - 1024) / 4];
  __syncthreads();
  if (dec) {
    // this sub-tile's frames (the meta blocks excluded): TD_RPW per wave at a time, one per row, over a static share of
    // the sub-tile's TD_SUBN / TD_RPW groups, the same for every wave (round 5's six waves of four rows: waves 2 and 3
    // took more, as the hardware puts a workgroup's waves on the SIMDs in order, so waves 0/4 and 1/5 shared a SIMD).
    // A frame the row cannot decode (bad[] = 2) then through the whole wave, in its wave's row area (or two waves');
    // then the last workgroup's wave 0 the meta blocks.
    const uint64_t hi = lo + TD_SUBN < tail ? lo + TD_SUBN : tail;
    const uint32_t r = lane / TD_RL, g = lane % TD_RL;
    constexpr uint32_t GPW = TD_SUBN / TD_RPW / TD_WAVES;  // groups a wave
    static_assert(GPW * TD_RPW <= 64, "a wave's groups: one descriptor a lane");
    const uint32_t gbeg = GPW * wv, gcnt = GPW;
    lds_u8* const rb = (lds_u8*)(td_lds + TDL_WORDS * 4 + wv * TD_WAVE_LDS + r * TR_ROW);
    const uint32_t* const inv = tab_c + TAB_INV;
    // the wave's frames lo + TD_RPW (gbeg + k) + r (k < gcnt): their descriptors loaded at once, lane TD_RPW k + r
    // holding frame k's of row r; each group's frames staged through registers one group ahead (RowStage)
    uint64_t d_off = 0;
    uint32_t d_len = 0;
    {
      const uint64_t f = lo + TD_RPW * (gbeg + lane / TD_RPW) + lane % TD_RPW;
      if (lane / TD_RPW < gcnt && f < hi) {
        d_len = frames[f].length;
        d_off = frames[f].offset;
        if (fstatus[f]) d_len |= 0x80000000u;  // (a frame whose framing walk failed: not live)
      }
    }
    auto group = [&](uint32_t k, uint32_t& len, bool& live, bool& elig, uint32_t& d, const uint32_t*& za,
                     uint32_t& ndw) {
      const int src = (int)(TD_RPW * (k % GPW) + r) * 4;
      const uint32_t lw = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)d_len);
      const uint64_t of = (uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)d_off) |
                          ((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(d_off >> 32)) << 32);
      const bool valid = k < gcnt && lo + TD_RPW * (gbeg + k) + r < hi;
      len = valid ? lw & 0x7FFFFFFFu : 0u;
      live = len && !(lw >> 31);
      elig = live && len + 3 <= TR_IN - 16;
      const uint8_t* pf = file + (valid ? of : 0);
      d = elig ? (uint32_t)((uintptr_t)pf & 3) : 0u;
      za = (const uint32_t*)(pf - d);
      ndw = elig ? (d + len + 3) >> 2 : 0u;
    };
    RowStage stg;
    uint32_t len, d, ndw;
    bool live, elig;
    const uint32_t* za;
    group(0, len, live, elig, d, za, ndw);
    row_stage_load(stg, za, ndw, g);
    for (uint32_t k = 0; k < gcnt && lo + TD_RPW * (gbeg + k) < hi; ++k) {
      const uint32_t len_c = len, d_c = d;
      const bool live_c = live, elig_c = elig;
      // the frame staged at the row's end (16-aligned), the decoded chunk growing from the row's start towards it
      const uint32_t ib = (TR_ROW - 16 - 4 * ndw) & ~15u;
      row_stage_store(stg, rb + ib, ndw, g);
      group(k + 1, len, live, elig, d, za, ndw);
      row_stage_load(stg, za, ndw, g);  // (in flight while this group decodes)
      __builtin_amdgcn_wave_barrier();
      const uint32_t v = row_frame(d_c, len_c, elig_c, T, rb, (const lds_u8*)(bad + 256 + 16), ib, g, lane, inv);
      if (live_c && g == 0) bad[TD_RPW * (gbeg + k) + r] = elig_c ? (uint8_t)v : 2;
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only: the next group's loads stay in flight
      __builtin_amdgcn_wave_barrier();  // (the next round overwrites the row staging)
    }
  }
  __syncthreads();  // every row done: the whole-wave decoder takes one or two (TD_WW) waves' row areas
  if (dec) {
    const uint64_t hi = lo + TD_SUBN < tail ? lo + TD_SUBN : tail;
    uint8_t* const lin = td_lds + TDL_WORDS * 4 + (wv / TD_WW) * TD_WW * TD_WAVE_LDS;
    uint8_t* const lout = lin + TD_IN + SN_SLACK;
    if (wv % TD_WW == 0)
      for (uint64_t f = lo + wv / TD_WW; f < hi; f += TD_WAVES / TD_WW)
        if (bad[f - lo] == 2) {
          const bool ok = td_frame(file + frames[f].offset, frames[f].length, T, tab_c, lin, lout, out, out_off[f] + before, lane);
          __builtin_amdgcn_s_waitcnt(0);
          __builtin_amdgcn_wave_barrier();
          if (lane == 0) bad[f - lo] = ok ? 0 : 1;
        }
    if (last && wv == 0)
      for (uint64_t f = tail; f < n; ++f) {
        const uint64_t tb = (f / 256 == t) ? before : 0;  // (a meta block in k_ts_finish's tile after this
        // workgroup's: its workspace offset is that tile's; the tiles before it are summed here)
        uint64_t base_o = tb;
        if (f / 256 != t) {  // (the tile after this workgroup's: k_ts_finish's tiles are 256 blocks)
          unsigned long long xb = 0;
          for (uint64_t w = lane; w < f / 256; w += 64) xb += tparts[2 * w];
          for (int d = 1; d < 64; d <<= 1) xb += __shfl_xor(xb, d, 64);
          base_o = xb;
        }
        if (frames[f].length && !fstatus[f] &&
            !td_frame(file + frames[f].offset, frames[f].length, T, tab_c, lin, lout, out, out_off[f] + base_o, lane) &&
            lane == 0)
          bad[256 + (f - tail)] = 1;
      }
  }
  __syncthreads();
  // content verdicts (k_ts_finish left fstatus = 1 for a frame whose framing walk failed)
  auto content = [&](uint64_t j, bool fb) {
    if (fstatus[j] || fb) blk[j].status = 3;  // LCRC_TBLK_BAD_CONTENT
    if (j > 0 && blk[j - 1].offset > blk[j].offset) st->unsorted = 1;
  };
  if (threadIdx.x < TD_SUBN && j < tail && j < lo + TD_SUBN) {  // (content() with the values loaded at the start)
    if (fs_j || bad[threadIdx.x]) blk[j].status = 3;  // LCRC_TBLK_BAD_CONTENT
    if (j > 0 && off_p > off_j) st->unsorted = 1;
  }
  TD_STAMP(4);
  if (threadIdx.x == 0 && (last || (n == 0 && blockIdx.x == 0))) {
    for (uint64_t k = tail; k < n; ++k) content(k, bad[256 + (k - tail)] != 0);
    if (over && st->status == TS_OK) st->status = TS_HOST;
    ts_final(st, blk, n_out, status_out);
  }
  TD_STAMP(5);
}

constexpr uint32_t TO_IN = 32768 + 16;  // compressed bytes staged (+ the dword alignment)
constexpr uint32_t TO_OUT = 65536;      // a whole chunk's output, V = 0^pad || M a multiple of 1 KiB
constexpr uint32_t TO_BM = 8192 + 16;   // the element-start bitmap (+ one word past the end)
// ---------------------------------------------------------------------------------------------------
// k_ts_open2 (lcrc_table_scan_async_ex with LCRC_TSCAN_SNAPPY_INDEX): the table scan's first launch when the table was
// written with compression -- its index block is then usually a Snappy frame (table.rs:430, write_block keeps the
// frame when it saves 12.5%) -- decodes that frame on the device, as Table::open's read_block_from_file does on the
// host (format.rs:194-206), so that the index walk reads the decoded contents instead of handing the table to the
// host. iopen[0]: 1 framed | 2 decoded (framing good, total within the workspace) | 4 over the workspace; iopen[1]:
// the decoded length; iopen[2]: set by a chunk that does not decode or check (the index walk's last ticket clears
// it). The index block's own checksum comes with the batch, as for a raw index; every verdict on the footer and the
// handle is ts_open_state's. A 16-wave workgroup per 64 KiB index chunk (round 4's one wave per chunk left 29 CUs
// decoding the bench table's index for 0.73 ms); the chunk's decode is data-parallel end to end:
//  A. every parse window (64 candidate element starts) gets, for each candidate, the element that would start there
//     and -- by pointer jumping inside the window, five ds_bpermute rounds (elements are >= 2 bytes) -- the first
//     start at or past the window's end reached from it (its exit; a malformed element on the way: none);
//  B. one thread follows the real chain from window to window through those exits (one LDS read per window);
//  C. each window's chain from its entry (the wave decoder's v_readlane walk): its element count and output bytes;
//  D. exclusive scans of both over the windows;
//  E. each window's element records and start bits at their global positions, with the wave decoder's validation;
//  F. every output byte's source -- a literal's input byte, or an earlier output byte -- in a global scratch array,
//     resolved by pointer jumping over the whole chunk (a copy of a copy of a copy: an index block's keys) until
//     every source is a literal byte, then the bytes gathered;
// then the chunk's masked CRC-32C with its 1 KiB passes spread over the waves and joined by one thread (Z1024), and
// the copy-out. A chunk with more elements than the record area holds goes through the wave decoder (one wave).
// ---------------------------------------------------------------------------------------------------
constexpr uint32_t T2_THREADS = 1024, T2_WAVES = 16, T2_GRID = 32;
constexpr uint32_t T2_ECAP = 6400;                 // element records (ea, eb)
constexpr uint32_t T2_NWIN = (TO_IN + 63) / 64;     // parse windows of a staged chunk
constexpr uint32_t T2_O_IN = 0, T2_O_OUT = TO_IN + SN_SLACK, T2_O_BM = T2_O_OUT + TO_OUT, T2_O_E = T2_O_BM + TO_BM;
constexpr uint32_t T2_O_WCNT = T2_O_E + 8 * T2_ECAP, T2_O_WOUT = T2_O_WCNT + ((4 * T2_NWIN + 15) & ~15u);
constexpr uint32_t T2_O_WENT = T2_O_WOUT + ((4 * T2_NWIN + 15) & ~15u);
constexpr uint32_t T2_O_PASS = T2_O_WENT + ((2 * T2_NWIN + 15) & ~15u), T2_O_CTL = T2_O_PASS + 256;
constexpr uint32_t T2_LDS = T2_O_CTL + 64;
static_assert(T2_NWIN * 64 * 2 <= TO_OUT + TO_BM, "the exit table: the output area and the head of the bitmap");
static_assert(8 * T2_ECAP >= TD_TAB_WORDS * 4, "the record area holds the CRC tables afterwards");
static_assert(4 * T2_NWIN >= 2 * 1024, "the window counts' area holds the per-block start counts");
static_assert(T2_LDS <= 163840 && T2_O_OUT % 16 == 0 && T2_O_E % 16 == 0 && T2_O_PASS % 16 == 0, "k_ts_open2's LDS");
enum { T2_FAIL = 0, T2_NE = 1, T2_NOUT = 2, T2_CRC = 3, T2_DONE = 4, T2_TYPE = 5, T2_Q = 6, T2_AT = 7, T2_ULEN = 8,
       T2_WANT = 9, T2_OCLO = 10, T2_OCHI = 11, T2_OK = 12, T2_LEN = 13 };
constexpr uint32_t T2_FIN = 0x80000000u;  // scratch: the source is a literal input byte (else an output position)
#ifdef LCRC_PROBE_CLOCK  // diagnostic build: k_ts_open2's phase stamps (thread 0, s_memrealtime, 100 MHz)
#define T2_STAMP(i)                                                                                 \
  do {                                                                                              \
    if (threadIdx.x == 0 && blockIdx.x < 1024) {                                                    \
      __builtin_amdgcn_s_waitcnt(0);                                                                \
      lcrc_dbg_stamp[(3072 + blockIdx.x) * 8 + (i)] = __builtin_amdgcn_s_memrealtime();            \
    }                                                                                               \
  } while (0)
#else
#define T2_STAMP(i) \
  do {              \
  } while (0)
#endif

// the element that would start at in[i] (i < qe + 64: the staging's slack), as the wave decoder decodes it
struct SnCand {
  uint32_t typ, hdr, outlen, a, size;
  bool good;
};
__device__ __forceinline__ SnCand sn_cand(const lds_u8* in, uint32_t i, uint32_t qe) {
  SnCand c;
  const uint32_t t = in[i], b1 = in[i + 1], b2 = in[i + 2], b3 = in[i + 3], b4 = in[i + 4];
  c.typ = t & 3;
  const uint32_t room = qe > i ? qe - i : 0;
  if (c.typ == 0) {
    const uint32_t L = t >> 2;
    const uint32_t nb = L >= 60 ? L - 59 : 0;
    const uint32_t ext = b1 | (b2 << 8) | (b3 << 16) | (b4 << 24);
    const uint32_t lm1 = nb ? (nb == 4 ? ext : ext & ((1u << (8 * nb)) - 1)) : L;
    c.hdr = 1 + nb;
    c.outlen = lm1 + 1;
    c.a = i + c.hdr;
    c.good = room >= c.hdr && lm1 < room - c.hdr && (nb == 0 || room >= 5);  // (as snappy_wave_decode)
  } else {
    c.hdr = c.typ == 1 ? 2 : c.typ == 2 ? 3 : 5;
    c.outlen = c.typ == 1 ? 4 + ((t >> 2) & 7) : 1 + (t >> 2);
    c.a = c.typ == 1 ? ((t >> 5) << 8) | b1 : c.typ == 2 ? b1 | (b2 << 8) : b1 | (b2 << 8) | (b3 << 16) | (b4 << 24);
    c.good = room >= c.hdr;
  }
  c.size = c.typ == 0 ? c.hdr + c.outlen : c.hdr;
  return c;
}

// the chain of real element starts of a window from its entry (lanes >= lim: past the input's end)
__device__ __forceinline__ uint64_t sn_chain(uint32_t nxt, uint32_t en, uint32_t lim) {
  uint64_t mask = 0;
  uint32_t cur = en;
  while (cur < lim) {
    mask |= 1ull << cur;
    cur = (uint32_t)__builtin_amdgcn_readlane((int)nxt, (int)cur);
  }
  return mask;
}

// the value of 1 KiB pass k of the chunk CRC (td_chunk_crc's loop body): lane 0 of the wave gets it
template <bool FROM_LDS>
__device__ __forceinline__ uint32_t td_pass(const uint32_t* T, const uint8_t* src, uint32_t k, uint32_t pad, uint32_t q,
                                            uint32_t lane) {
  const uint32_t g = lane & 15;
  const uint32_t x0 = 1024 * k + 16 * lane;
  u32x4 w;
  if constexpr (FROM_LDS) {
    w = *(const u32x4*)(src + x0);
  } else {
    if (x0 >= pad) {
      w = *(const u32x4_ua*)(src + (x0 - pad));
    } else {
      w = u32x4{0, 0, 0, 0};
      if (x0 + 16 > pad)
        for (uint32_t b = pad - x0; b < 16; ++b) w[b >> 2] |= (uint32_t)src[x0 + b - pad] << (8 * (b & 3));
    }
  }
  w = td_inject(w, x0, pad, q);
  uint32_t cv = step4(T, 0u, w.x);
  cv = step4(T, cv, w.y);
  cv = step4(T, cv, w.z);
  cv = step4(T, cv, w.w);
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const uint32_t pn = row_down(cv, m);
    if ((g & ((2u << m) - 1)) == 0) cv = zl(T, TAB_ZPIECE + m * 1024, cv) ^ pn;
  }
  const uint32_t r0 = __builtin_amdgcn_readlane(cv, 0), r1 = __builtin_amdgcn_readlane(cv, 16);
  const uint32_t r2 = __builtin_amdgcn_readlane(cv, 32), r3 = __builtin_amdgcn_readlane(cv, 48);
  const uint32_t a = zl(T, TAB_ZWIN, r0) ^ r1, b = zl(T, TAB_ZWIN, r2) ^ r3;
  return zl(T, TAB_ZWIN + 1024, a) ^ b;
}

// the raw CRC-32C of a chunk (ulen bytes: V = 0^pad || M in LDS, or M in global memory), every wave its passes,
// thread 0 joining them (Z1024); needs the tables in T and every thread of the workgroup
template <bool FROM_LDS>
__device__ __forceinline__ uint32_t t2_chunk_crc(const uint32_t* T, const uint8_t* src, uint32_t ulen, uint32_t* passv,
                                                 uint32_t* ctl, uint32_t tid) {
  const uint32_t lane = tid & 63, wv = tid >> 6;
  const uint32_t np = (ulen + 1023) >> 10, pad = (np << 10) - ulen, q = ulen < 4 ? ulen : 4u;
  for (uint32_t k = wv; k < np; k += T2_WAVES) {
    const uint32_t v = td_pass<FROM_LDS>(T, src, k, pad, q, lane);
    if (lane == 0) passv[k] = v;
  }
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = np ? passv[0] : 0u;
    for (uint32_t k = 1; k < np; ++k) acc = zl(T, TAB_ZWIN + 2048, acc) ^ passv[k];
    if (ulen < 4) acc ^= ulen ? 0xFFFFFFFFu >> (8 * ulen) : 0xFFFFFFFFu;
    ctl[T2_CRC] = acc ^ 0xFFFFFFFFu;
  }
  __syncthreads();
  return ctl[T2_CRC];
}

// the chunk's elements in[q0, qe) decoded into o[0, ulen) by the whole workgroup (A-F above). 1 decoded, 0 malformed,
// 2 more elements than T2_ECAP. S: this workgroup's scratch (ulen words).
__device__ uint32_t sn_par_decode(const lds_u8* in, uint32_t q0, uint32_t qe, uint32_t ulen, uint8_t* L,
                                  uint16_t* __restrict__ S, uint8_t* __restrict__ dst, uint32_t tid) {
  typedef __attribute__((address_space(3))) uint32_t lds_u32;
  typedef __attribute__((address_space(3))) uint16_t lds_u16;
  lds_u16* const xt = (lds_u16*)(L + T2_O_OUT);
  lds_u32* const bm = (lds_u32*)(L + T2_O_BM);
  lds_u32* const ea = (lds_u32*)(L + T2_O_E);
  lds_u32* const eb = ea + T2_ECAP;
  lds_u32* const wcnt = (lds_u32*)(L + T2_O_WCNT);
  lds_u32* const wout = (lds_u32*)(L + T2_O_WOUT);
  lds_u16* const went = (lds_u16*)(L + T2_O_WENT);
  lds_u32* const ctl = (lds_u32*)(L + T2_O_CTL);
  // each window's chain of element starts (C), kept for E in the output area (the exit table's, dead after B)
  typedef __attribute__((address_space(3))) uint64_t lds_u64;
  lds_u64* const wmask = (lds_u64*)(L + T2_O_OUT);
  const uint32_t lane = tid & 63, wv = tid >> 6;
  const uint32_t nw = (qe - q0 + 63) >> 6;
  // A: exits
  for (uint32_t w = wv; w < nw; w += T2_WAVES) {
    const uint32_t base = q0 + 64 * w, lim = qe - base < 64 ? qe - base : 64u;
    const SnCand c = sn_cand(in, base + lane, qe);
    uint32_t p = lane >= lim ? lane : c.good ? lane + c.size : 0x7FFFu;
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const uint32_t pj = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((p < lim ? p : lane) * 4), (int)p);
      if (p < lim) p = pj;
    }
    xt[w * 64 + lane] = p == 0x7FFFu ? (uint16_t)0xFFFF : (uint16_t)(base + p);
  }
  if (tid == 0) ctl[T2_FAIL] = 0;
  __syncthreads();
  T2_STAMP(2);
  // B: entries, over super-windows of 16 windows (the serial walk over every window cost 40 us a chunk):
  //  B1: for each super-window and each entry offset e in its first window, the exit reached through its windows
  //      (lane e of a wave, 16 dependent LDS reads); the records area is free until E
  const uint32_t nsw = (nw + 15) >> 4;
  lds_u32* const swx = ea;
  lds_u32* const swent = ea + 64 * ((T2_NWIN + 15) / 16);
  for (uint32_t sw = wv; sw < nsw; sw += T2_WAVES) {
    uint32_t pos = q0 + 1024 * sw + lane;
    bool bad = false;
    const uint32_t wend = 16 * sw + 16 < nw ? 16 * sw + 16 : nw;
#pragma unroll 1
    for (uint32_t w = 16 * sw; w < wend; ++w) {
      const uint32_t base = q0 + 64 * w;
      if (!bad && pos < qe && pos < base + 64) {
        const uint32_t x = xt[w * 64 + (pos - base)];
        bad = x == 0xFFFFu;
        pos = bad ? pos : x;
      }
    }
    swx[sw * 64 + lane] = bad ? 0xFFFFFFFFu : pos;
  }
  __syncthreads();
  //  B2: thread 0 follows the chain from super-window to super-window (an entry past the first window -- a literal
  //      longer than 64 B crossing into it -- walks that super-window's windows one by one)
  if (tid == 0) {
    uint32_t pos = q0;
    bool bad = false;
    for (uint32_t sw = 0; sw < nsw; ++sw) {
      swent[sw] = pos;
      if (bad || pos >= qe) continue;
      const uint32_t b0 = q0 + 1024 * sw;
      if (pos < b0 + 64) {
        const uint32_t x = swx[sw * 64 + (pos - b0)];
        bad = x == 0xFFFFFFFFu;
        pos = bad ? pos : x;
      } else {
        const uint32_t wend = 16 * sw + 16 < nw ? 16 * sw + 16 : nw;
        for (uint32_t w = 16 * sw; w < wend && !bad; ++w) {
          const uint32_t base = q0 + 64 * w;
          if (pos < qe && pos < base + 64) {
            const uint32_t x = xt[w * 64 + (pos - base)];
            bad = x == 0xFFFFu;
            pos = bad ? pos : x;
          }
        }
      }
    }
    ctl[T2_FAIL] = bad || pos != qe;
  }
  __syncthreads();
  if (ctl[T2_FAIL]) return 0;
  //  B3: every window's entry, one thread per super-window walking its windows from the super-window's entry
  if (tid < nsw) {
    uint32_t pos = swent[tid];
    const uint32_t wend = 16 * tid + 16 < nw ? 16 * tid + 16 : nw;
#pragma unroll 1
    for (uint32_t w = 16 * tid; w < wend; ++w) {
      const uint32_t base = q0 + 64 * w;
      uint32_t en = 0xFFFFu;
      if (pos < qe && pos < base + 64) {
        en = pos - base;
        pos = xt[w * 64 + en];  // (a good chain: B2)
      }
      went[w] = (uint16_t)en;
    }
  }
  __syncthreads();
  T2_STAMP(3);
  // C: counts and output bytes per window
  for (uint32_t w = wv; w < nw; w += T2_WAVES) {
    const uint32_t en = went[w];
    uint32_t cnt = 0, out = 0;
    if (en != 0xFFFFu) {
      const uint32_t base = q0 + 64 * w, lim = qe - base < 64 ? qe - base : 64u;
      const SnCand c = sn_cand(in, base + lane, qe);
      const uint32_t nxt = c.good ? lane + c.size : 0x7FFFFFFFu;
      const uint64_t mask = sn_chain(nxt, en, lim);
      const bool sel = (mask >> lane) & 1;
      cnt = (uint32_t)__builtin_popcountll(mask);
      out = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(sel ? c.outlen : 0u, lane), 63);
      if (lane == 0) wmask[w] = mask;
    }
    if (lane == 0) {
      wcnt[w] = cnt;
      wout[w] = out;
    }
  }
  __syncthreads();
  // D: exclusive scans over the windows (wave 0: nine windows per lane)
  if (wv == 0) {
    uint32_t lane9 = lane * 9;
    __asm__ volatile("" : "+v"(lane9));  // (computed here: hoisted out of the chunk loop, its nine addresses spill)
    uint32_t sc = 0, so = 0;
    for (uint32_t j = 0; j < 9; ++j) {
      const uint32_t w = lane9 + j;
      if (w < nw) {
        sc += wcnt[w];
        so += wout[w];
      }
    }
    const uint32_t ic = wave_incl_scan(sc, lane), io = wave_incl_scan(so, lane);
    uint32_t ec = ic - sc, eo = io - so;
    for (uint32_t j = 0; j < 9; ++j) {
      const uint32_t w = lane9 + j;
      if (w < nw) {
        const uint32_t c = wcnt[w], u = wout[w];
        wcnt[w] = ec;
        wout[w] = eo;
        ec += c;
        eo += u;
      }
    }
    if (lane == 63) {
      ctl[T2_NE] = ic;
      ctl[T2_NOUT] = io;
    }
  }
  __syncthreads();
  if (ctl[T2_NOUT] != ulen) return 0;
  if (ctl[T2_NE] > T2_ECAP) return 2;
  // the start bitmap (its head held the end of the exit table), whole 64-bit blocks
  const uint32_t nblk = (ulen + 63) >> 6;
  for (uint32_t k = tid; k < 2 * nblk; k += T2_THREADS) bm[k] = 0;
  __syncthreads();
  // E: records and start bits
  for (uint32_t w = wv; w < nw; w += T2_WAVES) {
    const uint32_t en = went[w];
    if (en == 0xFFFFu) continue;
    const uint32_t base = q0 + 64 * w, lim = qe - base < 64 ? qe - base : 64u;
    const SnCand c = sn_cand(in, base + lane, qe);
    const uint64_t mask = wmask[w];  // (C's chain)
    (void)lim;
    const bool sel = (mask >> lane) & 1;
    const uint32_t v = sel ? c.outlen : 0u;
    const uint32_t wpos = wout[w] + wave_incl_scan(v, lane) - v;
    const bool bad = sel && (wpos > ulen || c.outlen > ulen - wpos || (c.typ != 0 && (c.a == 0 || c.a > wpos)));
    if (__builtin_amdgcn_ballot_w64(bad)) {
      if (lane == 0) ctl[T2_FAIL] = 1;
      continue;
    }
    if (sel) {
      const uint32_t k = wcnt[w] + (uint32_t)__builtin_popcountll(mask & ((1ull << lane) - 1));
      ea[k] = wpos | ((c.outlen - 1) << 16);  // (wpos < ulen <= 65536, outlen <= 65536)
      eb[k] = c.typ == 0 ? (c.a | T2_FIN) : c.a;
      __hip_atomic_fetch_or((uint32_t*)&bm[wpos >> 5], 1u << (wpos & 31), __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  __syncthreads();
  if (ctl[T2_FAIL]) return 0;
  // F1: element starts before each 64-byte block (one thread per block; the counts' area reused)
  lds_u16* const bpre = (lds_u16*)wcnt;
  {
    const uint32_t b = tid;
    const uint32_t c = b < nblk ? (uint32_t)(__builtin_popcount(bm[2 * b]) + __builtin_popcount(bm[2 * b + 1])) : 0u;
    const uint32_t inc = wave_incl_scan(c, lane);
    if (lane == 63) wout[wv] = inc;  // the waves' totals (wout is free)
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t k = 0; k < wv; ++k) before += wout[k];
    __syncthreads();
    if (b < nblk) bpre[b] = (uint16_t)(before + inc - c);
  }
  __syncthreads();
  T2_STAMP(4);
  // F2: every output byte's source: a literal's byte is written to dst at once and is its own source (a root); a
  // copy's byte points at an earlier output position. The sources (16-bit: ulen <= 65536) go to the global scratch
  // first: the LDS still holds the input, the bitmap and the records this pass reads
  uint64_t todo = 0;
#pragma unroll 1  // (unrolled, the 64 per-thread addresses are hoisted out of the chunk loop and spill)
  for (uint32_t i = 0; i < 64; ++i) {
    const uint32_t x = tid + T2_THREADS * i;
    if (x >= ulen) break;
    const uint32_t b = x >> 6, l = x & 63;
    const uint64_t m = ((uint64_t)bm[2 * b + 1] << 32) | bm[2 * b];
    const uint32_t e = bpre[b] + (uint32_t)__builtin_popcountll(m & ((2ull << l) - 1)) - 1;
    const uint32_t A = ea[e], B = eb[e];
    const uint32_t ew = A & 0xFFFFu, elen = (A >> 16) + 1, off = x - ew;
    uint32_t src = x;
    if (B & T2_FIN) {
      dst[x] = in[(B & ~T2_FIN) + off];
    } else {
      const uint32_t per = B < elen ? B : 0u;  // (a copy is at most 64 bytes long: off < 64)
      src = per ? ew - B + small_mod(off, per) : x - B;
      todo |= 1ull << i;
    }
    S[x] = (uint16_t)src;
  }
  __syncthreads();
  // F3: the sources into the LDS (its first 128 KiB: input, output staging, bitmap and records are dead), then
  // pointer jumping there (S[x] <- S[S[x]]) until every copy byte points at a root. A copy of a copy of a copy -- an
  // index block's keys -- converges in log2 of its chain's length rounds; each round costs two LDS latencies per 16
  // positions instead of two global-memory latencies per 8 (round 4's scratch walk: 130 us a chunk)
  lds_u16* const S16 = (lds_u16*)L;
  for (uint32_t x = 8 * tid; x < ulen; x += 8 * T2_THREADS) *(__attribute__((address_space(3))) u32x4*)(S16 + x) =
      *(const u32x4*)(S + x);
  const uint64_t copies = todo;
  __syncthreads();
  T2_STAMP(5);
  while (__syncthreads_or(todo != 0)) {
#pragma unroll 1
    for (uint32_t i0 = 0; i0 < 64; i0 += 16) {
      if (!((todo >> i0) & 0xFFFF)) continue;
      uint32_t v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = ((todo >> (i0 + j)) & 1) ? S16[tid + T2_THREADS * (i0 + j)] : 0u;
      uint32_t u[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) u[j] = ((todo >> (i0 + j)) & 1) ? S16[v[j]] : 0u;
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if ((todo >> (i0 + j)) & 1) {
          if (u[j] == v[j]) todo &= ~(1ull << (i0 + j));  // v is a root: a literal byte
          else S16[tid + T2_THREADS * (i0 + j)] = (uint16_t)u[j];
        }
    }
  }
  T2_STAMP(6);
  // F4: the copy bytes gathered from their roots in dst (written by F2, before the barriers)
#pragma unroll 1
  for (uint32_t i0 = 0; i0 < 64; i0 += 16) {
    if (!((copies >> i0) & 0xFFFF)) continue;
    uint32_t v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = ((copies >> (i0 + j)) & 1) ? dst[S16[tid + T2_THREADS * (i0 + j)]] : 0u;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if ((copies >> (i0 + j)) & 1) dst[tid + T2_THREADS * (i0 + j)] = (uint8_t)v[j];
  }
  __threadfence_block();
  __syncthreads();
  return 1;
}

__global__ void __launch_bounds__(T2_THREADS) k_ts_open2(const uint8_t* __restrict__ file, uint64_t file_len,
                                                        const uint32_t* __restrict__ tab_c, uint8_t* __restrict__ idec,
                                                        uint64_t idec_cap, uint64_t* __restrict__ iopen,
                                                        uint32_t* __restrict__ scratch) {
  extern __shared__ __attribute__((aligned(16))) uint8_t t2_lds[];
  typedef __attribute__((address_space(3))) uint32_t lds_u32;
  uint8_t* const lin = t2_lds + T2_O_IN;
  uint8_t* const lout = t2_lds + T2_O_OUT;
  uint32_t* const T = (uint32_t*)(t2_lds + T2_O_E);
  uint32_t* const passv = (uint32_t*)(t2_lds + T2_O_PASS);
  lds_u32* const ctl = (lds_u32*)(t2_lds + T2_O_CTL);
  uint16_t* const S = (uint16_t*)(scratch + (uint64_t)blockIdx.x * 65536);
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  // the footer's index handle, by wave 0
  if (tid < 64) {
    uint64_t io = 0, is = 0;
    bool framed = false;
    if (file_len >= 48) {
      const uint8_t* f = file + file_len - 48;
      const uint64_t magic = (uint64_t)load_le32(f + 40) | ((uint64_t)load_le32(f + 44) << 32);
      uint64_t mo, ms;
      uint32_t p = magic == 0xdb4775248b80fb57ull ? dev_varint<64>(f, 0, 48, &mo) : ~0u;
      if (p != ~0u) p = dev_varint<64>(f, p, 48, &ms);
      if (p != ~0u) p = dev_varint<64>(f, p, 48, &io);
      if (p != ~0u) p = dev_varint<64>(f, p, 48, &is);
      framed = p != ~0u && io <= file_len && is + 5 <= file_len - io && is + 1 <= 0x7FFFFFFFull && file[io + is] == 1;
    }
    if (lane == 0) {
      ctl[T2_OK] = framed;
      ctl[T2_OCLO] = (uint32_t)io;
      ctl[T2_OCHI] = (uint32_t)(io >> 32);
      ctl[T2_LEN] = (uint32_t)is;
    }
  }
  __syncthreads();
  const bool framed = ctl[T2_OK] != 0;
  const uint8_t* const p = file + ((uint64_t)ctl[T2_OCHI] << 32 | ctl[T2_OCLO]);
  const uint32_t len = ctl[T2_LEN];
  // the frame's verdict (snap's framing walk: sizes, types, preambles) by the last workgroup's wave 1 -- the only walk
  // over the whole frame; the others find their own chunks without it (their decode is only used when it says so)
  if (blockIdx.x == gridDim.x - 1 && tid >= 64 && tid < 128) {
    uint64_t total = 0, chunks = 0, padded;
    uint32_t mi, mo;
    const bool ok = framed && snappy_frame_size(p, len, total, chunks, mi, mo, padded);
    const bool fits = total <= idec_cap;
    if (lane == 0) {
      iopen[1] = ok ? total : 0;
      iopen[0] = (framed ? 1u : 0u) | (ok && fits ? 2u : 0u) | (ok && !fits ? 4u : 0u);
    }
  }
  if (!framed) return;  // (uniform)
  T2_STAMP(0);
  // wave 0's walk to this workgroup's chunks (k % gridDim == blockIdx): each hop's header, stored CRC and preamble
  // (20 bytes) loaded by 20 lanes at once and read with v_readlane -- one memory latency a hop. Bounded by the frame:
  // a malformed frame ends the walk (its verdict is the last workgroup's)
  uint32_t at = 0, k = 0;  // (wave 0)
  uint64_t o = 0;
  bool good = true;  // (thread 0)
  while (true) {
    __syncthreads();
    if (tid < 64) {
      uint32_t done = 1;
      while (at < len && len - at >= 4) {
        const uint32_t bv = lane < 20 && lane < len - at ? ld_u8(p + at + lane) : 0u;
        auto B = [&](uint32_t i) { return (uint32_t)__builtin_amdgcn_readlane((int)bv, (int)i); };
        const uint32_t type = B(0), cl = B(1) | (B(2) << 8) | (B(3) << 16);
        const uint32_t body = at + 4;
        if (cl > len - body || cl > SN_MAX_CHUNK) break;
        at = body + cl;
        if (type > 1) continue;
        if (cl < 4) break;
        uint32_t ulen = cl - 4, q = body + 4, used = 0;
        if (type == 0) {
          if (!snappy_preamble([&](uint32_t i) { return B(8 + i); }, cl - 4, ulen, used)) break;
          q += used;
        }
        const uint64_t oc = o;
        o += ulen;
        if (k++ % gridDim.x != blockIdx.x || oc + ulen > idec_cap) continue;  // (over the workspace: verdict 4)
        if (lane == 0) {
          ctl[T2_TYPE] = type;
          ctl[T2_Q] = q;
          ctl[T2_AT] = at;
          ctl[T2_ULEN] = ulen;
          ctl[T2_WANT] = B(4) | (B(5) << 8) | (B(6) << 16) | (B(7) << 24);
          ctl[T2_OCLO] = (uint32_t)oc;
          ctl[T2_OCHI] = (uint32_t)(oc >> 32);
        }
        done = 0;
        break;
      }
      if (lane == 0) ctl[T2_DONE] = done;
    }
    __syncthreads();
    if (ctl[T2_DONE]) break;
    const uint32_t type = ctl[T2_TYPE], q = ctl[T2_Q], ae = ctl[T2_AT], ulen = ctl[T2_ULEN], want = ctl[T2_WANT];
    const uint64_t oc = (uint64_t)ctl[T2_OCHI] << 32 | ctl[T2_OCLO];
    const uint32_t pad = ((ulen + 1023) & ~1023u) - ulen;
    uint32_t crc = 0;
    bool cok = true;
    if (type == 1) {  // uncompressed: checksummed where it lies, copied out
      stage_to_lds(tab_c, (lds_u8*)(uint8_t*)T, TD_TAB_WORDS, tid, T2_THREADS);
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      crc = t2_chunk_crc<false>(T, p + q, ulen, passv, (uint32_t*)ctl, tid);
      for (uint32_t x = tid; x < ulen; x += T2_THREADS) idec[oc + x] = p[q + x];
    } else if (ae - q + 4 > TO_IN) {  // too large for the staging: lane-serial in the workspace, checksummed there
      if (tid == 0) {
        uint64_t oo = oc;
        ctl[T2_FAIL] = !sn_serial_decode(p + q, p + ae, idec, oo, oc + ulen);
      }
      __threadfence_block();
      __syncthreads();
      cok = !ctl[T2_FAIL];
      stage_to_lds(tab_c, (lds_u8*)(uint8_t*)T, TD_TAB_WORDS, tid, T2_THREADS);
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      if (cok) crc = t2_chunk_crc<false>(T, idec + oc, ulen, passv, (uint32_t*)ctl, tid);
    } else {
      const uint8_t* zs = p + q;
      const uint32_t d = (uint32_t)((uintptr_t)zs & 3);
      const uint32_t ndw = (d + (ae - q) + 3) >> 2;
      stage_to_lds((const uint32_t*)(zs - d), (lds_u8*)lin, ndw, tid, T2_THREADS);
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      T2_STAMP(1);
      const uint32_t r = sn_par_decode((const lds_u8*)lin, d, d + (ae - q), ulen, t2_lds, S, idec + oc, tid);
      if (r == 2) {  // more elements than the records hold: the wave decoder, on wave 0, in the LDS staging
        if (tid < 64) {
          const bool w_ok = snappy_wave_decode(lin, d, d + (ae - q), lout + pad, ulen, lane);
          if (lane == 0) ctl[T2_FAIL] = !w_ok;
        }
        __syncthreads();
        cok = !ctl[T2_FAIL];
        if (cok) {
          // V[0, pad) zeroed for the CRC passes -- exactly: the output starts at pad, which need not be 16-aligned
          for (uint32_t x = 16 * tid; x < pad; x += 16 * T2_THREADS) {
            if (x + 16 <= pad) {
              *(u32x4*)(lout + x) = u32x4{0, 0, 0, 0};
            } else {
              for (uint32_t b = x; b < pad; ++b) lout[b] = 0;
            }
          }
          stage_to_lds(tab_c, (lds_u8*)(uint8_t*)T, TD_TAB_WORDS, tid, T2_THREADS);
          __builtin_amdgcn_s_waitcnt(0);
          __syncthreads();
          crc = t2_chunk_crc<true>(T, lout, ulen, passv, (uint32_t*)ctl, tid);
          const uint8_t* src = lout + pad;
          uint32_t x0 = 0;
          if (((oc | pad) & 15) == 0) {  // whole 16 B pieces, then the tail byte by byte
            x0 = ulen & ~15u;
            for (uint32_t x = 16 * tid; x < x0; x += 16 * T2_THREADS) *(u32x4*)(idec + oc + x) = *(const u32x4*)(src + x);
          }
          for (uint32_t x = x0 + tid; x < ulen; x += T2_THREADS) idec[oc + x] = src[x];
        }
      } else {
        cok = r == 1;
        if (cok) {  // decoded into the workspace: checksummed there
          stage_to_lds(tab_c, (lds_u8*)(uint8_t*)T, TD_TAB_WORDS, tid, T2_THREADS);
          __builtin_amdgcn_s_waitcnt(0);
          __syncthreads();
          crc = t2_chunk_crc<false>(T, idec + oc, ulen, passv, (uint32_t*)ctl, tid);
        }
      }
    }
    T2_STAMP(7);
    if (tid == 0) good = good && cok && mask32c(crc) == want;
    __builtin_amdgcn_s_waitcnt(0);
  }
  if (tid == 0 && !good) iopen[2] = 1;  // (every writer stores the same 1)
}
}  // namespace lcrc_dev

// ---------------------------------------------------------------------------------------------------
// host-side launchers (called from lcrc_api.cpp)
// ---------------------------------------------------------------------------------------------------
// Kernel-carried timing for every launcher (lcrc_timer_kernels on the general path, the WAL and table scans):
// while an API call of a timed context runs (TkScope, lcrc_api.cpp), its launches carry the context's events --
// the first launch records the start at its own start, every launch the stop at its end (the last one wins) --
// through hipExtLaunchKernelGGL, so no marker packet sits between launches.
thread_local hipEvent_t lcrc_tl_ev_start = nullptr, lcrc_tl_ev_stop = nullptr;
thread_local bool lcrc_tl_ev_started = false, lcrc_tl_ev_stopped = false;
#define LCRC_LAUNCH(kern, grid, block, shmem, st, ...)                                                       \
  do {                                                                                                       \
    hipEvent_t ev_s_ = lcrc_tl_ev_start, ev_e_ = lcrc_tl_ev_stop;                                            \
    if (ev_s_ || ev_e_) {                                                                                    \
      hipExtLaunchKernelGGL(kern, grid, block, shmem, st, ev_s_, ev_e_, 0, __VA_ARGS__);                    \
      if (ev_s_) lcrc_tl_ev_started = true;                                                                  \
      if (ev_e_) lcrc_tl_ev_stopped = true;                                                                  \
      lcrc_tl_ev_start = nullptr;                                                                            \
    } else {                                                                                                 \
      hipLaunchKernelGGL(kern, grid, block, shmem, st, __VA_ARGS__);                                         \
    }                                                                                                        \
  } while (0)

extern "C" {

// the calling thread's launches carry (start, stop) until lcrc_launch_events_end; returns nothing
void lcrc_launch_events_begin(hipEvent_t start, hipEvent_t stop) {
  lcrc_tl_ev_start = start;
  lcrc_tl_ev_stop = stop;
  lcrc_tl_ev_started = lcrc_tl_ev_stopped = false;
}
// the stop event the launches carry, replaced by `ev` (nullptr: none); returns the previous one. A call whose
// launches fork over several streams takes it away from them and records it after the join itself
// (lcrc_launch_events_record_stop): the last launch issued need not be the last to end.
hipEvent_t lcrc_launch_events_swap_stop(hipEvent_t ev) {
  hipEvent_t old = lcrc_tl_ev_stop;
  lcrc_tl_ev_stop = ev;
  return old;
}
hipError_t lcrc_launch_events_record_stop(hipEvent_t ev, hipStream_t st) {
  hipError_t e = hipEventRecord(ev, st);
  if (e == hipSuccess) lcrc_tl_ev_stopped = true;
  return e;
}
// clears them; *started / *stopped: whether a launch recorded the start / the stop
void lcrc_launch_events_end(bool* started, bool* stopped) {
  *started = lcrc_tl_ev_started;
  *stopped = lcrc_tl_ev_stopped;
  lcrc_tl_ev_start = lcrc_tl_ev_stop = nullptr;
  lcrc_tl_ev_started = lcrc_tl_ev_stopped = false;
}

#ifdef LCRC_PROBE_CLOCK
// effective shader clock (MHz) of the last k_windows launch: median over workgroups of
// d(s_memtime) / d(s_memrealtime) * 100 MHz
// raw per-wave s_memrealtime stamps (100 MHz) of the last k_windows launch: entry, tables ready,
// first half-tile walked, end
int lcrc_probe_stamps(unsigned long long* dst) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(lcrc_dev::lcrc_dbg_stamp), sizeof(unsigned long long) * 4096 * 8) ==
                 hipSuccess ? 0 : -1;
}

int lcrc_probe_bstamps(unsigned long long* dst) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(lcrc_dev::lcrc_dbg_bstamp), sizeof(unsigned long long) * 8192 * 8) ==
                 hipSuccess ? 0 : -1;
}

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

// t_start / t_stop (nullable, final mode): events recorded by the dispatch itself, as in lcrc_launch_windows_queue
hipError_t lcrc_launch_windows(bool final_mode, int grid, const uint8_t* base, uint64_t span, const uint32_t* gtab,
                               uint32_t* out, uint64_t nblk, uint32_t fin, uint32_t flags,
                               const uint32_t* expected, uint32_t* mismatch, hipStream_t st, hipEvent_t t_start,
                               hipEvent_t t_stop) {
  const uint64_t nreg = (span + lcrc_dev::REGION - 1) / lcrc_dev::REGION;
  if (nreg == 0) return hipSuccess;
  grid *= lcrc_dev::A_WG_PER_CU;  // `grid` = CUs
  uint64_t need = (nreg + lcrc_dev::A_THREADS / 64 - 1) / (lcrc_dev::A_THREADS / 64);
  int g = (int)(need < (uint64_t)grid ? need : (uint64_t)grid);
  if (final_mode && (t_start || t_stop))
    hipExtLaunchKernelGGL(lcrc_dev::k_windows<true>, dim3(g), dim3(lcrc_dev::A_THREADS), 0, st, t_start, t_stop, 0,
                          base, span, nreg, gtab, out, nblk, fin, flags, expected, mismatch);
  else if (final_mode)
    LCRC_LAUNCH(lcrc_dev::k_windows<true>, dim3(g), dim3(lcrc_dev::A_THREADS), 0, st, base, span, nreg, gtab,
                       out, nblk, fin, flags, expected, mismatch);
  else
    LCRC_LAUNCH(lcrc_dev::k_windows<false>, dim3(g), dim3(lcrc_dev::A_THREADS), 0, st, base, span, nreg,
                       gtab, out, nblk, fin, flags, expected, mismatch);
  return hipGetLastError();
}

// A queue of uniform 4 KiB batches (lcrc_batch_uniform_queue), at most MAX_QJOBS per launch: jobs[k] =
// {base, out, expected, mismatch, nblk} (host array, copied into the kernel arguments).
// t_start / t_stop (nullable): events recorded by the dispatch itself (hipExtLaunchKernelGGL: the kernel's own
// start and end, no marker packet between launches)
hipError_t lcrc_launch_windows_queue(int grid, const lcrc_qjob_host* jobs, uint32_t njobs, const uint32_t* gtab,
                                     uint32_t fin, uint32_t flags, hipStream_t st, hipEvent_t t_start,
                                     hipEvent_t t_stop) {
  using lcrc_dev::QJobsArg;
  if (njobs == 0 || njobs > (uint32_t)lcrc_dev::MAX_QJOBS) return njobs ? hipErrorInvalidValue : hipSuccess;
  QJobsArg a;
  memset(&a, 0, sizeof(a));
  uint64_t reg = 0;
  uint32_t n = 0;
  for (uint32_t k = 0; k < njobs; ++k) {
    if (jobs[k].nblk == 0) continue;
    a.j[n].base = jobs[k].base;
    a.j[n].out = jobs[k].out;
    a.j[n].expected = jobs[k].expected;
    a.j[n].mismatch = jobs[k].mismatch;
    a.j[n].nblk = jobs[k].nblk;
    a.j[n].reg0 = reg;
    reg += (jobs[k].nblk * 4096 + lcrc_dev::REGION - 1) / lcrc_dev::REGION;
    ++n;
  }
  if (n == 0) return hipSuccess;
  a.n = n;
  a.nreg = reg;
  grid *= lcrc_dev::A_WG_PER_CU;
  const uint64_t need = (reg + lcrc_dev::A_THREADS / 64 - 1) / (lcrc_dev::A_THREADS / 64);
  const int g = (int)(need < (uint64_t)grid ? need : (uint64_t)grid);
  if (t_start || t_stop)
    hipExtLaunchKernelGGL(lcrc_dev::k_windows_q, dim3(g), dim3(lcrc_dev::A_THREADS), 0, st, t_start, t_stop, 0, a, gtab,
                          fin, flags);
  else
    LCRC_LAUNCH(lcrc_dev::k_windows_q, dim3(g), dim3(lcrc_dev::A_THREADS), 0, st, a, gtab, fin, flags);
  return hipGetLastError();
}

// ---- asynchronous table scan (lcrc_table_scan_async) ----
// grid: a bound on the restart segments (the workgroups past the device count only zero their share)
// gcap: the most workgroups (the rest of the tiles grid-stride)
// a Snappy-framed index block decoded into idec (k_ts_open2); scratch: T2_GRID x 65,536 words (its pointer-jumping
// sources)
hipError_t lcrc_launch_ts_open(const uint8_t* file, uint64_t file_len, const uint32_t* tab_c, uint8_t* idec,
                               uint64_t idec_cap, uint64_t* iopen, uint32_t* scratch, hipStream_t s) {
  static const hipError_t attr2 = hipFuncSetAttribute((const void*)lcrc_dev::k_ts_open2,
                                                      hipFuncAttributeMaxDynamicSharedMemorySize, lcrc_dev::T2_LDS);
  if (attr2 != hipSuccess) return attr2;
  LCRC_LAUNCH(lcrc_dev::k_ts_open2, dim3(lcrc_dev::T2_GRID), dim3(lcrc_dev::T2_THREADS), lcrc_dev::T2_LDS, s, file,
              file_len, tab_c, idec, idec_cap, iopen, scratch);
  return hipGetLastError();
}
uint64_t lcrc_ts_open_scratch_words() { return (uint64_t)lcrc_dev::T2_GRID * 65536; }
// the table scan's index walk and handles (k_ts_windows' index workgroups), with the file's window pass beside them
// when `windows` (grid = CUs; without it the index workgroups alone: the one-pass general path, or no result
// capacity). nidx_cap: the index workgroups' cap (lcrc_ctx_options.ts_grid); agg: TSA_MAX + 1 words, zero
hipError_t lcrc_launch_ts_windows(int grid, bool windows, const uint8_t* file, uint64_t file_len, const uint32_t* gtab,
                                  uint32_t* win, const lcrc_tscan_key* key, uint64_t cap, uint64_t vcap,
                                  lcrc_tscan_dev* st, uint64_t* local_c, uint32_t* zero, uint64_t nzero,
                                  const uint8_t* idec, const uint64_t* iopen_r, uint64_t* iopen, lcrc_tblk_dev* out,
                                  lcrc_desc_dev* descs, uint64_t* agg, uint32_t nidx_cap, hipStream_t s) {
  const uint64_t nreg = (file_len + lcrc_dev::REGION - 1) / lcrc_dev::REGION;
  const uint64_t need = (nreg + lcrc_dev::A_THREADS / 64 - 1) / (lcrc_dev::A_THREADS / 64);
  const uint64_t gw = (uint64_t)grid * lcrc_dev::A_WG_PER_CU;
  const uint32_t nwg = windows ? (uint32_t)(need < gw ? need : gw) : 0u;
  // one index workgroup per 512 restart segments (a segment names at least one block), at most one per CU
  uint64_t nidx = cap / lcrc_dev::A_THREADS + 1;
  if (nidx > nidx_cap) nidx = nidx_cap;
  if (nidx > (uint64_t)grid) nidx = (uint64_t)grid;
  if (nidx > lcrc_dev::TSA_MAX) nidx = lcrc_dev::TSA_MAX;
  if (nidx == 0) nidx = 1;
  lcrc_dev::TsIdxArgs ia{file, file_len, cap, cap, vcap, nzero, st, local_c, zero, idec, iopen_r, iopen, out, descs, agg};
  LCRC_LAUNCH(lcrc_dev::k_ts_windows, dim3((unsigned)(nwg + nidx)), dim3(lcrc_dev::A_THREADS), 0, s, file, file_len,
              nreg, gtab, win, nwg, *key, ia);
  return hipGetLastError();
}
hipError_t lcrc_launch_ts_finish(lcrc_tblk_dev* blk, uint64_t n, const uint32_t* crc, const uint32_t* mismatch,
                                 const uint8_t* file, lcrc_desc_dev* frames, uint64_t* out_off, uint64_t* choff,
                                 uint64_t* part, uint64_t* nchunks, uint8_t* fstatus, lcrc_tscan_dev* st,
                                 const uint32_t* gtab, uint32_t flags, hipStream_t s) {
  if (n == 0) return hipSuccess;
  LCRC_LAUNCH(lcrc_dev::k_ts_finish, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, blk, n, crc, mismatch,
              file, frames, out_off, choff, part, nchunks, fstatus, st, gtab, flags);
  return hipGetLastError();
}
// grid: a bound on the blocks

// the table scan's decode, chunk checks and close in one launch (k_ts_decode); bound: the result capacity
hipError_t lcrc_launch_ts_decode(const uint8_t* file, const lcrc_desc_dev* frames, const uint64_t* out_off, uint8_t* out,
                                 const uint8_t* fstatus, lcrc_tscan_dev* st, lcrc_tblk_dev* blk, const uint32_t* tab_c,
                                 uint64_t ts_out_cap, const uint64_t* tparts, uint64_t bound, uint64_t* n_out,
                                 uint32_t* status_out, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute((const void*)lcrc_dev::k_ts_decode,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, lcrc_dev::TD_LDS);
  if (attr != hipSuccess) return attr;
  const uint64_t g = (bound + 255) / 256 * lcrc_dev::TD_SUB;
  LCRC_LAUNCH(lcrc_dev::k_ts_decode, dim3((unsigned)(g ? g : 1)), dim3(64 * lcrc_dev::TD_WAVES), lcrc_dev::TD_LDS, s,
              file, frames, out_off, out, fstatus, st, blk, tab_c, ts_out_cap, tparts, n_out, status_out, bound);
  return hipGetLastError();
}

// k_blocks workgroups resident per CU (by its LDS image)
int lcrc_blocks_per_cu() {
  const int by_lds = 163840 / (lcrc_dev::B_LDS_DWORDS * 4);
  return by_lds < 4 ? by_lds : 4;
}

// n_dev (device, nullable): the actual count when it is only known on the device; n is then a bound
hipError_t lcrc_launch_blocks(bool uniform, int grid, const uint8_t* base, uint64_t base_len,
                              const lcrc_desc_dev* descs, uint64_t n, uint64_t ustride, uint32_t ulen,
                              const uint32_t* uexp, const uint32_t* win, const uint32_t* gtab, uint32_t init,
                              uint32_t xorout, uint32_t flags, uint32_t* out, uint32_t* mismatch,
                              const uint64_t* n_dev, lcrc_wal_rec_dev* recs, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const uint64_t per_wg = lcrc_dev::B_THREADS / 16;  // one range per 16-lane row
  uint64_t need = (n + per_wg - 1) / per_wg;
  int g = (int)(need < (uint64_t)grid ? need : (uint64_t)grid);
  if (uniform)
    LCRC_LAUNCH(lcrc_dev::k_blocks<true>, dim3(g), dim3(lcrc_dev::B_THREADS), 0, st, base, base_len, descs, n,
                       ustride, ulen, uexp, win, gtab, init, xorout, flags, out, mismatch, n_dev, recs);
  else
    LCRC_LAUNCH(lcrc_dev::k_blocks<false>, dim3(g), dim3(lcrc_dev::B_THREADS), 0, st, base, base_len, descs,
                       n, ustride, ulen, uexp, win, gtab, init, xorout, flags, out, mismatch, n_dev, recs);
  return hipGetLastError();
}

// general ranges in one pass (k_ranges); `grid` = CUs. inv: 4097 words x^(-8k) mod P (TAB_INV)
hipError_t lcrc_launch_ranges(bool uniform, int grid, const uint8_t* base, uint64_t base_len,
                              const lcrc_desc_dev* descs, uint64_t n, uint64_t ustride, uint32_t ulen,
                              const uint32_t* uexp, const uint32_t* gtab, uint32_t x4096, uint32_t poly,
                              uint32_t init, uint32_t xorout, uint32_t flags, uint32_t* out, uint32_t* mismatch,
                              const uint64_t* n_dev, lcrc_wal_rec_dev* recs, hipStream_t st, uint32_t rows_per_wg) {
  if (n == 0) return hipSuccess;
  grid *= lcrc_dev::R_WG_PER_CU;
  const uint64_t per_wg = rows_per_wg;  // ranges dealt per workgroup in the first round (32 rows: all of them)
  const uint64_t need = (n + per_wg - 1) / per_wg;
  const int g = (int)(need < (uint64_t)grid ? need : (uint64_t)grid);
  const uint32_t* inv = gtab + TAB_INV;
  if (uniform)
    LCRC_LAUNCH(lcrc_dev::k_ranges<true>, dim3(g), dim3(lcrc_dev::A_THREADS), 0, st, base, base_len, descs, n,
                       ustride, ulen, uexp, gtab, inv, x4096, poly, init, xorout, flags, out, mismatch, n_dev, recs);
  else
    LCRC_LAUNCH(lcrc_dev::k_ranges<false>, dim3(g), dim3(lcrc_dev::A_THREADS), 0, st, base, base_len, descs,
                       n, ustride, ulen, uexp, gtab, inv, x4096, poly, init, xorout, flags, out, mismatch, n_dev, recs);
  return hipGetLastError();
}

// n_total (device): the record count for k_blocks; n_out (device or pinned host, nullable): the same for
// the caller
hipError_t lcrc_launch_wal_parse(const uint8_t* file, uint64_t file_len, uint64_t nblocks, uint32_t* counts,
                                 uint2* slots, uint8_t* stops, uint64_t* local, uint64_t* part,
                                 lcrc_wal_rec_dev* recs, lcrc_desc_dev* descs, uint64_t max_recs, uint64_t* n_total,
                                 uint64_t* n_out, hipStream_t st) {
  const uint64_t nparts = (nblocks + lcrc_dev::WAL_PARTB - 1) / lcrc_dev::WAL_PARTB;
  if (nparts)
    LCRC_LAUNCH(lcrc_dev::k_wal_parse, dim3((unsigned)nparts), dim3(64), 0, st, file, file_len, nblocks,
                counts, slots, stops, local, part);
  const uint64_t nt = nblocks * lcrc_dev::WAL_SLOTS;
  const uint64_t g = (nt + 255) / 256;
  LCRC_LAUNCH(lcrc_dev::k_wal_emit, dim3((unsigned)(g ? g : 1)), dim3(256), 0, st, file, nblocks, counts, slots,
                     stops, local, part, recs, descs, max_recs, n_total, n_out);
  return hipGetLastError();
}

// several logs' header walks and record emits, two launches (lcrc_wal_scan_queue); m <= MAX_WJOBS
hipError_t lcrc_launch_wal_parse_queue(const lcrc_wjob_dev_host* jobs, uint32_t m, hipStream_t st) {
  using lcrc_dev::WalJobsArg;
  if (m == 0) return hipSuccess;
  if (m > (uint32_t)lcrc_dev::MAX_WJOBS) return hipErrorInvalidValue;
  WalJobsArg a;
  memset(&a, 0, sizeof(a));
  uint64_t gp = 1, ge = 1;
  for (uint32_t k = 0; k < m; ++k) {
    const lcrc_wjob_dev_host& j = jobs[k];
    a.j[k] = lcrc_dev::WalJobDev{j.file, j.file_len, j.nblocks, j.counts, j.slots, j.stops, j.local, j.part,
                                 j.recs, j.descs, j.max_recs, j.n_total, j.n_out};
    gp = std::max<uint64_t>(gp, (j.nblocks + lcrc_dev::WAL_PARTB - 1) / lcrc_dev::WAL_PARTB);
    ge = std::max<uint64_t>(ge, (j.nblocks * lcrc_dev::WAL_SLOTS + 255) / 256);
  }
  LCRC_LAUNCH(lcrc_dev::k_wal_parse_q, dim3((unsigned)gp, m), dim3(64), 0, st, a);
  LCRC_LAUNCH(lcrc_dev::k_wal_emit_q, dim3((unsigned)ge, m), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t lcrc_launch_snappy_size(const uint8_t* base, const lcrc_desc_dev* frames, uint64_t n, uint64_t* size,
                                   uint64_t* nchunks, uint8_t* status, uint32_t* maxes, const uint64_t* n_dev,
                                   hipStream_t st) {
  if (n == 0) return hipSuccess;
  LCRC_LAUNCH(lcrc_dev::k_snappy_size, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, base, frames, n, size,
                     nchunks, status, maxes, n_dev);
  return hipGetLastError();
}

// out_a / out_b: n + 1 entries (exclusive scans, totals at [n]); part: 2 * ceil(n / 256) scratch words
// n_dev (nullable): the count produced on the device, n is then its bound (the grid is sized by n + 1)
// the second half of lcrc_launch_scan2, after a kernel that scanned within its 256-entry workgroups
hipError_t lcrc_launch_scan2_add(uint64_t n, uint64_t* out_a, uint64_t* out_b, const uint64_t* part,
                                 const uint64_t* n_dev, hipStream_t st) {
  const uint64_t g = n_dev ? n / 256 + 1 : (n + 255) / 256;
  if (g == 0) return hipMemsetAsync(out_a, 0, 8, st) == hipSuccess ? hipMemsetAsync(out_b, 0, 8, st) : hipErrorUnknown;
  LCRC_LAUNCH(lcrc_dev::k_scan2_add, dim3((unsigned)g), dim3(256), 0, st, n, out_a, out_b, part, n_dev);
  return hipGetLastError();
}
hipError_t lcrc_launch_scan2(const uint64_t* a, const uint64_t* b, uint64_t n, uint64_t* out_a, uint64_t* out_b,
                             uint64_t* part, const uint64_t* n_dev, hipStream_t st) {
  const uint64_t g = n_dev ? n / 256 + 1 : (n + 255) / 256;
  if (g == 0) return hipMemsetAsync(out_a, 0, 8, st) == hipSuccess ? hipMemsetAsync(out_b, 0, 8, st) : hipErrorUnknown;
  LCRC_LAUNCH(lcrc_dev::k_scan2_local, dim3((unsigned)g), dim3(256), 0, st, a, b, n, out_a, out_b, part, n_dev);
  LCRC_LAUNCH(lcrc_dev::k_scan2_add, dim3((unsigned)g), dim3(256), 0, st, n, out_a, out_b, part, n_dev);
  return hipGetLastError();
}

hipError_t lcrc_launch_snappy_decode(const uint8_t* base, const lcrc_desc_dev* frames, uint64_t n,
                                     const uint64_t* out_off, const uint64_t* chunk_off, uint8_t* out, uint8_t* status,
                                     lcrc_desc_dev* cdesc, uint32_t* cexp, uint32_t* cframe, uint32_t max_in,
                                     uint32_t max_out, hipStream_t st) {
  using lcrc_dev::SN_MAX;
  if (n == 0) return hipSuccess;
  const uint64_t g = n < 16384 ? n : 16384;  // one wave per frame, grid-stride
  // LDS sized to the batch's largest chunk (bigger ones take the lane-serial path): small staging, many waves
  const uint32_t in_lim = max_in + 4 < SN_MAX ? (max_in + 4 + 15) & ~15u : SN_MAX;
  const uint32_t out_cap = max_out < SN_MAX ? (max_out + 15) & ~15u : SN_MAX;
  const size_t lds = (size_t)in_lim + lcrc_dev::SN_SLACK + out_cap;
  LCRC_LAUNCH(lcrc_dev::k_snappy_decode_wave, dim3((unsigned)g), dim3(64), lds, st, base, frames, n, out_off,
              chunk_off, out, status, cdesc, cexp, cframe, in_lim, out_cap);
  return hipGetLastError();
}

hipError_t lcrc_launch_snappy_check(const uint32_t* crc, const uint32_t* cexp, const uint32_t* cframe,
                                    const uint64_t* nch, uint64_t nch_bound, uint8_t* status, hipStream_t st) {
  if (nch_bound == 0) return hipSuccess;
  LCRC_LAUNCH(lcrc_dev::k_snappy_check, dim3((unsigned)((nch_bound + 255) / 256)), dim3(256), 0, st, crc, cexp,
                     cframe, nch, status);
  return hipGetLastError();
}

hipError_t lcrc_launch_idx_parse(bool pass2, const uint8_t* d, uint32_t len, uint32_t nres, uint64_t file_len,
                                 uint64_t* count, uint64_t* flag, const uint64_t* pos, lcrc_tblk_dev* out,
                                 lcrc_desc_dev* descs, hipStream_t st) {
  if (nres == 0) return hipSuccess;
  const dim3 g((nres + 255) / 256);
  if (pass2)
    LCRC_LAUNCH(lcrc_dev::k_idx_parse<true>, g, dim3(256), 0, st, d, len, nres, file_len, count, flag, pos, out,
                       descs);
  else
    LCRC_LAUNCH(lcrc_dev::k_idx_parse<false>, g, dim3(256), 0, st, d, len, nres, file_len, count, flag, pos, out,
                       descs);
  return hipGetLastError();
}

hipError_t lcrc_launch_tbl_finish(lcrc_tblk_dev* blk, uint64_t n, const uint32_t* crc, const uint32_t* mismatch,
                                  const uint8_t* file, lcrc_desc_dev* frames, const uint64_t* n_dev, hipStream_t st) {
  if (n == 0) return hipSuccess;
  LCRC_LAUNCH(lcrc_dev::k_tbl_finish, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, blk, n, crc, mismatch,
                     file, frames, n_dev);
  return hipGetLastError();
}

hipError_t lcrc_launch_tbl_content(lcrc_tblk_dev* blk, uint64_t n, const uint8_t* fstatus, uint32_t* unsorted,
                                   uint32_t gen, const uint64_t* n_dev, hipStream_t st) {
  if (n == 0) return hipSuccess;
  LCRC_LAUNCH(lcrc_dev::k_tbl_content, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, blk, n, fstatus,
                     unsorted, gen, n_dev);
  return hipGetLastError();
}

hipError_t lcrc_launch_gather_u8(const uint8_t* base, const uint64_t* pos, uint64_t n, uint8_t* out, hipStream_t st) {
  if (n == 0) return hipSuccess;
  LCRC_LAUNCH(lcrc_dev::k_gather_u8, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, base, pos, n, out);
  return hipGetLastError();
}

hipError_t lcrc_launch_store_crc(uint8_t* base, uint64_t base_len, const lcrc_desc_dev* descs, const uint32_t* crc, uint64_t n,
                                 hipStream_t st) {
  if (n == 0) return hipSuccess;
  LCRC_LAUNCH(lcrc_dev::k_store_crc, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, base, base_len, descs,
                     crc, n);
  return hipGetLastError();
}


}  // extern "C"
