// Layouts shared by the kernels (lcrc_kernels.hip) and the host launcher code (lcrc_api.cpp).
#pragma once
#include <stdint.h>

#ifndef LCRC_LOAD_AUX
#define LCRC_LOAD_AUX 2  // cache-policy bits of the streaming buffer loads: 2 = nt (read-once stream)
#endif

#ifndef LCRC_FLAG_MASK
#define LCRC_FLAG_MASK 0x1u
#endif
// kernel-only flag (k_blocks, k_ranges): the mismatch bitmap was NOT zeroed before the launch -- every range
// sets or clears its own bit, and the last range clears the bits past n in the last word (no fill kernel)
#define LCRC_KFLAG_SETCLR 0x100u

// Per-mode constant table image (uint32 words), uploaded once per context.
enum : int {
  TAB_SLICE = 0,      // T0..T3 slice-by-4, 4 x 256
  TAB_ZPIECE = 1024,  // Z16, Z32, Z64, Z128 byte-sliced shift tables, 4 x (4 x 256)
  TAB_ZWIN = 5120,    // Z256, Z512, Z1024, Z2048
  TAB_Z4096 = 9216,   // Z4096
  TAB_COLS = 10240,   // k_windows' LDS image as columns: 20 byte tables x 8 columns (table[1 << i]):
                      // S0 T_p (p = 0..3), S1 Z64[3 - p], then Z256, Z512, Z1024 in TAB_ZWIN word order
  TAB_INV = 10400,    // x^(-8k) mod P for k = 0..4096 (k_ranges: undo the zero padding of a last chunk)
  TAB_XCH = 14497,    // x^(8 * 4096 * k) mod P for k = 0..4095 (k_ranges: place a shared range's chunk)
  TAB_SCOLS = 18600,  // the queued fast path's block shifts as columns: Z_{256 k}, k = 0..15, byte position q =
                      // 0..3 (table index 4 k + q, entry b = Z_{256 k}(b << 8 q)), 8 columns each
  TAB_Z64K = 19112,   // Z65536 (the async table scan joins the 64 KiB pieces of a long block)
  TAB_TOTAL = 20136,
};

struct lcrc_desc_dev {  // == lcrc_desc
  uint64_t offset;
  uint32_t length;
  int32_t expect_rel;
};
#define LCRC_NO_EXPECT_DEV ((int32_t)0x80000000)

struct lcrc_tblk_dev {  // == lcrc_tblk
  uint64_t offset;
  uint64_t size;
  uint32_t crc;
  uint8_t kind, type, status, reserved;
};

struct lcrc_wal_rec_dev {  // == lcrc_wal_rec
  uint64_t header;
  uint32_t length;
  uint8_t type;
  uint8_t status;
  uint16_t block_end;
  uint32_t crc;
  uint32_t stop;
};
#define LCRC_WAL_STOP_TRAILER_DEV 0
#define LCRC_WAL_STOP_BAD_LENGTH_DEV 1
#define LCRC_WAL_STOP_ZERO_DEV 2
#define LCRC_WAL_MAX_FILE (1ull << 34)  // WAL scans: files below 16 GiB (record indices fit 32 bits)

// One batch of a queued uniform launch as the launcher receives it (lcrc_ujob minus the layout fields).
struct lcrc_qjob_host {
  const uint8_t* base;
  uint32_t* out;
  const uint32_t* expected;
  uint32_t* mismatch;
  uint64_t nblk;
};

// One log of a queued WAL scan as the launcher receives it (its workspace and outputs).
struct lcrc_wjob_dev_host {
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

// State of an asynchronous whole-table scan (lcrc_table_scan_async), in device memory.
struct lcrc_tscan_dev {
  uint32_t status;  // LCRC_TSCAN_* of include/lcrc.h: 0 ok, 1 corrupt (`code`), 2 host walk needed, 3 capacity
  uint32_t code;    // LCRC_TSCAN_MSG_* when corrupt
  uint32_t pcode;   // an index-contents error, reported only if the index checksum holds
  uint32_t has_filter;
  uint64_t meta_off, meta_size, idx_off, idx_size, filt_off, filt_size;
  uint64_t nres;     // restart segments of the index block (0: nothing to walk)
  uint64_t n_data;   // data blocks named by the index
  uint64_t n_total;  // blocks in the result (data, filter, metaindex, index)
  uint64_t n_chunks;  // Snappy data chunks of the compressed blocks (0 when over the capacity)
  uint32_t unsorted, gate;
  uint64_t need_out, need_chunks;  // the decoded bytes and chunks the Snappy frames need (set by the gate)
  uint32_t idx_only;  // a restart segment the device walk cannot vouch for: only the index block is verified
  uint32_t any_frame;  // k_ts_finish: some block has a Snappy frame with decoded bytes or chunks (0: the decode gate
                       // needs no sums)
  uint64_t n_verify;  // descriptors of the batched verify: the n_total blocks and the pieces below
  // filter, metaindex, index: a block longer than LCRC_TS_PIECE is verified as pieces of that size (one row of
  // the batch kernel each, instead of one row folding thousands of windows), combined afterwards
  uint32_t pbase[3], pcnt[3];
  // a Snappy-framed index block decoded on the device first (k_ts_open): the walk reads the decoded contents
  uint32_t idx_dec, pad_;
  uint64_t idx_clen;  // the index block's contents length (decoded when idx_dec, else idx_size)
};
#define LCRC_TS_PIECE 65536
struct lcrc_tscan_key {  // the metaindex key read_meta looks for: "filter" + the policy name
  uint32_t len;          // 0: no filter policy
  uint8_t key[124];
};
