/*
 * lcrc.h -- C ABI of the MI355X (gfx950) block/record checksum engine for leveldb-rust.
 *
 * This is the drop-in boundary for the checksum path of FateTHarlaown/leveldb-rust. The reference
 * computes every block-trailer and WAL-record checksum with the external crate `crc32fast`
 * (Cargo.toml:11, "1.2.0") through a stack-local `crc32fast::Hasher` at four call sites:
 *   (1) LogWriter::emit_physical_record   src/db/log.rs:61-64    crc over type_u8 || payload
 *   (2) LogReader::read_physical_record   src/db/log.rs:261-264  same, verified against header[0..4]
 *   (3) write_raw_block                   src/sstable/table.rs:519-522  crc over content || type_u8
 *   (4) BlockContent::read_block_from_file src/sstable/format.rs:164-166 verify data[0..n+1]
 * The masked CRC-32C named by the project metric appears only inside the `snap` crate's framing
 * (Cargo.toml:15; used at src/sstable/table.rs:486, src/sstable/format.rs:196).
 *
 * Entry points, and the reference interface each replaces:
 *   lcrc_hasher_{init,update,finalize}  <- crc32fast::Hasher::{new, update, finalize} (call sites 1-4)
 *   lcrc32_value / lcrc32_extend        <- Hasher::new().update(p).finalize() /
 *                                          Hasher::new_with_initial(crc).update(p).finalize()
 *   lcrc32c_{value,extend,mask,unmask}  <- the crc32c value/extend/mask surface (north star; the
 *                                          snap framing's masked CRC-32C)
 *   lcrc_combine                        <- crc32fast::Hasher::combine (zlib crc32_combine)
 *   lcrc_batch / lcrc_batch_uniform     <- N independent calls of (3)/(4): one launch checksums and
 *                                          optionally verifies thousands of device-resident blocks
 *   lcrc_batch_covered                  <- the same for a sparse set (Table::block_iter_from_index reading a
 *                                          few blocks of a file, table.rs:114-146): cost ~ the blocks read
 *   lcrc_batch_uniform_queue            <- the same for a queue of independent batches (e.g. every table of
 *                                          a compaction's output), submitted as one launch per 32 batches
 *   lcrc_batch_queue                    <- lcrc_batch for a queue of independent descriptor batches
 *   lcrc_batch_multi                    <- a host-resident descriptor batch sharded over several GPUs
 *   lcrc_batch_host_uniform             <- the same starting and ending in host memory (pinned H2D,
 *                                          kernel, D2H, double-buffered)
 *   lcrc_wal_scan / lcrc_wal_scan_async <- the header parse + CRC verify of (2) for every physical record
 *                                          of a device-resident log file, 32 KiB block by block
 *   lcrc_wal_scan_queue                 <- the same for several log files in one submission (recovery, scrub)
 *   lcrc_tb_* + lcrc_batch_seal         <- TableBuilder (table.rs:344-529) with the trailers sealed in batch
 *   lcrc_table_scan[_async]             <- Table::open with paranoid_checks (table.rs:39-103) followed by
 *                                          read_block_from_file(verify_checksum) (format.rs:146-171) of
 *                                          every data, filter, metaindex and index block: one batched verify
 *   lcrc_snappy_frames                  <- snap::read::FrameDecoder at format.rs:194-206 (decode + the masked
 *                                          CRC-32C of every chunk), for a batch of frames on the device
 *   lcrc_batch_seal                     <- (1)/(3) for a batch: the trailer CRCs of write_raw_block
 *                                          (table.rs:519-527) or the header CRCs of emit_physical_record
 *                                          (log.rs:61-70), computed and stored in place on the device
 *
 * Conventions: plain pointers and sizes, no exceptions cross the boundary, every call returns an int
 * status (LCRC_OK = 0). Buffers are owned by the caller. A context is bound to one device and one mode;
 * calls on one context must not race each other (use one context per host thread). `stream` is a
 * hipStream_t (NULL = the context's own stream). The batched calls are GPU-only: when no device or
 * kernel image is available they return LCRC_ENODEV and compute nothing -- there is no CPU fallback.
 */
#ifndef LCRC_H
#define LCRC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---- */
#define LCRC_OK 0
#define LCRC_EINVAL (-1)  /* bad argument */
#define LCRC_ENODEV (-2)  /* no HIP device / kernel image unavailable */
#define LCRC_EHIP (-3)    /* HIP runtime error (see lcrc_last_error) */
#define LCRC_ENOMEM (-4)  /* device or pinned allocation failed */
#define LCRC_ECORRUPT (-5) /* lcrc_table_scan: the table structure is corrupt (message in err) */
#define LCRC_ERANGE (-6)  /* output capacity too small; the count needed is returned */

/* ---- CRC modes ---- */
#define LCRC_MODE_REF 0 /* CRC-32/ISO-HDLC, refl. poly 0xEDB88320: bit-exact with crc32fast::Hasher */
#define LCRC_MODE_C 1   /* CRC-32C (Castagnoli), refl. poly 0x82F63B78 */

/* ---- flags ---- */
#define LCRC_FLAG_MASK 0x1u   /* outputs (and expected values) are LevelDB-masked: rotr15(crc)+0xa282ead8 */
#define LCRC_FLAG_DIRECT 0x2u /* lcrc_batch: skip the window pass, walk every block directly (sparse sets) */

/* ---- scalar host API (drop-in for crc32fast::Hasher at the four call sites) ---- */
uint32_t lcrc32_value(const uint8_t* p, size_t n);
uint32_t lcrc32_extend(uint32_t crc, const uint8_t* p, size_t n);
uint32_t lcrc32c_value(const uint8_t* p, size_t n);
uint32_t lcrc32c_extend(uint32_t crc, const uint8_t* p, size_t n);
uint32_t lcrc32c_mask(uint32_t crc);
uint32_t lcrc32c_unmask(uint32_t masked);
uint32_t lcrc_extend(int mode, uint32_t crc, const uint8_t* p, size_t n);
uint32_t lcrc_combine(int mode, uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

typedef struct lcrc_hasher {
  uint32_t state;  /* finalized CRC of the bytes seen so far */
  int32_t mode;    /* LCRC_MODE_* */
  uint64_t amount; /* bytes seen */
} lcrc_hasher;
void lcrc_hasher_init(lcrc_hasher* h, int mode);
void lcrc_hasher_update(lcrc_hasher* h, const uint8_t* p, size_t n);
uint32_t lcrc_hasher_finalize(const lcrc_hasher* h);

/* ---- batched device API ---- */
typedef struct lcrc_ctx lcrc_ctx;

/* One checksummed byte range. The covered bytes are base[offset, offset+length). If expect_rel !=
 * LCRC_NO_EXPECT the expected CRC is the little-endian u32 at base[offset + expect_rel]:
 *   SSTable block with handle (off, n):  {off, n + 1, n + 1}   (table.rs:507-529, format.rs:162-171)
 *   WAL physical record with header at h: {h + 6, 1 + len, -6}  (log.rs:58-80, log.rs:233-273)   */
typedef struct lcrc_desc {
  uint64_t offset;
  uint32_t length;
  int32_t expect_rel;
} lcrc_desc;
#define LCRC_NO_EXPECT ((int32_t)0x80000000)

/* WAL physical record as parsed on the device by lcrc_wal_scan (one per record, in file order). */
typedef struct lcrc_wal_rec {
  uint64_t header;   /* file offset of the 7-byte header */
  uint32_t length;   /* payload length (header bytes 4..6) */
  uint8_t type;      /* header byte 6 */
  uint8_t status;    /* LCRC_WAL_OK / LCRC_WAL_CRC_MISMATCH */
  uint16_t block_end; /* 1 if this is the last record parsed in its 32 KiB block (see stop) */
  uint32_t crc;      /* computed crc over type || payload */
  uint32_t stop;     /* for the last record of a block: why parsing stopped (LCRC_WAL_STOP_*) */
} lcrc_wal_rec;
#define LCRC_WAL_OK 0
#define LCRC_WAL_CRC_MISMATCH 1
#define LCRC_WAL_STOP_TRAILER 0    /* < 7 bytes left in the block */
#define LCRC_WAL_STOP_BAD_LENGTH 1 /* 7 + length exceeds the bytes left in the block */
#define LCRC_WAL_STOP_ZERO 2       /* type == 0 && length == 0 (zero fill) */
#define LCRC_WAL_STOP_MISMATCH 3   /* checksum mismatch: the reader drops the rest of the block */

/* Contexts and streams. A context owns per-call device workspace (window values, WAL and table-scan state,
 * the shard buffers of lcrc_batch_multi). Calls on ONE context must therefore be stream-ordered: issue them
 * on one stream (or order the streams with events); two calls of one context in flight on two unordered
 * streams race on that workspace. For concurrent streams use one context per stream (bench.py does: one
 * context per engine). Different contexts never share workspace. */
int lcrc_device_count(int* n);
/* The PCI bus ID of a device ("dddd:bb:dd.f", NUL-terminated in out[0, len)): a multi-process caller can check that
 * its ranks drive distinct GPUs (bench.py records it per rank and refuses two ranks on one GPU). */
int lcrc_device_pci_bus_id(int device, char* out, int len);
int lcrc_ctx_create(lcrc_ctx** out, int device, int mode, uint32_t flags);
/* Kernel-selection and grid overrides for tests and measurement (production callers use lcrc_ctx_create, which is
 * lcrc_ctx_create_ex with every option at its default). Zero-initialise, set size = sizeof(lcrc_ctx_options); a
 * field left 0 keeps the default. The library reads no environment variable. */
typedef struct lcrc_ctx_options {
  uint32_t size;
  int32_t general;        /* general path: 0 auto, 1 the one-pass k_ranges, 2 window pass + range pass always */
  uint32_t batch_grid_b;  /* lcrc_batch's range-pass workgroups (0: 2 per CU) */
  uint32_t wal_grid_b;    /* the WAL scan's range-pass workgroups (0: every resident one) */
  uint32_t ts_grid;       /* the table scan's index workgroup cap (0: one per 512 blocks of result capacity, at most
                             the CUs and 256) */
  uint32_t ts_blocks_div; /* divisor of the table scan's range-pass grid (0: 1) */
  uint32_t reserved[3];   /* must be 0 (LCRC_EINVAL otherwise): the round-5 measurement variants wal_onepass,
                             ts_open_v1 and ts_unfused were measured slower and removed */
} lcrc_ctx_options;
int lcrc_ctx_create_ex(lcrc_ctx** out, int device, int mode, uint32_t flags, const lcrc_ctx_options* opt);
int lcrc_ctx_destroy(lcrc_ctx* ctx);
/* Pre-allocate the device workspace for spans up to max_span bytes (so later calls allocate nothing
 * and can be captured in a hipGraph). */
int lcrc_ctx_reserve(lcrc_ctx* ctx, uint64_t max_span);
/* hipStream_t owned by the context (for callers that want to enqueue around it). */
void* lcrc_ctx_stream(lcrc_ctx* ctx);
int lcrc_ctx_sync(lcrc_ctx* ctx);
/* Order two contexts' streams: ctx's stream waits, on the device, for everything enqueued on other's stream so
 * far (an event; nothing synchronizes with the host). E.g. a scan on one context whose results another context
 * consumes, or one event timer closing over several contexts' work (bench.py). */
int lcrc_ctx_join(lcrc_ctx* ctx, lcrc_ctx* other);

/* CRC of n ranges of the device buffer base[0, base_len). out_crc[i] (device) gets the CRC (masked if
 * LCRC_FLAG_MASK). out_mismatch (device, nullable, ceil(n/32) u32 words, zeroed by the call) gets bit i
 * set when descriptor i has an expected value and it differs. Ranges may be in any order and may
 * overlap; every byte of [0, base_len) is streamed once unless LCRC_FLAG_DIRECT is given. A range that
 * does not lie inside [0, base_len) is never read: its CRC is 0 and its mismatch bit is set. */
int lcrc_batch(lcrc_ctx* ctx, const uint8_t* base, uint64_t base_len, const lcrc_desc* descs, size_t n,
               uint32_t* out_crc, uint32_t* out_mismatch, void* stream);

/* lcrc_batch with a hint: covered_bytes = the sum of the descriptors' lengths, or an upper bound (0 = not
 * known). A sparse batch -- a few blocks verified inside a large file, covered_bytes < base_len / 4 -- runs
 * the one-pass range kernel, which reads only the covered bytes (its cost follows the blocks, not the
 * file); otherwise exactly lcrc_batch. The results are the same either way. */
int lcrc_batch_covered(lcrc_ctx* ctx, const uint8_t* base, uint64_t base_len, const lcrc_desc* descs, size_t n,
                       uint64_t covered_bytes, uint32_t* out_crc, uint32_t* out_mismatch, void* stream);

/* n blocks of `length` bytes, block i at base + i*stride (device). expected (device, nullable):
 * per-block expected CRCs. The 4 KiB / stride 4 KiB case is the single-pass fast path. */
int lcrc_batch_uniform(lcrc_ctx* ctx, const uint8_t* base, size_t n, uint32_t length, uint64_t stride,
                       const uint32_t* expected, uint32_t* out_crc, uint32_t* out_mismatch, void* stream);

/* One batch of a queue (lcrc_batch_uniform_queue): n blocks of the queue's length at base + i*stride. */
typedef struct lcrc_ujob {
  const uint8_t* base;      /* device */
  uint64_t n;               /* blocks */
  const uint32_t* expected; /* device, nullable */
  uint32_t* out_crc;        /* device, n words */
  uint32_t* out_mismatch;   /* device, nullable, ceil(n/32) words, zeroed by the call */
} lcrc_ujob;

/* A queue of independent uniform batches (jobs: HOST array of njobs), each exactly as one
 * lcrc_batch_uniform(ctx, jobs[k].base, jobs[k].n, length, stride, ...) call, in one submission. For the
 * 4 KiB / stride 4 KiB layout the batches are streamed by ONE launch of the fast-path kernel per 32 jobs
 * (the LDS table image and the end-of-launch spread paid once per launch, not once per batch); other
 * layouts run batch by batch. Enqueued on `stream`, graph-capturable, nothing synchronized. */
int lcrc_batch_uniform_queue(lcrc_ctx* ctx, const lcrc_ujob* jobs, size_t njobs, uint32_t length, uint64_t stride,
                             void* stream);

/* One batch of a general queue (lcrc_batch_queue): exactly the arguments of one lcrc_batch call. */
typedef struct lcrc_gjob {
  const uint8_t* base;    /* device */
  uint64_t base_len;
  const lcrc_desc* descs; /* device, n descriptors */
  uint64_t n;
  uint32_t* out_crc;      /* device, n words */
  uint32_t* out_mismatch; /* device, nullable, ceil(n/32) words, zeroed by the call */
} lcrc_gjob;

/* A queue of independent descriptor batches (jobs: HOST array of njobs), each exactly as one
 * lcrc_batch(ctx, jobs[k].base, jobs[k].base_len, jobs[k].descs, jobs[k].n, ...) call -- e.g. every SSTable
 * of a compaction's output, or the files a recovery verifies. The batches alternate over two streams of the
 * context, so two batches' window passes share the HBM stream while their latency-bound range passes overlap.
 * Enqueued on `stream` (the forked work joins it before the call's end), graph-capturable (after
 * lcrc_ctx_reserve), nothing synchronized. */
int lcrc_batch_queue(lcrc_ctx* ctx, const lcrc_gjob* jobs, size_t njobs, void* stream);

/* Same as lcrc_batch_uniform but base / expected / out_crc / out_mismatch are HOST pointers. Data is
 * staged through pinned buffers in chunks of chunk_bytes (0 = default) with H2D copies overlapping
 * the kernels. Synchronous. */
int lcrc_batch_host_uniform(lcrc_ctx* ctx, const uint8_t* base, size_t n, uint32_t length, uint64_t stride,
                            const uint32_t* expected, uint32_t* out_crc, uint32_t* out_mismatch,
                            size_t chunk_bytes);

/* Several GPUs, one HOST-resident file (an mmap'd .ldb, a log buffer): the descriptor list (host), taken in
 * offset order, is cut into nctx contiguous shards of about equal covered bytes; shard k runs on ctxs[k] (its
 * own device, stream and host thread): the byte span its ranges and expected values read is copied H2D, its
 * descriptors are rebased to the span, one lcrc_batch, CRCs and mismatch bits D2H into out_crc / out_mismatch
 * (host, n and ceil(n/32) entries) at the descriptors' own positions (a list out of offset order is sorted on
 * the host and the results scattered back, so no shard copies more than its own span). Same results as
 * lcrc_batch over the whole file; no collective, the host concatenates. Several contexts may
 * share a device. Synchronous; on an error, lcrc_last_error() names the failing shard. */
int lcrc_batch_multi(lcrc_ctx* const* ctxs, int nctx, const uint8_t* base, uint64_t base_len, const lcrc_desc* descs,
                     size_t n, uint32_t* out_crc, uint32_t* out_mismatch);

/* Parse and verify every physical record of a device-resident log file (file_len bytes, 32 KiB
 * blocks, layout of src/db/log.rs). Records are written in file order to recs (device, capacity
 * max_recs); *n_recs (host) receives the count. Returns LCRC_EINVAL if max_recs is too small. */
int lcrc_wal_scan(lcrc_ctx* ctx, const uint8_t* file, uint64_t file_len, lcrc_wal_rec* recs,
                  size_t max_recs, size_t* n_recs, void* stream);
/* Asynchronous form: enqueued on `stream`, nothing is synchronized; the record count is written to
 * *n_recs (DEVICE or pinned host memory) by the last kernel. Records past max_recs are not written. */
int lcrc_wal_scan_async(lcrc_ctx* ctx, const uint8_t* file, uint64_t file_len, lcrc_wal_rec* recs,
                        size_t max_recs, uint64_t* n_recs, void* stream);

/* One log of a queued WAL scan (lcrc_wal_scan_queue): the arguments of one lcrc_wal_scan_async call. */
typedef struct lcrc_wjob {
  const uint8_t* file;   /* device */
  uint64_t file_len;
  lcrc_wal_rec* recs;    /* device, max_recs records */
  uint64_t max_recs;
  uint64_t* n_recs;      /* device or pinned host: the record count */
} lcrc_wjob;

/* Several logs scanned in one submission, each exactly as one lcrc_wal_scan_async call (jobs: HOST array) --
 * e.g. every log file a recovery or a scrub verifies. The header walks of all the logs run first, in one
 * launch, while the HBM stream is idle; then the logs alternate over two streams of the context as in
 * lcrc_batch_queue. Enqueued on `stream`, nothing is synchronized, graph-capturable after a first call of the
 * same shape (per-log workspaces are allocated on first use). */
int lcrc_wal_scan_queue(lcrc_ctx* ctx, const lcrc_wjob* jobs, size_t njobs, void* stream);

/* One block of an SSTable located by lcrc_table_scan (host struct, 24 B). */
typedef struct lcrc_tblk {
  uint64_t offset;  /* BlockHandle offset */
  uint64_t size;    /* BlockHandle size n; the 5-byte trailer [type][crc] follows */
  uint32_t crc;     /* computed CRC of data[0..n+1] (masked if LCRC_FLAG_MASK) */
  uint8_t kind;     /* LCRC_TBLK_DATA / _FILTER / _METAINDEX / _INDEX */
  uint8_t type;     /* stored type byte data[n] (0 raw, 1 snappy, other: "bad block type" on read) */
  uint8_t status;   /* LCRC_TBLK_OK / _CRC_MISMATCH / _TRUNCATED / _BAD_CONTENT / _BAD_TYPE */
  uint8_t reserved;
} lcrc_tblk;
#define LCRC_TBLK_DATA 0
#define LCRC_TBLK_FILTER 1
#define LCRC_TBLK_METAINDEX 2
#define LCRC_TBLK_INDEX 3
#define LCRC_TBLK_OK 0
#define LCRC_TBLK_CRC_MISMATCH 1 /* read_block_from_file(verify) -> "block checksum mismatch" */
#define LCRC_TBLK_TRUNCATED 2    /* handle past the end of the file -> "truncated block read" */
#define LCRC_TBLK_BAD_CONTENT 3  /* good checksum, type 1, Snappy frames corrupt -> "corrupted compressed block content" */
#define LCRC_TBLK_BAD_TYPE 4     /* good checksum, type byte > 1 -> "bad block type" */

/* Whole-table verify scan of a device-resident SSTable file (file_len bytes). The host reads the footer
 * and the index block (verified: paranoid_checks), and -- when filter_name is non-NULL, as read_meta does
 * for a filter policy -- the metaindex block and the "filter" + filter_name entry; then ONE batched
 * device pass checksums every data, filter, metaindex and index block, and every block whose checksum
 * holds is put through read_block_from_file's type dispatch: Snappy-framed blocks (type 1) are decoded
 * and their chunk CRCs checked on the device (lcrc_snappy_frames), other types > 1 are bad. blocks (host, capacity
 * max_blocks) receives them sorted by offset; *n_blocks the count (LCRC_ERANGE if it exceeds
 * max_blocks; blocks may be NULL to query). Structural corruption returns LCRC_ECORRUPT with the
 * reference's message ("file is too short to be an sstable", "not an sstable (bad magic number)",
 * "block checksum mismatch", "bad block type", "corrupted compressed block content", "bad block
 * contents", "bad entry in block", "truncated block read", "Error when decoding varint64") copied to
 * err (capacity err_cap, may be NULL). Synchronous. */
int lcrc_table_scan(lcrc_ctx* ctx, const uint8_t* file, uint64_t file_len, const char* filter_name,
                    lcrc_tblk* blocks, size_t max_blocks, size_t* n_blocks, char* err, size_t err_cap);

/* The same scan with no host round trip: every step -- footer, index walk (one thread per restart
 * segment), read_meta's filter entry, ONE batched verify of every block, the type dispatch, Snappy frames
 * decoded and their chunks checked -- is enqueued on `stream` and runs on the device; graph-capturable after
 * lcrc_table_scan_reserve. The index and metaindex are walked before their own checksums are known and
 * verified in the same batch; the outcome is then ordered as the reference's (index checksum first, a filter
 * named by a metaindex that does not verify dropped). blocks (DEVICE, capacity max_blocks) receives the
 * blocks in index order (by offset for a well-formed table); *n_blocks (device or pinned) their count;
 * status[0..1] (device or pinned u32) the verdict: LCRC_TSCAN_OK, LCRC_TSCAN_CORRUPT with status[1] the
 * message (lcrc_table_scan_message), LCRC_TSCAN_HOST when the table needs the synchronous scan's host
 * walk (a Snappy-framed index without LCRC_TSCAN_SNAPPY_INDEX or one that does not decode, a Snappy-framed
 * metaindex, a handle past the file, restart segments over 4 KiB, decoded bytes over the reserved workspace), or
 * LCRC_TSCAN_CAPACITY with *n_blocks the capacity needed. */
#define LCRC_TSCAN_OK 0
#define LCRC_TSCAN_CORRUPT 1
#define LCRC_TSCAN_HOST 2
#define LCRC_TSCAN_CAPACITY 3
int lcrc_table_scan_async(lcrc_ctx* ctx, const uint8_t* file, uint64_t file_len, const char* filter_name,
                          lcrc_tblk* blocks, size_t max_blocks, uint64_t* n_blocks, uint32_t* status, void* stream);
/* lcrc_table_scan_async with flags. LCRC_TSCAN_SNAPPY_INDEX: the table was written with Snappy compression (the
 * reference's default, option.rs:127), so its index block is likely a Snappy frame (table.rs:430, write_block):
 * one more launch decodes a framed index block on the device -- every chunk's masked CRC-32C checked -- and the walk
 * reads the decoded contents (without the flag such a table is LCRC_TSCAN_HOST; with it a raw index costs that
 * launch only). The decoded index takes workspace like the frames' (lcrc_table_scan_reserve's decoded_cap). */
#define LCRC_TSCAN_SNAPPY_INDEX 0x1u
int lcrc_table_scan_async_ex(lcrc_ctx* ctx, const uint8_t* file, uint64_t file_len, const char* filter_name,
                             lcrc_tblk* blocks, size_t max_blocks, uint64_t* n_blocks, uint32_t* status, uint32_t flags,
                             void* stream);
/* Workspace for lcrc_table_scan_async up to these sizes (decoded_cap: the Snappy frames' decoded bytes). */
int lcrc_table_scan_reserve(lcrc_ctx* ctx, uint64_t max_file_len, size_t max_blocks, uint64_t decoded_cap);
/* The reference's message for a LCRC_TSCAN_CORRUPT code ("" for none). */
const char* lcrc_table_scan_message(uint32_t code);

/* Writer side, for a batch: CRC of every descriptor (masked if LCRC_FLAG_MASK) stored little-endian at
 * base[offset + expect_rel] in place (device). SSTable block: {off, n + 1, n + 1} writes the trailer crc;
 * WAL record with header at h: {h + 6, 1 + len, -6} writes the header crc. out_crc (device, nullable)
 * also receives the values. Covered ranges must not contain another descriptor's CRC slot. */
int lcrc_batch_seal(lcrc_ctx* ctx, uint8_t* base, uint64_t base_len, const lcrc_desc* descs, size_t n,
                    uint32_t* out_crc, void* stream);

/* The SSTable writer (TableBuilder, src/sstable/table.rs:344-529: data blocks with restart points, the
 * filter block written raw under the table's compression type (table.rs:383-391), metaindex, index with
 * shortest separators, footer) in host memory. host_seal != 0 computes every trailer crc on the host
 * (write_raw_block, table.rs:504-529); host_seal == 0 leaves the 4 crc bytes zero, to be filled on the device
 * by one lcrc_batch_seal over lcrc_tb_seal_descs' descriptors. compression: 0 none, 1 Snappy framing. */
void* lcrc_tb_create(uint32_t block_size, int restart_interval, uint8_t compression, int mode, uint32_t flags,
                     int host_seal);
void lcrc_tb_destroy(void* tb);
int lcrc_tb_add(void* tb, const uint8_t* key, size_t klen, const uint8_t* val, size_t vlen); /* keys ascending */
/* n entries at once: keys[i * klen], vals[i * vlen] (fixed sizes, keys ascending) */
int lcrc_tb_add_many(void* tb, const uint8_t* keys, size_t klen, const uint8_t* vals, size_t vlen, size_t n);
void lcrc_tb_flush(void* tb);                                                                 /* end a data block */
int lcrc_tb_finish(void* tb, const char* filter_name, const uint8_t* filter, size_t filter_len);
size_t lcrc_tb_size(void* tb);
const uint8_t* lcrc_tb_data(void* tb); /* the file's bytes (lcrc_tb_size of them) */
/* the blocks that carry a trailer, in file order (crc 0 unless sealed on the host); returns their count */
size_t lcrc_tb_blocks(void* tb, lcrc_tblk* out, size_t cap);
/* one lcrc_batch_seal descriptor {offset, n + 1, n + 1} per block; returns their count */
size_t lcrc_tb_seal_descs(void* tb, lcrc_desc* out, size_t cap);

/* Snappy framing, on the device: the `snap` crate's FrameDecoder as read_block_from_file uses it for
 * compressed blocks (src/sstable/format.rs:194-206; written by FrameEncoder, table.rs:481-497). Decodes the
 * n frames base[frames[i].offset, +length) (device; expect_rel ignored) into out (device, capacity out_cap):
 * frame i's bytes at out_off[i] (device, n + 1 entries, out_off[n] = total). Every data chunk's masked
 * CRC-32C of its uncompressed bytes is checked whatever the context's mode. status[i] (device): 0 ok,
 * 1 bad framing or Snappy data, 2 chunk CRC mismatch -- both are read_block_from_file's "corrupted
 * compressed block content". *total (host) receives the decoded size; LCRC_ERANGE (nothing decoded) when
 * it exceeds out_cap. Synchronous. */
int lcrc_snappy_frames(lcrc_ctx* ctx, const uint8_t* base, const lcrc_desc* frames, size_t n, uint8_t* out,
                       uint64_t out_cap, uint64_t* out_off, uint8_t* status, uint64_t* total);

/* ---- device memory helpers (so a binding needs nothing but this library) ---- */
int lcrc_dev_alloc(int device, size_t bytes, void** out);
int lcrc_dev_free(void* p);
int lcrc_host_alloc_pinned(size_t bytes, void** out);
int lcrc_host_free_pinned(void* p);
int lcrc_memcpy_h2d(void* dst, const void* src, size_t bytes);
int lcrc_memcpy_d2h(void* dst, const void* src, size_t bytes);
int lcrc_memset_d(void* dst, int value, size_t bytes);
int lcrc_device_sync(void);
/* Event timing on the context stream (milliseconds between two recorded events). Or carried by the launches
 * themselves (every batched device call: lcrc_batch_uniform[_queue], lcrc_batch, lcrc_batch_queue, lcrc_batch_seal,
 * lcrc_wal_scan_async / _queue, lcrc_table_scan_async): lcrc_timer_kernels(ctx, 0) before the first timed call
 * (its first launch records the start), lcrc_timer_kernels(ctx, 1) before the last (its launches record the end,
 * the last one wins), lcrc_timer_kernels(ctx, 2) disarms; no marker between launches. lcrc_timer_stop ends either
 * form. */
int lcrc_timer_start(lcrc_ctx* ctx);
int lcrc_timer_kernels(lcrc_ctx* ctx, int edge);
int lcrc_timer_stop(lcrc_ctx* ctx, float* ms);
/* Kernel-carried timing across contexts (one stream each, same device): `first`'s start event (edge 0) to
 * `last`'s stop event (edge 1), for submissions rotated over several streams (lcrc_batch_uniform included). */
int lcrc_timer_span(lcrc_ctx* first, lcrc_ctx* last, float* ms);

/* HIP graphs of the context's own stream: lcrc_graph_begin starts capturing the calls made on the context
 * with stream NULL (they must allocate nothing: reserve first; the queued calls' two side streams are created
 * by lcrc_graph_begin itself, so even a first queued call can be captured), lcrc_graph_end instantiates them as
 * one replayable graph; lcrc_graph_launch replays it on the context stream. */
int lcrc_graph_begin(lcrc_ctx* ctx);
int lcrc_graph_end(lcrc_ctx* ctx, void** graph_exec);
int lcrc_graph_launch(lcrc_ctx* ctx, void* graph_exec);
int lcrc_graph_destroy(void* graph_exec);

/* Last HIP error string for this thread ("" if none). */
const char* lcrc_last_error(void);
/* Library build identification (kernel arch, version). */
const char* lcrc_version(void);

#ifdef __cplusplus
}
#endif
#endif /* LCRC_H */
