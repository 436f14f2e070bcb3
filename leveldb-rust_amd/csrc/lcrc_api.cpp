// C ABI of the batched device engine (include/lcrc.h). Host-side only: contexts, table upload,
// workspace, launch sequencing, the host-resident pipeline and the WAL scan driver. All checksum
// arithmetic on the batched path runs in the gfx950 kernels of lcrc_kernels.hip; when no device is
// present every batched call returns LCRC_ENODEV.
#include <hip/hip_runtime_api.h>

#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lcrc.h"
#include "lcrc_device.h"
#include "lcrc_math.h"
#include "lcrc_table.h"

extern "C" {
void lcrc_launch_events_begin(hipEvent_t start, hipEvent_t stop);
void lcrc_launch_events_end(bool* started, bool* stopped);
hipEvent_t lcrc_launch_events_swap_stop(hipEvent_t ev);
hipError_t lcrc_launch_events_record_stop(hipEvent_t ev, hipStream_t st);
hipError_t lcrc_launch_windows(bool final_mode, int grid, const uint8_t* base, uint64_t span, const uint32_t* gtab,
                               uint32_t* out, uint64_t nblk, uint32_t fin, uint32_t flags,
                               const uint32_t* expected, uint32_t* mismatch, hipStream_t st,
                               hipEvent_t t_start = nullptr, hipEvent_t t_stop = nullptr);
hipError_t lcrc_launch_ranges(bool uniform, int grid, const uint8_t* base, uint64_t base_len,
                              const lcrc_desc_dev* descs, uint64_t n, uint64_t ustride, uint32_t ulen,
                              const uint32_t* uexp, const uint32_t* gtab, uint32_t x4096, uint32_t poly,
                              uint32_t init, uint32_t xorout, uint32_t flags, uint32_t* out, uint32_t* mismatch,
                              const uint64_t* n_dev, lcrc_wal_rec_dev* recs, hipStream_t st, uint32_t rows_per_wg = 32);
hipError_t lcrc_launch_windows_queue(int grid, const lcrc_qjob_host* jobs, uint32_t njobs, const uint32_t* gtab,
                                     uint32_t fin, uint32_t flags, hipStream_t st, hipEvent_t t_start,
                                     hipEvent_t t_stop);
hipError_t lcrc_launch_ts_open(const uint8_t* file, uint64_t file_len, const uint32_t* tab_c, uint8_t* idec,
                               uint64_t idec_cap, uint64_t* iopen, uint32_t* scratch, hipStream_t s);
uint64_t lcrc_ts_open_scratch_words();
hipError_t lcrc_launch_ts_windows(int grid, bool windows, const uint8_t* file, uint64_t file_len, const uint32_t* gtab,
                                  uint32_t* win, const lcrc_tscan_key* key, uint64_t cap, uint64_t vcap,
                                  lcrc_tscan_dev* st, uint64_t* local_c, uint32_t* zero, uint64_t nzero,
                                  const uint8_t* idec, const uint64_t* iopen_r, uint64_t* iopen, lcrc_tblk_dev* out,
                                  lcrc_desc_dev* descs, uint64_t* agg, uint32_t nidx_cap, hipStream_t s);
hipError_t lcrc_launch_ts_finish(lcrc_tblk_dev* blk, uint64_t n, const uint32_t* crc, const uint32_t* mismatch,
                                 const uint8_t* file, lcrc_desc_dev* frames, uint64_t* out_off, uint64_t* choff,
                                 uint64_t* part, uint64_t* nchunks, uint8_t* fstatus, lcrc_tscan_dev* st,
                                 const uint32_t* gtab, uint32_t flags, hipStream_t s);
hipError_t lcrc_launch_ts_decode(const uint8_t* file, const lcrc_desc_dev* frames, const uint64_t* out_off, uint8_t* out,
                                 const uint8_t* fstatus, lcrc_tscan_dev* st, lcrc_tblk_dev* blk, const uint32_t* tab_c,
                                 uint64_t ts_out_cap, const uint64_t* tparts, uint64_t bound, uint64_t* n_out,
                                 uint32_t* status_out, hipStream_t s);
hipError_t lcrc_launch_scan2_add(uint64_t n, uint64_t* out_a, uint64_t* out_b, const uint64_t* part,
                                 const uint64_t* n_dev, hipStream_t st);
int lcrc_blocks_per_cu();
hipError_t lcrc_launch_blocks(bool uniform, int grid, const uint8_t* base, uint64_t base_len,
                              const lcrc_desc_dev* descs, uint64_t n, uint64_t ustride, uint32_t ulen,
                              const uint32_t* uexp, const uint32_t* win, const uint32_t* gtab, uint32_t init,
                              uint32_t xorout, uint32_t flags, uint32_t* out, uint32_t* mismatch,
                              const uint64_t* n_dev, lcrc_wal_rec_dev* recs, hipStream_t st);
hipError_t lcrc_launch_wal_parse(const uint8_t* file, uint64_t file_len, uint64_t nblocks, uint32_t* counts,
                                 uint2* slots, uint8_t* stops, uint64_t* local, uint64_t* part,
                                 lcrc_wal_rec_dev* recs, lcrc_desc_dev* descs, uint64_t max_recs, uint64_t* n_total,
                                 uint64_t* n_out, hipStream_t st);
hipError_t lcrc_launch_wal_parse_queue(const lcrc_wjob_dev_host* jobs, uint32_t m, hipStream_t st);

hipError_t lcrc_launch_snappy_size(const uint8_t* base, const lcrc_desc_dev* frames, uint64_t n, uint64_t* size,
                                   uint64_t* nchunks, uint8_t* status, uint32_t* maxes, const uint64_t* n_dev,
                                   hipStream_t st);
hipError_t lcrc_launch_scan2(const uint64_t* a, const uint64_t* b, uint64_t n, uint64_t* out_a, uint64_t* out_b,
                             uint64_t* part, const uint64_t* n_dev, hipStream_t st);
hipError_t lcrc_launch_snappy_decode(const uint8_t* base, const lcrc_desc_dev* frames, uint64_t n,
                                     const uint64_t* out_off, const uint64_t* chunk_off, uint8_t* out, uint8_t* status,
                                     lcrc_desc_dev* cdesc, uint32_t* cexp, uint32_t* cframe, uint32_t max_in,
                                     uint32_t max_out, hipStream_t st);
hipError_t lcrc_launch_snappy_check(const uint32_t* crc, const uint32_t* cexp, const uint32_t* cframe,
                                    const uint64_t* nch, uint64_t nch_bound, uint8_t* status, hipStream_t st);
hipError_t lcrc_launch_idx_parse(bool pass2, const uint8_t* d, uint32_t len, uint32_t nres, uint64_t file_len,
                                 uint64_t* count, uint64_t* flag, const uint64_t* pos, lcrc_tblk_dev* out,
                                 lcrc_desc_dev* descs, hipStream_t st);
hipError_t lcrc_launch_tbl_finish(lcrc_tblk_dev* blk, uint64_t n, const uint32_t* crc, const uint32_t* mismatch,
                                  const uint8_t* file, lcrc_desc_dev* frames, const uint64_t* n_dev, hipStream_t st);
hipError_t lcrc_launch_tbl_content(lcrc_tblk_dev* blk, uint64_t n, const uint8_t* fstatus, uint32_t* unsorted,
                                   uint32_t gen, const uint64_t* n_dev, hipStream_t st);
hipError_t lcrc_launch_gather_u8(const uint8_t* base, const uint64_t* pos, uint64_t n, uint8_t* out, hipStream_t st);
hipError_t lcrc_launch_store_crc(uint8_t* base, uint64_t base_len, const lcrc_desc_dev* descs, const uint32_t* crc, uint64_t n,
                                 hipStream_t st);
}

static_assert(sizeof(lcrc_desc) == sizeof(lcrc_desc_dev), "desc layout");
static_assert(sizeof(lcrc_wal_rec) == sizeof(lcrc_wal_rec_dev), "wal rec layout");
static_assert(sizeof(lcrc_tblk) == sizeof(lcrc_tblk_dev), "table block layout");

namespace {

thread_local std::string g_last_error;

int fail_hip(hipError_t e, const char* what) {
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  if (e == hipErrorOutOfMemory) return LCRC_ENOMEM;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice || e == hipErrorNoBinaryForGpu ||
      e == hipErrorInvalidDeviceFunction)
    return LCRC_ENODEV;
  return LCRC_EHIP;
}

#define HIPCHK(expr)                                  \
  do {                                                \
    hipError_t _e = (expr);                           \
    if (_e != hipSuccess) return fail_hip(_e, #expr); \
  } while (0)

// Device buffer that grows on demand (reserve() up front keeps the hot calls allocation-free).
template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;  // elements
  int ensure(size_t n) {
    if (n <= cap) return LCRC_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n, 1024);
    HIPCHK(hipMalloc(&p, want * sizeof(T)));
    cap = want;
    return LCRC_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

}  // namespace

struct lcrc_ctx {
  int device = 0;
  int mode = LCRC_MODE_C;
  uint32_t flags = 0;
  hipStream_t stream = nullptr;
  hipStream_t copy_stream = nullptr;
  hipEvent_t t0 = nullptr, t1 = nullptr;
  bool tk_start = false, tk_stop = false, tk_any = false;  // lcrc_timer_kernels: launches that record t0 / t1
  bool tk_end = false;  // a launch after edge 1 recorded t1
  bool tk_armed0 = false;  // edge 0 armed since the last lcrc_timer_start: t0 is valid only once a launch recorded it
  uint32_t* d_tab = nullptr;
  uint32_t init = lcrc::CRC_INIT, xorout = lcrc::CRC_XOROUT, fin4096 = 0;
  uint32_t poly = 0, x4096 = 0;  // this mode's polynomial and x^(8*4096) mod P (k_ranges' chunk shift)
  int general = 0;  // general path: 0 auto (k_ranges for uniform one-chunk layouts), 1 k_ranges, 2 k_windows + k_blocks
  int grid_a = 256, grid_b = 1024;
  DevBuf<uint32_t> win;       // window partials for the general path
  DevBuf<uint32_t> win2;      // lcrc_batch_queue: the second window buffer (batches alternate)
  hipStream_t side = nullptr, side2 = nullptr;  // the two lanes of the queued calls (lcrc_*_queue)
  hipEvent_t q_fork = nullptr, q_join = nullptr, q_join2 = nullptr;
  hipEvent_t x_join = nullptr;  // lcrc_ctx_join: this context's stream as seen by another context
  DevBuf<uint8_t> chunk[2];   // host-resident pipeline staging
  DevBuf<uint32_t> hexp[2];   // expected values per chunk
  hipEvent_t ev_copied[2] = {nullptr, nullptr}, ev_done[2] = {nullptr, nullptr};
  DevBuf<uint64_t> wal_offsets;
  DevBuf<lcrc_desc_dev> wal_descs;
  DevBuf<uint32_t> wal_crcs;
  DevBuf<uint32_t> wal_counts;
  DevBuf<uint2> wal_slots;
  DevBuf<uint8_t> wal_stops;
  // lcrc_batch_multi: this context's shard (the byte span its descriptors cover, the rebased descriptors,
  // CRCs and mismatch words)
  DevBuf<uint8_t> ms_data;
  DevBuf<lcrc_desc_dev> ms_desc;
  DevBuf<uint32_t> ms_out, ms_mm;
  // lcrc_wal_scan_queue: one workspace per log of a submission (header walk, records, window values)
  struct WalWs {
    DevBuf<uint32_t> counts;
    DevBuf<uint2> slots;
    DevBuf<uint8_t> stops;
    DevBuf<uint64_t> offsets;
    DevBuf<lcrc_desc_dev> descs;
    DevBuf<uint32_t> crcs, win;
  };
  std::vector<WalWs> wq;
  uint64_t* h_count = nullptr;  // pinned, 8 words: [0] record count of the synchronous WAL scan, [1..3] table
                                // scan staging, [4..6] Snappy totals and maxima, [7] table scan order flag
  // Snappy frames: chunk CRCs are CRC-32C whatever the context's mode
  uint32_t* d_tab_c = nullptr;  // CRC-32C image when mode != C (created on first use)
  DevBuf<uint64_t> sn_size, sn_nch, sn_choff, sn_part;
  DevBuf<uint32_t> sn_max;  // largest compressed / decoded chunk of a batch (sizes the decode's LDS)
  DevBuf<lcrc_desc_dev> sn_cdesc;
  DevBuf<uint32_t> sn_cexp, sn_cframe, sn_ccrc;
  DevBuf<uint32_t> sn_cmm;  // the table scan's chunk mismatch bits (set or cleared by the CRC pass)
  DevBuf<uint64_t> sn_out_off;  // table scan: frame output offsets
  DevBuf<lcrc_tblk_dev> tbl_blk;  // table scan on the device: the blocks being assembled
  DevBuf<uint32_t> tbl_flag;      // = tbl_gen when that scan's blocks are out of offset order
  uint32_t tbl_gen = 0;
  DevBuf<uint64_t> idx_count, idx_flag, idx_pos, idx_fpos;
  DevBuf<lcrc_desc_dev> tbl_frames;
  DevBuf<uint8_t> sn_out, sn_status;
  DevBuf<lcrc_desc_dev> tbl_descs;  // table scan / seal
  DevBuf<uint32_t> tbl_crcs, tbl_mm;
  DevBuf<uint64_t> tbl_pos;
  DevBuf<uint8_t> tbl_types;
  // asynchronous table scan: its device state, the result staging of the synchronous wrapper, capacities
  DevBuf<lcrc_tscan_dev> ts_state;
  DevBuf<uint8_t> ts_idx;    // table scan: a Snappy-framed index block decoded on the device (k_ts_open)
  DevBuf<uint64_t> ts_open;  // k_ts_open's verdict words (zeroed when allocated)
  DevBuf<uint64_t> ts_agg;   // k_ts_windows' index workgroups: their entry counts, done count and ticket (zeroed when
                             // allocated; the last ticket zeroes them again)
  DevBuf<uint32_t> ts_open_scr;  // k_ts_open2's per-workgroup source arrays (pointer jumping)
  DevBuf<lcrc_tblk_dev> ts_blocks;
  DevBuf<uint64_t> ts_count;
  uint32_t* ts_count_status = nullptr;  // device: the async scan's status words (synchronous wrapper)
  void* ts_host = nullptr;              // pinned: the state read back by the synchronous wrapper
  uint64_t ts_decoded_cap = 0;
  uint64_t ts_out_cap = 0;  // the decode workspace: ts_decoded_cap + the 16-alignment of its (large) chunks
  // lcrc_ctx_options (lcrc_ctx_create_ex; tests and measurement only -- the library reads no environment variable)
  uint32_t ts_grid = 4096;  // the table scan's index/emit grid cap (tests reach the tile loops with a small one)
  // k_blocks grid divisor of the table scan (0: 1). With the index walk beside the window pass (k_ts_windows) the
  // full grid is faster both alone (79.6 against 81.4 us) and on two streams (3,521-3,543 against 3,416-3,436 GiB/s)
  int ts_blocks_div = 0;
  uint32_t batch_grid_b = 0;  // lcrc_batch's k_blocks grid (0: 2 per CU)
  uint32_t wal_grid_b = 0;    // the WAL scan's k_blocks grid (0: every resident workgroup)
};

namespace {

// Kernel-carried timing (lcrc_timer_kernels) for the multi-kernel calls: while the OUTERMOST timed API call of a
// context runs, every launch it makes carries the context's armed events (the first launch the start, each launch
// the stop: the last one wins). Nested API calls (lcrc_batch_seal -> lcrc_batch) share the outer scope.
thread_local int g_tk_depth = 0;
struct TkScope {
  lcrc_ctx* c;
  bool outer;
  explicit TkScope(lcrc_ctx* ctx) : c(ctx), outer(ctx && g_tk_depth == 0) {
    ++g_tk_depth;
    if (outer) lcrc_launch_events_begin(c->tk_start ? c->t0 : nullptr, c->tk_stop ? c->t1 : nullptr);
  }
  ~TkScope() {
    --g_tk_depth;
    if (!outer) return;
    bool started = false, stopped = false;
    lcrc_launch_events_end(&started, &stopped);
    if (started) {
      c->tk_any = true;
      c->tk_start = false;
    }
    if (stopped) c->tk_end = true;
  }
};

// The per-mode constant image (TAB_* layout, lcrc_device.h), uploaded to a new device allocation.
int upload_tables(int mode, uint32_t** d_tab) {
  const uint32_t poly = lcrc::poly_of(mode);
  std::vector<uint32_t> tab(TAB_TOTAL);
  lcrc::make_slice_tables(poly, tab.data() + TAB_SLICE, 4);
  for (int m = 0; m < 4; ++m) lcrc::make_shift_tables(poly, 16ull << m, tab.data() + TAB_ZPIECE + m * 1024);
  for (int m = 0; m < 4; ++m) lcrc::make_shift_tables(poly, 256ull << m, tab.data() + TAB_ZWIN + m * 1024);
  lcrc::make_shift_tables(poly, 4096, tab.data() + TAB_Z4096);
  lcrc::make_shift_tables(poly, LCRC_TS_PIECE, tab.data() + TAB_Z64K);
  // k_windows builds its LDS image from columns (entries 1, 2, 4, .., 128) of the byte tables it uses
  for (int t = 0; t < 20; ++t) {
    const uint32_t src = t < 4 ? TAB_SLICE + t * 256                    // S0: T_p
                         : t < 8 ? TAB_ZPIECE + 2048 + (7 - t) * 256      // S1: Z64[3 - p], p = t - 4
                                 : TAB_ZWIN + (t - 8) * 256;              // Z256, Z512, Z1024
    for (int i = 0; i < 8; ++i) tab[TAB_COLS + t * 8 + i] = tab[src + (1u << i)];
  }
  // the queued fast path's per-window shifts to the block end: Z_{256 k} of byte q, by columns
  for (int k = 0; k < 16; ++k) {
    const uint32_t xp = lcrc::x8n(256ull * k, poly);
    for (int q = 0; q < 4; ++q)
      for (int i = 0; i < 8; ++i)
        tab[TAB_SCOLS + (4 * k + q) * 8 + i] = lcrc::multmodp(xp, 1u << (8 * q + i), poly);
  }
  // inverses of the zero-byte shifts for k_ranges: x^-1 = (P - 1) / x, i.e. (poly << 1) | 1 reflected
  const uint32_t xinv = (poly << 1) | 1u;
  if (lcrc::multmodp(xinv, 1u << 30, poly) != (1u << 31)) return LCRC_EINVAL;  // x * x^-1 == 1
  uint32_t xinv8 = 1u << 31;
  for (int i = 0; i < 8; ++i) xinv8 = lcrc::multmodp(xinv8, xinv, poly);
  tab[TAB_INV] = 1u << 31;
  for (int k = 1; k <= 4096; ++k) tab[TAB_INV + k] = lcrc::multmodp(tab[TAB_INV + k - 1], xinv8, poly);
  const uint32_t x4096 = lcrc::x8n(4096, poly);
  tab[TAB_XCH] = 1u << 31;
  for (int k = 1; k < 4096; ++k) tab[TAB_XCH + k] = lcrc::multmodp(tab[TAB_XCH + k - 1], x4096, poly);
  HIPCHK(hipMalloc(d_tab, TAB_TOTAL * sizeof(uint32_t)));
  HIPCHK(hipMemcpy(*d_tab, tab.data(), TAB_TOTAL * sizeof(uint32_t), hipMemcpyHostToDevice));
  return LCRC_OK;
}

int set_device(lcrc_ctx* ctx) {
  HIPCHK(hipSetDevice(ctx->device));
  return LCRC_OK;
}

hipStream_t pick_stream(lcrc_ctx* ctx, void* stream) { return stream ? (hipStream_t)stream : ctx->stream; }

// A newly allocated word array the kernels expect zero (tickets, look-back words), zeroed and FINISHED before any
// later launch on any stream: hipMemset goes to the null stream, which the contexts' non-blocking streams do not wait
// for, and a freshly allocated buffer may hold a freed one's bytes
hipError_t zero_now(lcrc_ctx* ctx, void* p, size_t bytes) {
  hipError_t e = hipMemsetAsync(p, 0, bytes, ctx->stream);
  return e != hipSuccess ? e : hipStreamSynchronize(ctx->stream);
}

}  // namespace

extern "C" {

const char* lcrc_last_error(void) { return g_last_error.c_str(); }
#ifndef LCRC_SRC_HASH
#define LCRC_SRC_HASH "unknown"
#endif
const char* lcrc_version(void) {
  return "lcrc 0.2 src " LCRC_SRC_HASH " (gfx950: k_windows slice4x32-LDS + DPP16 transpose, queued batches, k_blocks row16)";
}

int lcrc_device_count(int* n) {
  if (!n) return LCRC_EINVAL;
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *n = 0;
    return fail_hip(e, "hipGetDeviceCount");
  }
  *n = c;
  return c > 0 ? LCRC_OK : LCRC_ENODEV;
}

int lcrc_device_pci_bus_id(int device, char* out, int len) {
  if (!out || len < 13) return LCRC_EINVAL;
  const hipError_t e = hipDeviceGetPCIBusId(out, len, device);
  if (e != hipSuccess) {
    out[0] = 0;
    return fail_hip(e, "hipDeviceGetPCIBusId");
  }
  return LCRC_OK;
}

int lcrc_ctx_create(lcrc_ctx** out, int device, int mode, uint32_t flags) {
  return lcrc_ctx_create_ex(out, device, mode, flags, nullptr);
}

int lcrc_ctx_create_ex(lcrc_ctx** out, int device, int mode, uint32_t flags, const lcrc_ctx_options* opt) {
  if (!out || (mode != LCRC_MODE_REF && mode != LCRC_MODE_C)) return LCRC_EINVAL;
  // (a caller built against the round-4 header passes the struct without the reserved words: accepted)
  if (opt && (opt->size < offsetof(lcrc_ctx_options, reserved) || opt->general < 0 || opt->general > 2))
    return LCRC_EINVAL;
  for (size_t k = 0; opt && k < 3; ++k)
    if (opt->size >= offsetof(lcrc_ctx_options, reserved) + (k + 1) * sizeof(uint32_t) && opt->reserved[k]) {
      g_last_error = "lcrc_ctx_options.reserved: must be 0 (the round-5 variants wal_onepass, ts_open_v1 and "
                     "ts_unfused are no longer in the library)";
      return LCRC_EINVAL;
    }
  *out = nullptr;
  int ndev = 0;
  int rc = lcrc_device_count(&ndev);
  if (rc != LCRC_OK) return LCRC_ENODEV;
  if (device < 0 || device >= ndev) return LCRC_EINVAL;
  lcrc_ctx* ctx = new lcrc_ctx();
  ctx->device = device;
  ctx->mode = mode;
  ctx->flags = flags;
  auto bail = [&](int code) {
    lcrc_ctx_destroy(ctx);
    return code;
  };
  if ((rc = set_device(ctx)) != LCRC_OK) return bail(rc);
  hipDeviceProp_t prop;
  hipError_t e = hipGetDeviceProperties(&prop, device);
  if (e != hipSuccess) return bail(fail_hip(e, "hipGetDeviceProperties"));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    g_last_error = std::string("kernels are built for gfx950 only; device is ") + prop.gcnArchName;
    return bail(LCRC_ENODEV);
  }
  ctx->grid_a = prop.multiProcessorCount;      // k_windows: CUs (the launcher scales by workgroups per CU)
  // k_blocks (40 KiB LDS, 512-thread workgroups): up to 4 per CU. lcrc_batch launches 2 per CU so that the
  // next batch's k_windows workgroups (76 KiB) fit beside them (config 3 on two streams: 4,198 GiB/s against
  // 3,681 with 4 per CU, at +4 % per launch alone); the WAL scan, whose k_blocks follows its own window
  // pass, uses all 4.
  ctx->grid_b = prop.multiProcessorCount * lcrc_blocks_per_cu();  // k_blocks: every resident workgroup
  if ((e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)) != hipSuccess)
    return bail(fail_hip(e, "hipStreamCreate"));
  // (the copy stream of lcrc_batch_host_uniform is created on its first call, as the queue lanes)
#ifdef LCRC_EAGER_STREAMS  // measurement build: every stream at creation, as before round 2's last changes
  for (hipStream_t* l : {&ctx->copy_stream, &ctx->side, &ctx->side2})
    if ((e = hipStreamCreateWithFlags(l, hipStreamNonBlocking)) != hipSuccess) return bail(fail_hip(e, "hipStreamCreate"));
#endif
  if ((e = hipEventCreate(&ctx->t0)) != hipSuccess || (e = hipEventCreate(&ctx->t1)) != hipSuccess)
    return bail(fail_hip(e, "hipEventCreate"));
  for (int i = 0; i < 2; ++i)
    if ((e = hipEventCreateWithFlags(&ctx->ev_copied[i], hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&ctx->ev_done[i], hipEventDisableTiming)) != hipSuccess)
      return bail(fail_hip(e, "hipEventCreate"));
  // (the queue lanes' streams are created on first use, ensure_lanes: every stream a context creates takes one of
  // the process's few hardware queues, and two contexts' main streams sharing one serialize)
  for (hipEvent_t* ev : {&ctx->q_fork, &ctx->q_join, &ctx->q_join2, &ctx->x_join})
    if ((e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess) return bail(fail_hip(e, "hipEventCreate"));
  if ((e = hipHostMalloc(&ctx->h_count, 8 * sizeof(uint64_t), hipHostMallocDefault)) != hipSuccess)
    return bail(fail_hip(e, "hipHostMalloc"));
  if ((e = hipHostMalloc(&ctx->ts_host, sizeof(lcrc_tscan_dev), hipHostMallocDefault)) != hipSuccess)
    return bail(fail_hip(e, "hipHostMalloc"));
  if ((e = hipMalloc(&ctx->ts_count_status, 4 * sizeof(uint32_t))) != hipSuccess) return bail(fail_hip(e, "hipMalloc"));

  // constant tables for this mode
  const uint32_t poly = lcrc::poly_of(mode);
  if ((rc = upload_tables(mode, &ctx->d_tab)) != LCRC_OK) return bail(rc);
  ctx->fin4096 = lcrc::zshift(ctx->init, 4096, poly) ^ ctx->xorout;
  ctx->poly = poly;
  ctx->x4096 = lcrc::x8n(4096, poly);
  if (opt) {
    ctx->general = opt->general;
    ctx->batch_grid_b = opt->batch_grid_b;
    ctx->wal_grid_b = opt->wal_grid_b;
    if (opt->ts_grid) ctx->ts_grid = opt->ts_grid;
    if (opt->ts_blocks_div) ctx->ts_blocks_div = (int)opt->ts_blocks_div;
  }
  *out = ctx;
  return LCRC_OK;
}

int lcrc_ctx_destroy(lcrc_ctx* ctx) {
  if (!ctx) return LCRC_OK;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->copy_stream) (void)hipStreamSynchronize(ctx->copy_stream);
  for (hipStream_t l : {ctx->side, ctx->side2})
    if (l) (void)hipStreamSynchronize(l);
  ctx->win.release();
  ctx->win2.release();
  for (hipEvent_t ev : {ctx->q_fork, ctx->q_join, ctx->q_join2, ctx->x_join})
    if (ev) (void)hipEventDestroy(ev);
  for (int i = 0; i < 2; ++i) {
    ctx->chunk[i].release();
    ctx->hexp[i].release();
    if (ctx->ev_copied[i]) (void)hipEventDestroy(ctx->ev_copied[i]);
    if (ctx->ev_done[i]) (void)hipEventDestroy(ctx->ev_done[i]);
  }
  ctx->wal_offsets.release();
  ctx->wal_descs.release();
  ctx->wal_crcs.release();
  ctx->wal_counts.release();
  ctx->wal_slots.release();
  ctx->wal_stops.release();
  ctx->ms_data.release();
  ctx->ms_desc.release();
  ctx->ms_out.release();
  ctx->ms_mm.release();
  for (auto& w : ctx->wq)
    for (auto* d : {&w.counts, &w.crcs, &w.win}) d->release();
  for (auto& w : ctx->wq) {
    w.slots.release();
    w.stops.release();
    w.offsets.release();
    w.descs.release();
  }
  if (ctx->h_count) (void)hipHostFree(ctx->h_count);
  if (ctx->d_tab_c) (void)hipFree(ctx->d_tab_c);
  for (auto* b : {&ctx->sn_size, &ctx->sn_nch, &ctx->sn_choff, &ctx->sn_part, &ctx->sn_out_off}) b->release();
  ctx->sn_max.release();
  for (auto* b : {&ctx->sn_cexp, &ctx->sn_cframe, &ctx->sn_ccrc, &ctx->sn_cmm}) b->release();
  ctx->sn_cdesc.release();
  ctx->tbl_blk.release();
  ctx->tbl_flag.release();
  for (auto* b : {&ctx->idx_count, &ctx->idx_flag, &ctx->idx_pos, &ctx->idx_fpos}) b->release();
  ctx->tbl_frames.release();
  ctx->sn_out.release();
  ctx->sn_status.release();
  ctx->tbl_descs.release();
  ctx->tbl_crcs.release();
  ctx->tbl_mm.release();
  ctx->tbl_pos.release();
  ctx->tbl_types.release();
  ctx->ts_state.release();
  ctx->ts_idx.release();
  ctx->ts_open.release();
  ctx->ts_agg.release();
  ctx->ts_open_scr.release();
  ctx->ts_blocks.release();
  ctx->ts_count.release();
  if (ctx->ts_host) (void)hipHostFree(ctx->ts_host);
  if (ctx->ts_count_status) (void)hipFree(ctx->ts_count_status);
  if (ctx->d_tab) (void)hipFree(ctx->d_tab);
  if (ctx->t0) (void)hipEventDestroy(ctx->t0);
  if (ctx->t1) (void)hipEventDestroy(ctx->t1);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->copy_stream) (void)hipStreamDestroy(ctx->copy_stream);
  for (hipStream_t l : {ctx->side, ctx->side2})
    if (l) (void)hipStreamDestroy(l);
  delete ctx;
  return LCRC_OK;
}

void* lcrc_ctx_stream(lcrc_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

// ctx's stream waits (on the device) for everything enqueued on other's stream so far
int lcrc_ctx_join(lcrc_ctx* ctx, lcrc_ctx* other) {
  if (!ctx || !other) return LCRC_EINVAL;
  if (ctx == other) return LCRC_OK;
  HIPCHK(hipEventRecord(other->x_join, other->stream));
  HIPCHK(hipStreamWaitEvent(ctx->stream, other->x_join, 0));
  return LCRC_OK;
}

int lcrc_ctx_sync(lcrc_ctx* ctx) {
  if (!ctx) return LCRC_EINVAL;
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return LCRC_OK;
}

static size_t lcrc_wal_queue_max() { return 16; }  // MAX_WJOBS in lcrc_kernels.hip
#ifndef LCRC_WAL_GRID_DIV
#define LCRC_WAL_GRID_DIV 1  // the WAL scan's range pass: the full grid (half: 100.6 vs 96.2 us per launch, same 2-stream wall)
#endif
#ifndef LCRC_WALQ_WG_PER_CU
#define LCRC_WALQ_WG_PER_CU 2  // range-pass workgroups per CU beside a window pass (its 76 KiB workgroup must fit)
#endif

static uint64_t window_words(uint64_t span) { return ((span + 16383) / 16384) * 64; }

// the two queue lanes (ctx->side, ctx->side2), created on the first queued call. Created with every context, four
// streams per context made two contexts' main streams share a hardware queue (GPU_MAX_HW_QUEUES = 4 here): the
// table bench's two scanners ran one after the other, 110 vs 86 us per scan.
static int ensure_lanes(lcrc_ctx* ctx) {
  for (hipStream_t* l : {&ctx->side, &ctx->side2})
    if (!*l) HIPCHK(hipStreamCreateWithFlags(l, hipStreamNonBlocking));
  return LCRC_OK;
}

// `st` waits for both queue lanes (ctx->side, ctx->side2)
static int lanes_join(lcrc_ctx* ctx, hipStream_t st) {
  HIPCHK(hipEventRecord(ctx->q_join, ctx->side));
  HIPCHK(hipStreamWaitEvent(st, ctx->q_join, 0));
  HIPCHK(hipEventRecord(ctx->q_join2, ctx->side2));
  HIPCHK(hipStreamWaitEvent(st, ctx->q_join2, 0));
  return LCRC_OK;
}

// `st` waits for both lanes; a timer stop event armed for the call (lcrc_timer_kernels edge 1) was taken from the
// lane launches (held_stop, lcrc_launch_events_swap_stop) and is recorded here, after the join, so that it closes
// over whichever lane ends last
static int lanes_join_timed(lcrc_ctx* ctx, hipStream_t st, hipEvent_t held_stop) {
  int rc = lanes_join(ctx, st);
  lcrc_launch_events_swap_stop(held_stop);
  if (rc) return rc;
  if (held_stop) HIPCHK(lcrc_launch_events_record_stop(held_stop, st));
  return LCRC_OK;
}

int lcrc_ctx_reserve(lcrc_ctx* ctx, uint64_t max_span) {
  if (!ctx) return LCRC_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  if ((rc = ctx->win.ensure(window_words(max_span)))) return rc;
  return ctx->win2.ensure(window_words(max_span));  // lcrc_batch_queue's second window buffer
}

#ifndef LCRC_BATCH_WG_PER_CU
#define LCRC_BATCH_WG_PER_CU 2  // 16 waves per CU: a full 32-wave grid cut config 3 k_blocks alone 22.0 -> 18.0 us but
                                // crowded a concurrent batch on another stream (2-stream wall 4.1-4.3K -> 3.8K GiB/s)
#endif
int lcrc_batch(lcrc_ctx* ctx, const uint8_t* base, uint64_t base_len, const lcrc_desc* descs, size_t n,
               uint32_t* out_crc, uint32_t* out_mismatch, void* stream) {
  TkScope tk_scope(ctx);
  if (!ctx || (n && (!descs || !out_crc || !base))) return LCRC_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  hipStream_t st = pick_stream(ctx, stream);
  if (n == 0) return LCRC_OK;
  // no fill of out_mismatch: every range sets or clears its own bit (LCRC_KFLAG_SETCLR)
  const uint32_t kflags = (ctx->flags & LCRC_FLAG_MASK) | LCRC_KFLAG_SETCLR;
  const bool direct = (ctx->flags & LCRC_FLAG_DIRECT) != 0;
  if (!direct && ctx->general == 1) {
    HIPCHK(lcrc_launch_ranges(false, ctx->grid_a, base, base_len, (const lcrc_desc_dev*)descs, n, 0, 0, nullptr,
                              ctx->d_tab, ctx->x4096, ctx->poly, ctx->init, ctx->xorout, kflags,
                              out_crc, out_mismatch, nullptr, nullptr, st));
    return LCRC_OK;
  }
  const uint32_t* win = nullptr;
  if (!direct && base_len) {
    if ((rc = ctx->win.ensure(window_words(base_len))) != LCRC_OK) return rc;
    HIPCHK(lcrc_launch_windows(false, ctx->grid_a, base, base_len, ctx->d_tab, ctx->win.p, 0, 0, 0, nullptr, nullptr,
                               st));
    win = ctx->win.p;
  }
  const uint32_t gb = ctx->batch_grid_b ? ctx->batch_grid_b : std::min(ctx->grid_b, ctx->grid_a * LCRC_BATCH_WG_PER_CU);
  HIPCHK(lcrc_launch_blocks(false, gb, base, base_len, (const lcrc_desc_dev*)descs, n, 0, 0, nullptr, win,
                            ctx->d_tab, ctx->init, ctx->xorout, kflags, out_crc,
                            out_mismatch, nullptr, nullptr, st));
  return LCRC_OK;
}

// The general path over a queue of batches on two lanes: the side streams take alternate batches, each
// running a batch's window pass and then its range pass, so the lanes' window passes share the HBM stream and
// then their latency-bound range passes run together -- the schedule two contexts on two streams settle into,
// the best of those measured (per step, config 3: two contexts 56 us, one stream 63.5 us; window passes back
// to back on one stream with each range pass forked beside the next window pass 70-77 us: beside a window
// pass the range pass runs three times slower and slows the window pass by 15-30 %). The lanes' fork and join
// cost ~35 us per call and an odd batch runs alone (5 batches per call: 65 us per batch).
// The lanes first wait for everything enqueued on `stream` before the call, and `stream` waits for both
// lanes before anything enqueued after it: a fork and a join, so the call behaves as its batches would one
// after another on `stream` (and captures into a graph as two branches).
int lcrc_batch_queue(lcrc_ctx* ctx, const lcrc_gjob* jobs, size_t njobs, void* stream) {
  TkScope tk_scope(ctx);
  if (!ctx || (njobs && !jobs)) return LCRC_EINVAL;
  for (size_t k = 0; k < njobs; ++k)
    if (jobs[k].n && (!jobs[k].descs || !jobs[k].out_crc || !jobs[k].base)) return LCRC_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  hipStream_t st = pick_stream(ctx, stream);
  const bool direct = (ctx->flags & LCRC_FLAG_DIRECT) != 0;
  if (direct || ctx->general == 1 || njobs < 2) {  // one pass per batch (or nothing to pipeline)
    for (size_t k = 0; k < njobs; ++k)
      if ((rc = lcrc_batch(ctx, jobs[k].base, jobs[k].base_len, jobs[k].descs, jobs[k].n, jobs[k].out_crc,
                           jobs[k].out_mismatch, st)))
        return rc;
    return LCRC_OK;
  }
  uint64_t span = 0;
  for (size_t k = 0; k < njobs; ++k) span = std::max(span, jobs[k].base_len);
  if ((rc = ctx->win.ensure(window_words(span))) || (rc = ctx->win2.ensure(window_words(span)))) return rc;
  uint32_t* wins[2] = {ctx->win.p, ctx->win2.p};
  if ((rc = ensure_lanes(ctx))) return rc;
  hipStream_t lane[2] = {ctx->side, ctx->side2};
  const int grid_b = std::min(ctx->grid_b, ctx->grid_a * LCRC_BATCH_WG_PER_CU);
  HIPCHK(hipEventRecord(ctx->q_fork, st));
  for (hipStream_t l : lane) HIPCHK(hipStreamWaitEvent(l, ctx->q_fork, 0));
  hipEvent_t held_stop = lcrc_launch_events_swap_stop(nullptr);  // recorded after the join (lanes_join_timed)
  for (size_t k = 0; k < njobs; ++k) {
    const lcrc_gjob& j = jobs[k];
    const int b = (int)(k & 1);
    if (j.n && j.base_len)
      HIPCHK(lcrc_launch_windows(false, ctx->grid_a, j.base, j.base_len, ctx->d_tab, wins[b], 0, 0, 0, nullptr,
                                 nullptr, lane[b]));
    HIPCHK(lcrc_launch_blocks(false, grid_b, j.base, j.base_len, (const lcrc_desc_dev*)j.descs, j.n, 0, 0, nullptr,
                              j.base_len ? wins[b] : nullptr, ctx->d_tab, ctx->init, ctx->xorout,
                              (ctx->flags & LCRC_FLAG_MASK) | LCRC_KFLAG_SETCLR, j.out_crc, j.out_mismatch, nullptr,
                              nullptr, lane[b]));
  }
  return lanes_join_timed(ctx, st, held_stop);
}

int lcrc_batch_covered(lcrc_ctx* ctx, const uint8_t* base, uint64_t base_len, const lcrc_desc* descs, size_t n,
                       uint64_t covered_bytes, uint32_t* out_crc, uint32_t* out_mismatch, void* stream) {
  if (!ctx || (n && (!descs || !out_crc || !base))) return LCRC_EINVAL;
  // sparse: the window pass would stream all of base_len for a small fraction of it
  if (covered_bytes == 0 || covered_bytes >= base_len / 4 || (ctx->flags & LCRC_FLAG_DIRECT))
    return lcrc_batch(ctx, base, base_len, descs, n, out_crc, out_mismatch, stream);
  int rc = set_device(ctx);
  if (rc) return rc;
  hipStream_t st = pick_stream(ctx, stream);
  if (n == 0) return LCRC_OK;
  // a few ranges: one wave's four rows per workgroup, so the walks spread over the CUs instead of sharing a
  // few CUs' VALU and LDS eight waves apiece
  HIPCHK(lcrc_launch_ranges(false, ctx->grid_a, base, base_len, (const lcrc_desc_dev*)descs, n, 0, 0, nullptr,
                            ctx->d_tab, ctx->x4096, ctx->poly, ctx->init, ctx->xorout,
                            (ctx->flags & LCRC_FLAG_MASK) | LCRC_KFLAG_SETCLR, out_crc, out_mismatch, nullptr, nullptr,
                            st, 4));
  return LCRC_OK;
}

static int batch_uniform_impl(lcrc_ctx* ctx, const uint8_t* base, size_t n, uint32_t length, uint64_t stride,
                              const uint32_t* expected, uint32_t* out_crc, uint32_t* out_mismatch, hipStream_t st,
                              bool clear_mismatch) {
  if (out_mismatch && n && clear_mismatch)
    HIPCHK(hipMemsetAsync(out_mismatch, 0, ((n + 31) / 32) * sizeof(uint32_t), st));
  if (n == 0) return LCRC_OK;
  const uint32_t mflags = ctx->flags & LCRC_FLAG_MASK;
  if (length == 4096 && stride == 4096) {
    // single pass: k_windows folds each 4 KiB block and writes the final CRC
    // kernel-carried timing (lcrc_timer_kernels), as in lcrc_batch_uniform_queue
    hipEvent_t ts = ctx->tk_start ? ctx->t0 : nullptr, te = ctx->tk_stop ? ctx->t1 : nullptr;
    HIPCHK(lcrc_launch_windows(true, ctx->grid_a, base, (uint64_t)n * 4096, ctx->d_tab, out_crc, n, ctx->fin4096,
                               mflags, expected, out_mismatch, st, ts, te));
    if (ts) ctx->tk_any = true;
    if (te) ctx->tk_end = true;
    ctx->tk_start = false;
    return LCRC_OK;
  }
  const uint64_t span = (uint64_t)(n - 1) * stride + length;
  // k_ranges walks whole 4 KiB chunks: it wins when every range is one well-filled chunk (measured,
  // tools/probe/ranges_time.py: 4092/4096 B 53 vs 65 us, sparse 4096/8192 B 31 vs 55 us per launch) and
  // loses on short or multi-chunk ranges (512 B 50 vs 34, 4097 B 91 vs 67, 64 KiB 107 vs 54)
  // (a range just past one chunk -- 4,097 B blocks -- walks its last bytes on at the end: 71 vs 67 us, kept out)
  const bool one_chunk = length >= 2048 && length + (stride & 3 ? 3u : 0u) <= 4096;
  if (!(ctx->flags & LCRC_FLAG_DIRECT) && (ctx->general == 1 || (ctx->general == 0 && one_chunk))) {
    HIPCHK(lcrc_launch_ranges(true, ctx->grid_a, base, span, nullptr, n, stride, length, expected, ctx->d_tab,
                              ctx->x4096, ctx->poly, ctx->init, ctx->xorout, mflags, out_crc, out_mismatch, nullptr,
                              nullptr, st));
    return LCRC_OK;
  }
  const uint32_t* win = nullptr;
  if (!(ctx->flags & LCRC_FLAG_DIRECT) && span) {
    int rc = ctx->win.ensure(window_words(span));
    if (rc) return rc;
    HIPCHK(lcrc_launch_windows(false, ctx->grid_a, base, span, ctx->d_tab, ctx->win.p, 0, 0, 0, nullptr, nullptr,
                               st));
    win = ctx->win.p;
  }
  HIPCHK(lcrc_launch_blocks(true, ctx->grid_b, base, span, nullptr, n, stride, length, expected, win, ctx->d_tab,
                            ctx->init, ctx->xorout, mflags, out_crc, out_mismatch, nullptr, nullptr, st));
  return LCRC_OK;
}

int lcrc_batch_uniform(lcrc_ctx* ctx, const uint8_t* base, size_t n, uint32_t length, uint64_t stride,
                       const uint32_t* expected, uint32_t* out_crc, uint32_t* out_mismatch, void* stream) {
  if (!ctx || (n && (!base || !out_crc))) return LCRC_EINVAL;
  if (n > 1 && stride < length) return LCRC_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  return batch_uniform_impl(ctx, base, n, length, stride, expected, out_crc, out_mismatch, pick_stream(ctx, stream),
                            true);
}

int lcrc_batch_uniform_queue(lcrc_ctx* ctx, const lcrc_ujob* jobs, size_t njobs, uint32_t length, uint64_t stride,
                             void* stream) {
  if (!ctx || (njobs && !jobs)) return LCRC_EINVAL;
  for (size_t k = 0; k < njobs; ++k)
    if ((jobs[k].n && (!jobs[k].base || !jobs[k].out_crc)) || (jobs[k].n > 1 && stride < length)) return LCRC_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  hipStream_t st = pick_stream(ctx, stream);
  if (!(length == 4096 && stride == 4096)) {
    for (size_t k = 0; k < njobs; ++k)
      if ((rc = batch_uniform_impl(ctx, jobs[k].base, jobs[k].n, length, stride, jobs[k].expected, jobs[k].out_crc,
                                   jobs[k].out_mismatch, st, true)))
        return rc;
    return LCRC_OK;
  }
#ifndef LCRC_MAX_QJOBS
#define LCRC_MAX_QJOBS 32
#endif
  lcrc_qjob_host q[LCRC_MAX_QJOBS];
  size_t k = 0;
  while (k < njobs) {
    uint32_t m = 0;
    for (; k < njobs && m < LCRC_MAX_QJOBS; ++k) {
      const lcrc_ujob& j = jobs[k];
      if (j.out_mismatch && j.n) HIPCHK(hipMemsetAsync(j.out_mismatch, 0, ((j.n + 31) / 32) * sizeof(uint32_t), st));
      if (j.n == 0) continue;
      q[m].base = j.base;
      q[m].out = j.out_crc;
      q[m].expected = j.expected;
      q[m].mismatch = j.out_mismatch;
      q[m].nblk = j.n;
      ++m;
    }
    if (m) {
      // kernel-carried timing (lcrc_timer_kernels): the launch after edge 0 records the start event, the launches
      // after edge 1 the stop event (the last one recorded wins)
      hipEvent_t ts = ctx->tk_start ? ctx->t0 : nullptr, te = ctx->tk_stop ? ctx->t1 : nullptr;
      HIPCHK(lcrc_launch_windows_queue(ctx->grid_a, q, m, ctx->d_tab, ctx->fin4096, ctx->flags & LCRC_FLAG_MASK, st,
                                       ts, te));
      if (ts) ctx->tk_any = true;
      if (te) ctx->tk_end = true;
      ctx->tk_start = false;
    }
  }
  return LCRC_OK;
}

int lcrc_batch_host_uniform(lcrc_ctx* ctx, const uint8_t* base, size_t n, uint32_t length, uint64_t stride,
                            const uint32_t* expected, uint32_t* out_crc, uint32_t* out_mismatch, size_t chunk_bytes) {
  if (!ctx || (n && (!base || !out_crc))) return LCRC_EINVAL;
  if (n > 1 && stride < length) return LCRC_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  if (n == 0) return LCRC_OK;
  if (!ctx->copy_stream) HIPCHK(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
  if (chunk_bytes == 0) chunk_bytes = 64ull << 20;
  // blocks per chunk: a multiple of 32 so every chunk starts on a mismatch-bitmap word
  size_t bpc = std::max<size_t>(chunk_bytes / std::max<uint64_t>(stride, 1), 1);
  bpc = std::max<size_t>(32, bpc / 32 * 32);
  bpc = std::min(bpc, ((n + 31) / 32) * 32);
  const uint64_t chunk_span = (uint64_t)(bpc - 1) * stride + length;
  uint32_t* d_out = nullptr;
  uint32_t* d_mm = nullptr;
  const size_t mm_words = (n + 31) / 32;
  HIPCHK(hipMalloc(&d_out, n * sizeof(uint32_t)));
  if (out_mismatch) {
    hipError_t e = hipMalloc(&d_mm, mm_words * sizeof(uint32_t));
    if (e != hipSuccess) {
      (void)hipFree(d_out);
      return fail_hip(e, "hipMalloc");
    }
  }
  int result = LCRC_OK;
  for (int i = 0; i < 2 && result == LCRC_OK; ++i) {
    result = ctx->chunk[i].ensure(chunk_span);
    if (result == LCRC_OK && expected) result = ctx->hexp[i].ensure(bpc);
  }
  if (result == LCRC_OK && !(length == 4096 && stride == 4096) && !(ctx->flags & LCRC_FLAG_DIRECT))
    result = ctx->win.ensure(window_words(chunk_span));
  if (result == LCRC_OK && d_mm) {
    hipError_t e = hipMemsetAsync(d_mm, 0, mm_words * sizeof(uint32_t), ctx->stream);
    if (e != hipSuccess) result = fail_hip(e, "hipMemsetAsync");
  }
  const size_t nchunks = (n + bpc - 1) / bpc;
  for (size_t k = 0; k < nchunks && result == LCRC_OK; ++k) {
    const int b = (int)(k & 1);
    const size_t first = k * bpc;
    const size_t cnt = std::min(bpc, n - first);
    const uint64_t span = (uint64_t)(cnt - 1) * stride + length;
    hipError_t e;
    // the staging buffer is free once the kernel that read it two chunks ago has finished
    if (k >= 2 && (e = hipStreamWaitEvent(ctx->copy_stream, ctx->ev_done[b], 0)) != hipSuccess) {
      result = fail_hip(e, "hipStreamWaitEvent");
      break;
    }
    if ((e = hipMemcpyAsync(ctx->chunk[b].p, base + first * stride, span, hipMemcpyHostToDevice,
                            ctx->copy_stream)) != hipSuccess) {
      result = fail_hip(e, "hipMemcpyAsync");
      break;
    }
    if (expected && (e = hipMemcpyAsync(ctx->hexp[b].p, expected + first, cnt * sizeof(uint32_t),
                                        hipMemcpyHostToDevice, ctx->copy_stream)) != hipSuccess) {
      result = fail_hip(e, "hipMemcpyAsync");
      break;
    }
    if ((e = hipEventRecord(ctx->ev_copied[b], ctx->copy_stream)) != hipSuccess ||
        (e = hipStreamWaitEvent(ctx->stream, ctx->ev_copied[b], 0)) != hipSuccess) {
      result = fail_hip(e, "hipEventRecord");
      break;
    }
    result = batch_uniform_impl(ctx, ctx->chunk[b].p, cnt, length, stride, expected ? ctx->hexp[b].p : nullptr,
                                d_out + first, d_mm ? d_mm + first / 32 : nullptr, ctx->stream, false);
    if (result == LCRC_OK && (e = hipEventRecord(ctx->ev_done[b], ctx->stream)) != hipSuccess)
      result = fail_hip(e, "hipEventRecord");
  }
  if (result == LCRC_OK) {
    hipError_t e = hipMemcpyAsync(out_crc, d_out, n * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess && d_mm)
      e = hipMemcpyAsync(out_mismatch, d_mm, mm_words * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) result = fail_hip(e, "D2H");
  }
  (void)hipStreamSynchronize(ctx->stream);
  (void)hipStreamSynchronize(ctx->copy_stream);
  (void)hipFree(d_out);
  if (d_mm) (void)hipFree(d_mm);
  return result;
}

// One shard of lcrc_batch_multi on its context's device: the span [lo, hi) of the file its descriptors read
// (ranges and expected values) goes H2D, the descriptors are rebased to it, one lcrc_batch, results D2H.
static int multi_shard(lcrc_ctx* ctx, const uint8_t* base, uint64_t base_len, const lcrc_desc* descs, size_t n,
                       uint32_t* out_crc, uint32_t* out_mismatch) {
  int rc = set_device(ctx);
  if (rc) return rc;
  if (n == 0) return LCRC_OK;
  uint64_t lo = UINT64_MAX, hi = 0;
  for (size_t i = 0; i < n; ++i) {
    const lcrc_desc& d = descs[i];
    if (d.offset > base_len) continue;  // never read: out of bounds in the shard too
    lo = std::min<uint64_t>(lo, d.offset);
    hi = std::max<uint64_t>(hi, std::min<uint64_t>(base_len, d.offset + d.length));
    if (d.expect_rel != LCRC_NO_EXPECT) {
      const int64_t xp = (int64_t)d.offset + d.expect_rel;
      if (xp >= 0 && (uint64_t)xp + 4 <= base_len) {
        lo = std::min<uint64_t>(lo, (uint64_t)xp);
        hi = std::max<uint64_t>(hi, (uint64_t)xp + 4);
      }
    }
  }
  if (lo > hi) lo = hi = 0;
  const uint64_t span = hi - lo;
  std::vector<lcrc_desc_dev> rb(n);
  for (size_t i = 0; i < n; ++i) {
    // rebased: anything outside [lo, hi) stays outside [0, span) (a range past the file ends past the span, an
    // offset past the file lies past it, an expected value outside the file falls outside the span)
    rb[i].offset = descs[i].offset > base_len ? UINT64_MAX / 2 : descs[i].offset - lo;
    rb[i].length = descs[i].length;
    rb[i].expect_rel = descs[i].expect_rel;
  }
  const size_t words = (n + 31) / 32;
  if ((rc = ctx->ms_data.ensure(std::max<uint64_t>(span, 1))) || (rc = ctx->ms_desc.ensure(n)) ||
      (rc = ctx->ms_out.ensure(n)) || (rc = ctx->ms_mm.ensure(words)))
    return rc;
  hipStream_t st = ctx->stream;
  if (span) HIPCHK(hipMemcpyAsync(ctx->ms_data.p, base + lo, span, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(ctx->ms_desc.p, rb.data(), n * sizeof(lcrc_desc_dev), hipMemcpyHostToDevice, st));
  if ((rc = lcrc_batch(ctx, ctx->ms_data.p, span, (const lcrc_desc*)ctx->ms_desc.p, n, ctx->ms_out.p,
                       out_mismatch ? ctx->ms_mm.p : nullptr, st)))
    return rc;
  HIPCHK(hipMemcpyAsync(out_crc, ctx->ms_out.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  if (out_mismatch) HIPCHK(hipMemcpyAsync(out_mismatch, ctx->ms_mm.p, words * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return LCRC_OK;
}

int lcrc_batch_multi(lcrc_ctx* const* ctxs, int nctx, const uint8_t* base, uint64_t base_len, const lcrc_desc* descs,
                     size_t n, uint32_t* out_crc, uint32_t* out_mismatch) {
  if (!ctxs || nctx < 1 || (n && (!descs || !out_crc || !base))) return LCRC_EINVAL;
  for (int k = 0; k < nctx; ++k)
    if (!ctxs[k]) return LCRC_EINVAL;
  if (n == 0) return LCRC_OK;
  // Shards are contiguous in OFFSET order, so that each one copies only the span its own ranges cover (a
  // descriptor list out of file order would otherwise give every shard nearly the whole file). Already sorted
  // lists keep their order; otherwise the results are scattered back to the caller's positions.
  std::vector<size_t> order(n);
  for (size_t i = 0; i < n; ++i) order[i] = i;
  bool sorted = true;
  for (size_t i = 1; i < n && sorted; ++i) sorted = descs[i - 1].offset <= descs[i].offset;
  if (!sorted)
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return descs[a].offset < descs[b].offset; });
  std::vector<lcrc_desc> sd;
  if (!sorted) {
    sd.resize(n);
    for (size_t i = 0; i < n; ++i) sd[i] = descs[order[i]];
  }
  const lcrc_desc* D = sorted ? descs : sd.data();
  // about equal covered bytes per shard (+64 per descriptor for its fixed cost); in place (sorted) the cuts fall on
  // multiples of 32 descriptors so that no mismatch-bitmap word is shared by two shards
  std::vector<size_t> cut(nctx + 1, n);
  cut[0] = 0;
  double total = 0;
  for (size_t i = 0; i < n; ++i) total += (double)D[i].length + 64.0;
  double acc = 0;
  int k = 1;
  for (size_t i = 0; i < n && k < nctx; ++i) {
    acc += (double)D[i].length + 64.0;
    while (k < nctx && acc >= total * k / nctx) {
      cut[k] = sorted ? std::min(n, (i + 1 + 31) / 32 * 32) : i + 1;
      ++k;
    }
  }
  for (int j = 1; j <= nctx; ++j) cut[j] = std::max(cut[j], cut[j - 1]);
  // out of order: each shard writes its own result arrays, scattered afterwards
  std::vector<uint32_t> scrc(sorted ? 0 : n), smm(sorted || !out_mismatch ? 0 : (n + 31) / 32 + nctx);
  std::vector<int> rcs(nctx, LCRC_OK);
  std::vector<std::string> errs(nctx);  // each worker's lcrc_last_error (thread-local there)
  std::vector<std::thread> th;
  for (int j = 0; j < nctx; ++j) {
    const size_t a = cut[j], b = cut[j + 1];
    if (a == b) continue;
    th.emplace_back([&, j, a, b] {
      uint32_t* oc = sorted ? out_crc + a : scrc.data() + a;
      // a private bitmap per shard when scattering: shard j's words start at a / 32 + j (its own words)
      uint32_t* om = !out_mismatch ? nullptr : sorted ? out_mismatch + a / 32 : smm.data() + a / 32 + j;
      rcs[j] = multi_shard(ctxs[j], base, base_len, D + a, b - a, oc, om);
      if (rcs[j]) errs[j] = g_last_error;
    });
  }
  for (auto& t : th) t.join();
  for (int j = 0; j < nctx; ++j)
    if (rcs[j]) {
      g_last_error = "lcrc_batch_multi shard " + std::to_string(j) + ": " + errs[j];
      return rcs[j];
    }
  if (!sorted) {
    for (int j = 0; j < nctx; ++j) {
      const size_t a = cut[j], b = cut[j + 1];
      for (size_t i = a; i < b; ++i) {
        const size_t o = order[i];
        out_crc[o] = scrc[i];
        if (out_mismatch) {
          const size_t w = a / 32 + j, bit = i - a;  // the shard's own bitmap, bit i - a
          const bool bad = (smm[w + bit / 32] >> (bit & 31)) & 1u;
          if (bad) out_mismatch[o >> 5] |= 1u << (o & 31);
          else out_mismatch[o >> 5] &= ~(1u << (o & 31));
        }
      }
    }
    if (out_mismatch && (n & 31)) out_mismatch[n >> 5] &= (1u << (n & 31)) - 1u;  // bits past n, as lcrc_batch
  }
  return LCRC_OK;
}

int lcrc_wal_scan_async(lcrc_ctx* ctx, const uint8_t* file, uint64_t file_len, lcrc_wal_rec* recs, size_t max_recs,
                        uint64_t* n_recs, void* stream) {
  TkScope tk_scope(ctx);
  if (!ctx || !n_recs || (file_len && !file) || (max_recs && !recs)) return LCRC_EINVAL;
  if (file_len >= LCRC_WAL_MAX_FILE) return LCRC_EINVAL;  // record indices and counts are 32-bit on the device
  int rc = set_device(ctx);
  if (rc) return rc;
  hipStream_t st = pick_stream(ctx, stream);
  const uint64_t nblocks = (file_len + 32767) / 32768;
  // wal_offsets: [0] the total, then per block the in-workgroup offsets and per 64 blocks the totals, as packed
  // (records | one-window records << 32) counts
  if ((rc = ctx->wal_counts.ensure(nblocks + 1)) || (rc = ctx->wal_slots.ensure(nblocks * 64 + 1)) ||
      (rc = ctx->wal_stops.ensure(nblocks + 1)) ||
      (rc = ctx->wal_offsets.ensure(1 + nblocks + (nblocks + 63) / 64 + 1)))
    return rc;
  if (max_recs && ((rc = ctx->wal_descs.ensure(max_recs)) || (rc = ctx->wal_crcs.ensure(max_recs)) ||
                   (rc = ctx->win.ensure(window_words(file_len)))))
    return rc;
  uint64_t* n_total = ctx->wal_offsets.p;
  uint64_t* local = ctx->wal_offsets.p + 1;
  uint64_t* part = ctx->wal_offsets.p + 1 + nblocks;
  // One stream: the header walk (k_wal_parse, one lane per 32 KiB block following the 7-byte headers,
  // then k_wal_emit), the window pass over the whole file, then one k_blocks over all records (the log format stores
  // the raw crc: no mask) that also stores each record's crc and verdict.
  HIPCHK(lcrc_launch_wal_parse(file, file_len, nblocks, ctx->wal_counts.p, ctx->wal_slots.p, ctx->wal_stops.p, local,
                               part, (lcrc_wal_rec_dev*)recs, ctx->wal_descs.p, max_recs, n_total, n_recs, st));
  if (max_recs && ctx->general == 1) {
    HIPCHK(lcrc_launch_ranges(false, ctx->grid_a, file, file_len, ctx->wal_descs.p, max_recs, 0, 0, nullptr,
                              ctx->d_tab, ctx->x4096, ctx->poly, ctx->init, ctx->xorout, 0, ctx->wal_crcs.p, nullptr,
                              n_total, (lcrc_wal_rec_dev*)recs, st));
  } else if (max_recs) {
    HIPCHK(lcrc_launch_windows(false, ctx->grid_a, file, file_len, ctx->d_tab, ctx->win.p, 0, 0, 0, nullptr, nullptr,
                               st));
    HIPCHK(lcrc_launch_blocks(false, ctx->wal_grid_b ? ctx->wal_grid_b : ctx->grid_b / LCRC_WAL_GRID_DIV, file, file_len,
                              ctx->wal_descs.p, max_recs, 0, 0, nullptr,
                              ctx->win.p, ctx->d_tab, ctx->init, ctx->xorout, 0, ctx->wal_crcs.p, nullptr, n_total,
                              (lcrc_wal_rec_dev*)recs, st));
  }
  return LCRC_OK;
}

// Several logs in one submission. The header walks of all of them run first, in one launch (five 256 MiB
// logs' walks in 24 us, about one log's alone: a dependent chain of memory round trips per 32 KiB block, run
// here with the HBM stream idle instead of beside another scan's window pass, which triples its round trips),
// and their records are emitted in one more. Then the logs alternate over the two queue lanes, each running a
// log's window pass and range pass (as lcrc_batch_queue). Each log has its own workspace; the lanes join
// `stream` before the call's end. Measured (config 4, 5 logs per call): 3.1K GiB/s against 3.4K for two
// contexts taking alternate logs -- the lanes' fork and join cost ~35 us per call and an odd log runs alone.
int lcrc_wal_scan_queue(lcrc_ctx* ctx, const lcrc_wjob* jobs, size_t njobs, void* stream) {
  TkScope tk_scope(ctx);
  if (!ctx || (njobs && !jobs)) return LCRC_EINVAL;
  for (size_t k = 0; k < njobs; ++k)
    if (!jobs[k].n_recs || (jobs[k].file_len && !jobs[k].file) || (jobs[k].max_recs && !jobs[k].recs) ||
        jobs[k].file_len >= LCRC_WAL_MAX_FILE)
      return LCRC_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  hipStream_t st = pick_stream(ctx, stream);
  if (ctx->general == 1) {  // the one-pass range kernel: log by log
    for (size_t k = 0; k < njobs; ++k)
      if ((rc = lcrc_wal_scan_async(ctx, jobs[k].file, jobs[k].file_len, jobs[k].recs, jobs[k].max_recs,
                                    jobs[k].n_recs, st)))
        return rc;
    return LCRC_OK;
  }
  const size_t M = lcrc_wal_queue_max();
  for (size_t k0 = 0; k0 < njobs; k0 += M) {
    const uint32_t m = (uint32_t)std::min(M, njobs - k0);
    if (ctx->wq.size() < m) ctx->wq.resize(m);
    lcrc_wjob_dev_host h[64];
    for (uint32_t k = 0; k < m; ++k) {
      const lcrc_wjob& j = jobs[k0 + k];
      auto& w = ctx->wq[k];
      const uint64_t nblocks = (j.file_len + 32767) / 32768;
      if ((rc = w.counts.ensure(nblocks + 1)) || (rc = w.slots.ensure(nblocks * 64 + 1)) ||
          (rc = w.stops.ensure(nblocks + 1)) ||
          (rc = w.offsets.ensure(1 + nblocks + (nblocks + 63) / 64 + 1)))
        return rc;
      if (j.max_recs && ((rc = w.descs.ensure(j.max_recs)) || (rc = w.crcs.ensure(j.max_recs)) ||
                         (rc = w.win.ensure(window_words(j.file_len)))))
        return rc;
      h[k] = lcrc_wjob_dev_host{j.file, j.file_len, nblocks, w.counts.p, w.slots.p, w.stops.p,
                                w.offsets.p + 1, w.offsets.p + 1 + nblocks,
                                (lcrc_wal_rec_dev*)j.recs, w.descs.p, j.max_recs, w.offsets.p, j.n_recs};
    }
    if ((rc = ensure_lanes(ctx))) return rc;
    HIPCHK(lcrc_launch_wal_parse_queue(h, m, st));
    HIPCHK(hipEventRecord(ctx->q_fork, st));
    hipStream_t lane[2] = {ctx->side, ctx->side2};
    for (hipStream_t l : lane) HIPCHK(hipStreamWaitEvent(l, ctx->q_fork, 0));
    hipEvent_t held_stop = lcrc_launch_events_swap_stop(nullptr);  // recorded after the join (lanes_join_timed)
    for (uint32_t k = 0; k < m; ++k) {
      const lcrc_wjob& j = jobs[k0 + k];
      if (!j.max_recs) continue;
      auto& w = ctx->wq[k];
      hipStream_t l = lane[k & 1];
      HIPCHK(lcrc_launch_windows(false, ctx->grid_a, j.file, j.file_len, ctx->d_tab, w.win.p, 0, 0, 0, nullptr, nullptr,
                                 l));
      HIPCHK(lcrc_launch_blocks(false, std::min(ctx->grid_b, ctx->grid_a * LCRC_WALQ_WG_PER_CU), j.file, j.file_len,
                                w.descs.p, j.max_recs, 0, 0, nullptr, w.win.p, ctx->d_tab, ctx->init, ctx->xorout, 0,
                                w.crcs.p, nullptr, h[k].n_total, (lcrc_wal_rec_dev*)j.recs, l));
    }
    if ((rc = lanes_join_timed(ctx, st, held_stop))) return rc;
  }
  return LCRC_OK;
}

int lcrc_wal_scan(lcrc_ctx* ctx, const uint8_t* file, uint64_t file_len, lcrc_wal_rec* recs, size_t max_recs,
                  size_t* n_recs, void* stream) {
  if (!ctx || !n_recs) return LCRC_EINVAL;
  *n_recs = 0;
  *ctx->h_count = 0;
  int rc = lcrc_wal_scan_async(ctx, file, file_len, recs, max_recs, ctx->h_count, stream);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(pick_stream(ctx, stream)));
  const uint64_t total = *ctx->h_count;
  *n_recs = total;
  return total > max_recs ? LCRC_EINVAL : LCRC_OK;
}

// ---- Snappy framing: decode + per-chunk masked CRC-32C verify ----
// Snappy framing in two halves around the one host round trip it needs. plan: sizes, chunk counts and the
// batch maxima on the device, their scans, and the totals queued for the pinned staging (h_count[4..6])
// -- no synchronisation. run (after the caller synchronised): capacity check, decode, masked CRC-32C of
// every chunk and the compare -- enqueued, no synchronisation.
static int snappy_plan(lcrc_ctx* ctx, const uint8_t* base, const lcrc_desc_dev* frames, size_t n, uint64_t* out_off,
                       uint8_t* status, hipStream_t st) {
  int rc;
  const size_t nparts = (n + 255) / 256;
  if ((rc = ctx->sn_size.ensure(n)) || (rc = ctx->sn_nch.ensure(n)) || (rc = ctx->sn_choff.ensure(n + 1)) ||
      (rc = ctx->sn_part.ensure(2 * nparts)) || (rc = ctx->sn_max.ensure(2)))
    return rc;
  HIPCHK(hipMemsetAsync(ctx->sn_max.p, 0, 8, st));
  HIPCHK(lcrc_launch_snappy_size(base, frames, n, ctx->sn_size.p, ctx->sn_nch.p, status, ctx->sn_max.p, nullptr, st));
  HIPCHK(lcrc_launch_scan2(ctx->sn_size.p, ctx->sn_nch.p, n, out_off, ctx->sn_choff.p, ctx->sn_part.p, nullptr, st));
  uint64_t* tot = ctx->h_count + 4;  // pinned staging: decoded total, chunk total, then the two maxima
  HIPCHK(hipMemcpyAsync(&tot[0], out_off + n, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&tot[1], ctx->sn_choff.p + n, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(ctx->h_count + 6, ctx->sn_max.p, 8, hipMemcpyDeviceToHost, st));
  return LCRC_OK;
}

static int snappy_run(lcrc_ctx* ctx, const uint8_t* base, const lcrc_desc_dev* frames, size_t n, uint8_t* out,
                      uint64_t out_cap, uint64_t* out_off, uint8_t* status, uint64_t* total_out, hipStream_t st) {
  int rc;
  const uint64_t* tot = ctx->h_count + 4;
  const uint32_t* mx = (const uint32_t*)(ctx->h_count + 6);
  *total_out = tot[0];
  if (tot[0] > out_cap || (tot[0] && !out)) return LCRC_ERANGE;
  const uint64_t nch = tot[1];
  if (nch == 0) return LCRC_OK;
  if ((rc = ctx->sn_cdesc.ensure(nch)) || (rc = ctx->sn_cexp.ensure(nch)) || (rc = ctx->sn_cframe.ensure(nch)) ||
      (rc = ctx->sn_ccrc.ensure(nch)) || (rc = ctx->win.ensure(window_words(tot[0]))))
    return rc;
  if (ctx->mode != LCRC_MODE_C && !ctx->d_tab_c && (rc = upload_tables(LCRC_MODE_C, &ctx->d_tab_c))) return rc;
  const uint32_t* tab_c = ctx->mode == LCRC_MODE_C ? ctx->d_tab : ctx->d_tab_c;
  HIPCHK(lcrc_launch_snappy_decode(base, frames, n, out_off, ctx->sn_choff.p, out, status, ctx->sn_cdesc.p,
                                   ctx->sn_cexp.p, ctx->sn_cframe.p, mx[0], mx[1], st));
  // masked CRC-32C of every decoded chunk: the general path over the decoded bytes
  if (ctx->general == 1) {
    static const uint32_t x4096_c = lcrc::x8n(4096, lcrc::POLY_C);
    HIPCHK(lcrc_launch_ranges(false, ctx->grid_a, out, tot[0], ctx->sn_cdesc.p, nch, 0, 0, nullptr, tab_c, x4096_c,
                              lcrc::POLY_C, lcrc::CRC_INIT, lcrc::CRC_XOROUT, LCRC_FLAG_MASK, ctx->sn_ccrc.p, nullptr,
                              nullptr, nullptr, st));
  } else {
    HIPCHK(lcrc_launch_windows(false, ctx->grid_a, out, tot[0], tab_c, ctx->win.p, 0, 0, 0, nullptr, nullptr, st));
    HIPCHK(lcrc_launch_blocks(false, ctx->grid_b, out, tot[0], ctx->sn_cdesc.p, nch, 0, 0, nullptr, ctx->win.p, tab_c,
                              lcrc::CRC_INIT, lcrc::CRC_XOROUT, LCRC_FLAG_MASK, ctx->sn_ccrc.p, nullptr, nullptr,
                              nullptr, st));
  }
  HIPCHK(lcrc_launch_snappy_check(ctx->sn_ccrc.p, ctx->sn_cexp.p, ctx->sn_cframe.p, ctx->sn_choff.p + n, nch, status,
                                  st));
  return LCRC_OK;
}

static int snappy_frames_impl(lcrc_ctx* ctx, const uint8_t* base, const lcrc_desc_dev* frames, size_t n, uint8_t* out,
                              uint64_t out_cap, uint64_t* out_off, uint8_t* status, uint64_t* total_out, hipStream_t st) {
  int rc;
  *total_out = 0;
  if (n == 0) return LCRC_OK;
  if ((rc = snappy_plan(ctx, base, frames, n, out_off, status, st))) return rc;
  HIPCHK(hipStreamSynchronize(st));
  if ((rc = snappy_run(ctx, base, frames, n, out, out_cap, out_off, status, total_out, st))) return rc;
  HIPCHK(hipStreamSynchronize(st));
  return LCRC_OK;
}

int lcrc_snappy_frames(lcrc_ctx* ctx, const uint8_t* base, const lcrc_desc* frames, size_t n, uint8_t* out,
                       uint64_t out_cap, uint64_t* out_off, uint8_t* status, uint64_t* total) {
  if (!ctx || !total || (n && (!base || !frames || !out_off || !status))) return LCRC_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  return snappy_frames_impl(ctx, base, (const lcrc_desc_dev*)frames, n, out, out_cap, out_off, status, total,
                            ctx->stream);
}

// ---- whole-table verify scan ----
// Whole-table scan with the index block walked on the device (one thread per restart segment). Returns
// TBL_FALLBACK when the index block is not one the segmented walk can vouch for; the host walk then
// repeats it sequentially with the reference's messages.
static constexpr int TBL_FALLBACK = 1000;

static int table_scan_device(lcrc_ctx* ctx, const uint8_t* file, uint64_t file_len, const char* filter_name,
                             const lcrc_tbl::Handle& meta_h, const lcrc_tbl::Handle& index_h, lcrc_tblk* blocks,
                             size_t max_blocks, size_t* n_blocks, const std::function<int(const char*)>& corrupt) {
  using namespace lcrc_tbl;
  hipStream_t st = ctx->stream;
  int rc;
  if (index_h.offset > file_len || index_h.size + BLOCK_TRAILER_SIZE > file_len - index_h.offset ||
      index_h.size + 1 > 0x7FFFFFFFull)
    return TBL_FALLBACK;
  // Table::open: read_block_from_file(index, verify_checksum = paranoid_checks) -- the checksum and the
  // type byte on the device
  // the window pass spans the buffer it is given: verify the index block on its own bytes
  lcrc_desc_dev idesc;
  idesc.offset = 0;
  idesc.length = (uint32_t)(index_h.size + 1);
  idesc.expect_rel = (int32_t)(index_h.size + 1);
  const uint64_t tpos = index_h.offset + index_h.size;
  if ((rc = ctx->tbl_descs.ensure(1)) || (rc = ctx->tbl_crcs.ensure(1)) || (rc = ctx->tbl_mm.ensure(1)) ||
      (rc = ctx->tbl_pos.ensure(1)) || (rc = ctx->tbl_types.ensure(1)))
    return rc;
  HIPCHK(hipMemcpyAsync(ctx->tbl_descs.p, &idesc, sizeof(idesc), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(ctx->tbl_pos.p, &tpos, sizeof(tpos), hipMemcpyHostToDevice, st));
  if ((rc = lcrc_batch(ctx, file + index_h.offset, index_h.size + BLOCK_TRAILER_SIZE,
                       (const lcrc_desc*)ctx->tbl_descs.p, 1, ctx->tbl_crcs.p, ctx->tbl_mm.p, st)))
    return rc;
  HIPCHK(lcrc_launch_gather_u8(file, ctx->tbl_pos.p, 1, ctx->tbl_types.p, st));
  // one pinned round trip: the mismatch bit, the type byte and (for a raw index) its restart count
  uint8_t* hs = (uint8_t*)(ctx->h_count + 1);
  memset(hs, 0, 16);
  HIPCHK(hipMemcpyAsync(hs, ctx->tbl_mm.p, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(hs + 4, ctx->tbl_types.p, 1, hipMemcpyDeviceToHost, st));
  if (index_h.size >= 4)
    HIPCHK(hipMemcpyAsync(hs + 8, file + index_h.offset + index_h.size - 4, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  uint32_t imm, nres_raw;
  memcpy(&imm, hs, 4);
  memcpy(&nres_raw, hs + 8, 4);
  const uint8_t itype = hs[4];
  if (imm & 1) return corrupt("block checksum mismatch");
  const uint8_t* contents = file + index_h.offset;
  uint64_t clen = index_h.size;
  if (itype == 1) {  // Snappy-framed index block, decoded on the device
    if ((rc = ctx->sn_out_off.ensure(2)) || (rc = ctx->sn_status.ensure(1))) return rc;
    idesc.offset = index_h.offset;
    idesc.length = (uint32_t)index_h.size;
    idesc.expect_rel = LCRC_NO_EXPECT_DEV;
    HIPCHK(hipMemcpyAsync(ctx->tbl_descs.p, &idesc, sizeof(idesc), hipMemcpyHostToDevice, st));
    uint64_t total = 0;
    rc = snappy_frames_impl(ctx, file, ctx->tbl_descs.p, 1, ctx->sn_out.p, ctx->sn_out.cap, ctx->sn_out_off.p,
                            ctx->sn_status.p, &total, st);
    if (rc == LCRC_ERANGE) {
      if ((rc = ctx->sn_out.ensure(total))) return rc;
      rc = snappy_frames_impl(ctx, file, ctx->tbl_descs.p, 1, ctx->sn_out.p, ctx->sn_out.cap, ctx->sn_out_off.p,
                              ctx->sn_status.p, &total, st);
    }
    if (rc) return rc;
    uint8_t fst = 0;
    HIPCHK(hipMemcpy(&fst, ctx->sn_status.p, 1, hipMemcpyDeviceToHost));
    if (fst) return corrupt("corrupted compressed block content");
    contents = ctx->sn_out.p;
    clen = total;
  } else if (itype != 0) {
    return corrupt("bad block type");
  }
  // Block::from_content (block.rs:21-41)
  if (clen < 4) return corrupt("bad block contents, size smaller than u32");
  if (clen > 0xFFFFFFFFull) return TBL_FALLBACK;
  uint32_t nres = nres_raw;
  if (itype == 1) HIPCHK(hipMemcpy(&nres, contents + clen - 4, 4, hipMemcpyDeviceToHost));
  if ((uint64_t)nres > (clen - 4) / 4) return corrupt("bad block contents");
  // entries without restart points, or segments so long that one thread per segment would be slower than
  // the host (the reference's index blocks restart at every entry, table.rs:272): the sequential walk
  if (nres == 0 || (clen - 4) / nres > 4096) return TBL_FALLBACK;
  const uint32_t len = (uint32_t)clen;
  // entries per restart segment -> their positions
  if ((rc = ctx->idx_count.ensure(nres)) || (rc = ctx->idx_flag.ensure(nres)) || (rc = ctx->idx_pos.ensure(nres + 1)) ||
      (rc = ctx->idx_fpos.ensure(nres + 1)) || (rc = ctx->sn_part.ensure(2 * ((nres + 255) / 256))))
    return rc;
  HIPCHK(lcrc_launch_idx_parse(false, contents, len, nres, file_len, ctx->idx_count.p, ctx->idx_flag.p, nullptr, nullptr,
                               nullptr, st));
  HIPCHK(lcrc_launch_scan2(ctx->idx_count.p, ctx->idx_flag.p, nres, ctx->idx_pos.p, ctx->idx_fpos.p, ctx->sn_part.p,
                           nullptr, st));
  uint64_t* tot = ctx->h_count + 2;  // pinned
  HIPCHK(hipMemcpyAsync(&tot[0], ctx->idx_pos.p + nres, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&tot[1], ctx->idx_fpos.p + nres, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (tot[1]) return TBL_FALLBACK;
  const uint64_t nd = tot[0];
  // read_meta: only with a filter policy, and its errors are not propagated (table.rs:81-103); the
  // metaindex block is small and walked on the host
  std::vector<lcrc_tblk> extra;
  auto add = [&](const Handle& h, uint8_t kind) {
    lcrc_tblk b;
    memset(&b, 0, sizeof(b));
    b.offset = h.offset;
    b.size = h.size;
    b.kind = kind;
    extra.push_back(b);
  };
  if (filter_name && meta_h.offset <= file_len && meta_h.size + BLOCK_TRAILER_SIZE <= file_len - meta_h.offset) {
    std::vector<uint8_t> raw(meta_h.size + BLOCK_TRAILER_SIZE), mc;
    HIPCHK(hipMemcpy(raw.data(), file + meta_h.offset, raw.size(), hipMemcpyDeviceToHost));
    if (!block_contents(raw.data(), meta_h.size, true, ctx->mode, ctx->flags, mc)) {
      const std::string want = std::string("filter") + filter_name;
      block_entries(mc, [&](const std::string& key, const uint8_t* v, uint32_t vn) {
        if (key < want) return true;  // seek: first key >= want
        Handle h;
        const uint8_t* p = v;
        if (key == want && !decode_handle(p, v + vn, h)) add(h, LCRC_TBLK_FILTER);
        return false;
      });
    }
  }
  add(meta_h, LCRC_TBLK_METAINDEX);
  add(index_h, LCRC_TBLK_INDEX);
  const size_t n = nd + extra.size();
  *n_blocks = n;
  if (!blocks || max_blocks < n) return LCRC_ERANGE;
  if ((rc = ctx->tbl_blk.ensure(n)) || (rc = ctx->tbl_descs.ensure(n)) || (rc = ctx->tbl_crcs.ensure(n)) ||
      (rc = ctx->tbl_mm.ensure((n + 31) / 32)) || (rc = ctx->tbl_frames.ensure(n)) ||
      (rc = ctx->sn_out_off.ensure(n + 1)) || (rc = ctx->sn_status.ensure(n)))
    return rc;
  HIPCHK(lcrc_launch_idx_parse(true, contents, len, nres, file_len, nullptr, nullptr, ctx->idx_pos.p, ctx->tbl_blk.p,
                               ctx->tbl_descs.p, st));
  std::vector<lcrc_desc_dev> xd(extra.size());
  for (size_t k = 0; k < extra.size(); ++k) {
    lcrc_tblk& b = extra[k];
    const bool in = b.offset <= file_len && b.size + BLOCK_TRAILER_SIZE <= file_len - b.offset &&
                    b.size + 1 <= 0x7FFFFFFFull;
    xd[k].offset = in ? b.offset : 0;
    xd[k].length = in ? (uint32_t)(b.size + 1) : 0;
    xd[k].expect_rel = in ? (int32_t)(b.size + 1) : LCRC_NO_EXPECT_DEV;
    if (!in) {
      b.status = LCRC_TBLK_TRUNCATED;
      b.type = 0xFF;
    }
  }
  HIPCHK(hipMemcpyAsync(ctx->tbl_blk.p + nd, extra.data(), extra.size() * sizeof(lcrc_tblk), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(ctx->tbl_descs.p + nd, xd.data(), xd.size() * sizeof(lcrc_desc_dev), hipMemcpyHostToDevice, st));
  // ONE batched verify of every block, then read_block_from_file's type dispatch: Snappy frames decoded and
  // checked on the device
  if ((rc = lcrc_batch(ctx, file, file_len, (const lcrc_desc*)ctx->tbl_descs.p, n, ctx->tbl_crcs.p, ctx->tbl_mm.p, st)))
    return rc;
  if (!ctx->tbl_flag.p) {
    if ((rc = ctx->tbl_flag.ensure(1))) return rc;
    HIPCHK(hipMemsetAsync(ctx->tbl_flag.p, 0, sizeof(uint32_t), st));
  }
  if (++ctx->tbl_gen == 0) ctx->tbl_gen = 1;
  HIPCHK(lcrc_launch_tbl_finish(ctx->tbl_blk.p, n, ctx->tbl_crcs.p, ctx->tbl_mm.p, file, ctx->tbl_frames.p, nullptr,
                                st));
  // the Snappy frames' framing pass (a malformed frame is already status 3 here), then the results and the
  // frame totals come back in ONE round trip; only a table with compressed blocks goes on to decode them
  if ((rc = snappy_plan(ctx, file, ctx->tbl_frames.p, n, ctx->sn_out_off.p, ctx->sn_status.p, st))) return rc;
  HIPCHK(lcrc_launch_tbl_content(ctx->tbl_blk.p, n, ctx->sn_status.p, ctx->tbl_flag.p, ctx->tbl_gen, nullptr, st));
  HIPCHK(hipMemcpyAsync(blocks, ctx->tbl_blk.p, n * sizeof(lcrc_tblk), hipMemcpyDeviceToHost, st));
  uint32_t* h_unsorted = (uint32_t*)(ctx->h_count + 7);  // pinned
  HIPCHK(hipMemcpyAsync(h_unsorted, ctx->tbl_flag.p, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const bool sorted = *h_unsorted != ctx->tbl_gen;
  if (ctx->h_count[5]) {  // data chunks to decode and check
    uint64_t total = 0;
    if ((rc = ctx->sn_out.ensure(ctx->h_count[4]))) return rc;
    if ((rc = snappy_run(ctx, file, ctx->tbl_frames.p, n, ctx->sn_out.p, ctx->sn_out.cap, ctx->sn_out_off.p,
                         ctx->sn_status.p, &total, st)))
      return rc;
    HIPCHK(lcrc_launch_tbl_content(ctx->tbl_blk.p, n, ctx->sn_status.p, nullptr, 0, nullptr, st));
    HIPCHK(hipMemcpyAsync(blocks, ctx->tbl_blk.p, n * sizeof(lcrc_tblk), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  // sorted by offset (a well-formed table already is; the order was checked by k_tbl_finish)
  if (!sorted)
    std::stable_sort(blocks, blocks + n, [](const lcrc_tblk& a, const lcrc_tblk& b) { return a.offset < b.offset; });
  return LCRC_OK;
}

// ---- asynchronous whole-table scan: every step on the device, nothing synchronized ----
static const char* const kTscanMsg[] = {"",
                                        "file is too short to be an sstable",
                                        "not an sstable (bad magic number)",
                                        "Error when decoding varint64",
                                        "block checksum mismatch",
                                        "bad block type",
                                        "bad block contents, size smaller than u32",
                                        "bad block contents"};

const char* lcrc_table_scan_message(uint32_t code) {
  return code < sizeof(kTscanMsg) / sizeof(kTscanMsg[0]) ? kTscanMsg[code] : "";
}

// the batched verify's descriptors: the blocks and the pieces of a long filter / metaindex / index block
static uint64_t ts_verify_cap(size_t max_blocks, uint64_t file_len) {
  return max_blocks + 1 + file_len / LCRC_TS_PIECE + 3;
}

// the device-only scan's workspace (every buffer its launches touch; nothing else: the host-assisted scan and
// lcrc_snappy_frames size their own)
constexpr uint32_t TS_AGG_WORDS = 257;  // k_ts_windows: at most 256 index workgroups' words, then the ticket counter
constexpr uint32_t TS_MAX_IDX = 256;

static int ts_reserve(lcrc_ctx* ctx, uint64_t max_file_len, size_t max_blocks, uint64_t decoded_cap) {
  int rc = set_device(ctx);
  if (rc) return rc;
  const uint64_t nb = max_blocks + 1;
  const uint64_t nv = ts_verify_cap(max_blocks, max_file_len);
  decoded_cap = std::max<uint64_t>(decoded_cap, ctx->ts_decoded_cap);
  if ((rc = ctx->ts_state.ensure(1)) || (rc = ctx->idx_count.ensure(nb)) || (rc = ctx->idx_flag.ensure(nb)) ||
      (rc = ctx->sn_part.ensure(2 * (nb / 256 + 2))) || (rc = ctx->tbl_descs.ensure(nv)) ||
      (rc = ctx->tbl_crcs.ensure(nv)) || (rc = ctx->tbl_mm.ensure(nv / 32 + 1)) || (rc = ctx->tbl_frames.ensure(nb)) ||
      (rc = ctx->sn_nch.ensure(nb)) || (rc = ctx->sn_out_off.ensure(nb)) || (rc = ctx->sn_choff.ensure(nb)) ||
      (rc = ctx->sn_status.ensure(nb)) || (rc = ctx->sn_out.ensure(decoded_cap + 16 * (decoded_cap / 4096 + 1) + 16)) ||
      (rc = ctx->win.ensure(window_words(max_file_len))) || (rc = ctx->ts_idx.ensure(decoded_cap)) ||
      (rc = ctx->ts_open_scr.ensure(lcrc_ts_open_scratch_words())))
    return rc;
  if (!ctx->ts_open.p) {
    if ((rc = ctx->ts_open.ensure(4))) return rc;
    HIPCHK(zero_now(ctx, ctx->ts_open.p, 4 * sizeof(uint64_t)));
  }
  if (!ctx->ts_agg.p) {
    if ((rc = ctx->ts_agg.ensure(TS_AGG_WORDS))) return rc;
    HIPCHK(zero_now(ctx, ctx->ts_agg.p, TS_AGG_WORDS * sizeof(uint64_t)));
  }
  if (ctx->mode != LCRC_MODE_C && !ctx->d_tab_c && (rc = upload_tables(LCRC_MODE_C, &ctx->d_tab_c))) return rc;
  ctx->ts_decoded_cap = decoded_cap;
  // the workspace holds only the chunks k_ts_decode cannot decode in LDS (over 12 KiB compressed or 16 KiB decoded),
  // each 16-aligned: a caller reserving the exact decoded total still scans on the device
  ctx->ts_out_cap = decoded_cap + 16 * (decoded_cap / 4096 + 1);
  return LCRC_OK;
}

int lcrc_table_scan_reserve(lcrc_ctx* ctx, uint64_t max_file_len, size_t max_blocks, uint64_t decoded_cap) {
  if (!ctx) return LCRC_EINVAL;
  return ts_reserve(ctx, max_file_len, max_blocks, decoded_cap);
}

int lcrc_table_scan_async(lcrc_ctx* ctx, const uint8_t* file, uint64_t file_len, const char* filter_name,
                          lcrc_tblk* blocks, size_t max_blocks, uint64_t* n_blocks, uint32_t* status, void* stream) {
  return lcrc_table_scan_async_ex(ctx, file, file_len, filter_name, blocks, max_blocks, n_blocks, status, 0, stream);
}

int lcrc_table_scan_async_ex(lcrc_ctx* ctx, const uint8_t* file, uint64_t file_len, const char* filter_name,
                             lcrc_tblk* blocks, size_t max_blocks, uint64_t* n_blocks, uint32_t* status, uint32_t flags,
                             void* stream) {
  TkScope tk_scope(ctx);
  if (!ctx || !n_blocks || !status || (file_len && !file) || (max_blocks && !blocks) ||
      (flags & ~LCRC_TSCAN_SNAPPY_INDEX))
    return LCRC_EINVAL;
  lcrc_tscan_key key;
  memset(&key, 0, sizeof(key));
  if (filter_name) {
    const size_t nl = strlen(filter_name);
    if (nl + 6 > sizeof(key.key)) return LCRC_EINVAL;
    memcpy(key.key, "filter", 6);
    memcpy(key.key + 6, filter_name, nl);
    key.len = (uint32_t)(nl + 6);
  }
  // workspace for this size (reserved beforehand, this allocates nothing: graph-capturable)
  int rc = ts_reserve(ctx, file_len, max_blocks, 0);
  if (rc) return rc;
  hipStream_t st = pick_stream(ctx, stream);
  lcrc_tscan_dev* S = ctx->ts_state.p;
  lcrc_tblk_dev* blk = (lcrc_tblk_dev*)blocks;
  const uint64_t cap = max_blocks;
  const uint32_t* tab_c = ctx->mode == LCRC_MODE_C ? ctx->d_tab : ctx->d_tab_c;
  // Four dependent launches (five with LCRC_TSCAN_SNAPPY_INDEX: a Snappy-framed index block decoded first). The
  // footer, the index block header and the metaindex filter entry (optimistic: checksums come with the batch) with
  // the index block's restart segments walked in ranges, one per index workgroup
  const bool sidx = flags & LCRC_TSCAN_SNAPPY_INDEX;
  if (sidx)
    HIPCHK(lcrc_launch_ts_open(file, file_len, tab_c, ctx->ts_idx.p, ctx->ts_idx.cap, ctx->ts_open.p,
                               ctx->ts_open_scr.p, st));
  const uint64_t vcap = ts_verify_cap(cap, file_len);
  const uint64_t* nver = &S->n_verify;
  const bool fused = cap && ctx->general != 1;
  // the index walk and the handles (k_ts_windows' index workgroups), beside the file's window pass when the batch
  // goes through it (the window values do not depend on the handles)
  HIPCHK(lcrc_launch_ts_windows(ctx->grid_a, fused, file, file_len, ctx->d_tab, ctx->win.p, &key, cap, vcap, S,
                                ctx->idx_count.p, ctx->tbl_mm.p, vcap / 32 + 1, ctx->ts_idx.p,
                                sidx ? ctx->ts_open.p : nullptr, ctx->ts_open.p, blk, ctx->tbl_descs.p, ctx->ts_agg.p,
                                std::min<uint32_t>(ctx->ts_grid, TS_MAX_IDX), st));
  // ONE batched verify of every block (data, filter, metaindex, index, and the pieces of long ones)
  if (cap) {
    if (ctx->general == 1) {  // options.general = 1: the one-pass kernel
      HIPCHK(lcrc_launch_ranges(false, ctx->grid_a, file, file_len, ctx->tbl_descs.p, vcap, 0, 0, nullptr, ctx->d_tab,
                                ctx->x4096, ctx->poly, ctx->init, ctx->xorout, ctx->flags & LCRC_FLAG_MASK,
                                ctx->tbl_crcs.p, ctx->tbl_mm.p, nver, nullptr, st));
    } else {
      const int div = ctx->ts_blocks_div ? ctx->ts_blocks_div : 1;
      HIPCHK(lcrc_launch_blocks(false, ctx->grid_b / div, file, file_len, ctx->tbl_descs.p, vcap, 0, 0,
                                nullptr, ctx->win.p, ctx->d_tab, ctx->init, ctx->xorout, ctx->flags & LCRC_FLAG_MASK,
                                ctx->tbl_crcs.p, ctx->tbl_mm.p, nver, nullptr, st));
    }
    // read_block_from_file's type dispatch and the Snappy framing walk (the frames' padded decoded sizes scanned per
    // 256-block tile)
    HIPCHK(lcrc_launch_ts_finish(blk, cap, ctx->tbl_crcs.p, ctx->tbl_mm.p, file, ctx->tbl_frames.p, ctx->sn_out_off.p,
                                 ctx->sn_choff.p, ctx->sn_part.p, ctx->sn_nch.p, ctx->sn_status.p, S, ctx->d_tab,
                                 ctx->flags, st));
  }
  // the frames decoded and every chunk's masked CRC-32C checked in the decoding wave, the content verdicts and the
  // reference's order of outcomes; the count and the status for the caller
  HIPCHK(lcrc_launch_ts_decode(file, ctx->tbl_frames.p, ctx->sn_out_off.p, ctx->sn_out.p, ctx->sn_status.p, S, blk, tab_c,
                               ctx->ts_out_cap, ctx->sn_part.p, cap, n_blocks, status, st));
  return LCRC_OK;
}

int lcrc_table_scan(lcrc_ctx* ctx, const uint8_t* file, uint64_t file_len, const char* filter_name,
                    lcrc_tblk* blocks, size_t max_blocks, size_t* n_blocks, char* err, size_t err_cap) {
  using namespace lcrc_tbl;
  if (!ctx || !n_blocks || (file_len && !file)) return LCRC_EINVAL;
  *n_blocks = 0;
  if (err && err_cap) err[0] = 0;
  int rc = set_device(ctx);
  if (rc) return rc;
  hipStream_t st = ctx->stream;
  auto corrupt = [&](const char* msg) {
    if (err && err_cap) {
      strncpy(err, msg, err_cap - 1);
      err[err_cap - 1] = 0;
    }
    return LCRC_ECORRUPT;
  };
  // the host reads only what locates the blocks: footer, index block, metaindex block
  auto read_raw = [&](const Handle& h, std::vector<uint8_t>& raw) -> const char* {
    if (h.offset > file_len || h.size + BLOCK_TRAILER_SIZE > file_len - h.offset) return "truncated block read";
    raw.resize(h.size + BLOCK_TRAILER_SIZE);
    if (hipMemcpy(raw.data(), file + h.offset, raw.size(), hipMemcpyDeviceToHost) != hipSuccess)
      return "device read failed";
    return nullptr;
  };
  if (file_len < FOOTER_ENCODED_LENGTH) return corrupt("file is too short to be an sstable");
  // the device-only scan first (one synchronisation); it grows its own result capacity as needed. A filter
  // policy name too long for the device's metaindex key, or a workspace the device scan cannot get, leaves the
  // table to the paths below (read_meta opens such tables: table.rs:86-112).
  const bool key_fits = !filter_name || strlen(filter_name) + 6 <= sizeof(((lcrc_tscan_key*)nullptr)->key);
  if (key_fits) {
    uint64_t cap = std::max<uint64_t>(std::max<uint64_t>(max_blocks, ctx->ts_blocks.cap), 1024);
    lcrc_tscan_dev* hs = (lcrc_tscan_dev*)ctx->ts_host;
    bool ran = true;
    // up to three independent reasons to grow (the decoded index over the workspace -- reported first, as
    // ts_open_state stops there --, the result capacity, the decoded frames over the workspace), then the scan itself
    for (int attempt = 0; attempt < 4; ++attempt) {
      rc = ctx->ts_blocks.ensure(cap);
      if (!rc) rc = ctx->ts_count.ensure(1);
      if (!rc)
        rc = lcrc_table_scan_async_ex(ctx, file, file_len, filter_name, (lcrc_tblk*)ctx->ts_blocks.p, cap,
                                      ctx->ts_count.p, ctx->ts_count_status, LCRC_TSCAN_SNAPPY_INDEX, nullptr);
      if (rc == LCRC_ENOMEM) {  // no workspace for the device-only scan: the paths below (other errors propagate)
        ran = false;
        break;
      }
      if (rc) return rc;
      HIPCHK(hipMemcpyAsync(hs, ctx->ts_state.p, sizeof(lcrc_tscan_dev), hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      if (hs->status == 3) {  // capacity: grow to what the table needs and scan again
        cap = std::max<uint64_t>(hs->n_data + 16, cap * 2);
      } else if (hs->status == 2 && hs->gate == 1) {  // decoded frames or index over the workspace: grow it, scan again
        rc = ts_reserve(ctx, file_len, cap, hs->need_out + hs->need_out / 4 + 4096);
        if (rc == LCRC_ENOMEM) {
          ran = false;
          break;
        }
        if (rc) return rc;
      } else {
        break;
      }
    }
    if (ran && hs->status == 1) return corrupt(lcrc_table_scan_message(hs->code));
    if (ran && hs->status == 0) {
      const size_t n = hs->n_total;
      *n_blocks = n;
      if (!blocks || max_blocks < n) return LCRC_ERANGE;
      HIPCHK(hipMemcpyAsync(blocks, ctx->ts_blocks.p, n * sizeof(lcrc_tblk), hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      if (hs->unsorted)
        std::stable_sort(blocks, blocks + n, [](const lcrc_tblk& a, const lcrc_tblk& b) { return a.offset < b.offset; });
      return LCRC_OK;
    }
    // status 2: what the device walk cannot vouch for (a Snappy-framed index or metaindex, long restart
    // segments, a handle past the file, decoded frames over the workspace) -- the paths below
  }
  uint8_t footer[FOOTER_ENCODED_LENGTH];
  HIPCHK(hipMemcpy(footer, file + file_len - FOOTER_ENCODED_LENGTH, FOOTER_ENCODED_LENGTH, hipMemcpyDeviceToHost));
  Handle meta_h, index_h;
  if (const char* e = decode_footer(footer, meta_h, index_h)) return corrupt(e);
  rc = table_scan_device(ctx, file, file_len, filter_name, meta_h, index_h, blocks, max_blocks, n_blocks,
                         [&](const char* m) { return corrupt(m); });
  if (rc != TBL_FALLBACK) return rc;
  *n_blocks = 0;
  // the host walk (an index block the segmented device walk cannot vouch for: the reference's messages)

  std::vector<lcrc_tblk> found;
  auto add = [&](const Handle& h, uint8_t kind) {
    lcrc_tblk b;
    memset(&b, 0, sizeof(b));
    b.offset = h.offset;
    b.size = h.size;
    b.kind = kind;
    found.push_back(b);
  };
  // Table::open: the index block is read with verify_checksum = paranoid_checks (true here)
  std::vector<uint8_t> raw, contents;
  if (const char* e = read_raw(index_h, raw)) return corrupt(e);
  if (const char* e = block_contents(raw.data(), index_h.size, true, ctx->mode, ctx->flags, contents))
    return corrupt(e);
  const char* herr = nullptr;
  const char* berr = block_entries(contents, [&](const std::string&, const uint8_t* v, uint32_t vn) {
    Handle h;
    const uint8_t* p = v;
    if ((herr = decode_handle(p, v + vn, h))) return false;
    add(h, LCRC_TBLK_DATA);
    return true;
  });
  if (berr) return corrupt(berr);
  if (herr) return corrupt(herr);
  // read_meta: only with a filter policy, and its errors are not propagated (table.rs:81-103)
  if (filter_name && !read_raw(meta_h, raw) &&
      !block_contents(raw.data(), meta_h.size, true, ctx->mode, ctx->flags, contents)) {
    const std::string want = std::string("filter") + filter_name;
    block_entries(contents, [&](const std::string& key, const uint8_t* v, uint32_t vn) {
      if (key < want) return true;  // seek: first key >= want
      Handle h;
      const uint8_t* p = v;
      if (key == want && !decode_handle(p, v + vn, h)) add(h, LCRC_TBLK_FILTER);
      return false;
    });
  }
  add(meta_h, LCRC_TBLK_METAINDEX);
  add(index_h, LCRC_TBLK_INDEX);
  std::stable_sort(found.begin(), found.end(),
                   [](const lcrc_tblk& a, const lcrc_tblk& b) { return a.offset < b.offset; });
  const size_t n = found.size();
  *n_blocks = n;
  if (!blocks || max_blocks < n) return LCRC_ERANGE;

  // ONE batched pass over the file for every block in range
  std::vector<lcrc_desc_dev> descs;
  std::vector<uint64_t> pos;
  std::vector<size_t> which;
  for (size_t i = 0; i < n; ++i) {
    lcrc_tblk& b = found[i];
    if (b.offset > file_len || b.size + BLOCK_TRAILER_SIZE > file_len - b.offset || b.size + 1 > 0xFFFFFFFFull) {
      b.status = LCRC_TBLK_TRUNCATED;
      b.type = 0xFF;
      continue;
    }
    lcrc_desc_dev d;
    d.offset = b.offset;
    d.length = (uint32_t)(b.size + 1);
    d.expect_rel = (int32_t)(b.size + 1);
    if ((uint64_t)d.expect_rel != b.size + 1) d.expect_rel = LCRC_NO_EXPECT_DEV;  // > 2 GiB block
    descs.push_back(d);
    pos.push_back(b.offset + b.size);
    which.push_back(i);
  }
  const size_t m = descs.size();
  if (m) {
    if ((rc = ctx->tbl_descs.ensure(m)) || (rc = ctx->tbl_crcs.ensure(m)) || (rc = ctx->tbl_mm.ensure((m + 31) / 32)) ||
        (rc = ctx->tbl_pos.ensure(m)) || (rc = ctx->tbl_types.ensure(m)))
      return rc;
    HIPCHK(hipMemcpyAsync(ctx->tbl_descs.p, descs.data(), m * sizeof(lcrc_desc_dev), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(ctx->tbl_pos.p, pos.data(), m * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    if ((rc = lcrc_batch(ctx, file, file_len, (const lcrc_desc*)ctx->tbl_descs.p, m, ctx->tbl_crcs.p, ctx->tbl_mm.p,
                         st)))
      return rc;
    HIPCHK(lcrc_launch_gather_u8(file, ctx->tbl_pos.p, m, ctx->tbl_types.p, st));
    std::vector<uint32_t> crcs(m), mm((m + 31) / 32);
    std::vector<uint8_t> types(m);
    HIPCHK(hipMemcpyAsync(crcs.data(), ctx->tbl_crcs.p, m * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(mm.data(), ctx->tbl_mm.p, mm.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(types.data(), ctx->tbl_types.p, m, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    std::vector<lcrc_desc_dev> frames;
    std::vector<size_t> fwhich;
    for (size_t k = 0; k < m; ++k) {
      lcrc_tblk& b = found[which[k]];
      b.crc = crcs[k];
      b.type = types[k];
      b.status = ((mm[k >> 5] >> (k & 31)) & 1) ? LCRC_TBLK_CRC_MISMATCH : LCRC_TBLK_OK;
      // read_block_from_file's type dispatch after a good checksum (format.rs:175-210)
      if (b.status == LCRC_TBLK_OK && b.type > 1) b.status = LCRC_TBLK_BAD_TYPE;
      if (b.status == LCRC_TBLK_OK && b.type == 1 && b.size <= 0xFFFFFFFFull) {
        lcrc_desc_dev f;
        f.offset = b.offset;
        f.length = (uint32_t)b.size;
        f.expect_rel = LCRC_NO_EXPECT_DEV;
        frames.push_back(f);
        fwhich.push_back(which[k]);
      }
    }
    // Snappy-framed blocks: decoded and their chunk CRCs checked on the device, all in one batch
    const size_t nf = frames.size();
    if (nf) {
      if ((rc = ctx->tbl_descs.ensure(nf)) || (rc = ctx->sn_out_off.ensure(nf + 1)) || (rc = ctx->sn_status.ensure(nf)))
        return rc;
      HIPCHK(hipMemcpyAsync(ctx->tbl_descs.p, frames.data(), nf * sizeof(lcrc_desc_dev), hipMemcpyHostToDevice, st));
      uint64_t total = 0;
      rc = snappy_frames_impl(ctx, file, ctx->tbl_descs.p, nf, ctx->sn_out.p, ctx->sn_out.cap, ctx->sn_out_off.p,
                              ctx->sn_status.p, &total, st);
      if (rc == LCRC_ERANGE) {
        if ((rc = ctx->sn_out.ensure(total))) return rc;
        rc = snappy_frames_impl(ctx, file, ctx->tbl_descs.p, nf, ctx->sn_out.p, ctx->sn_out.cap, ctx->sn_out_off.p,
                                ctx->sn_status.p, &total, st);
      }
      if (rc) return rc;
      std::vector<uint8_t> fst(nf);
      HIPCHK(hipMemcpy(fst.data(), ctx->sn_status.p, nf, hipMemcpyDeviceToHost));
      for (size_t k = 0; k < nf; ++k)
        if (fst[k]) found[fwhich[k]].status = LCRC_TBLK_BAD_CONTENT;
    }
  }
  memcpy(blocks, found.data(), n * sizeof(lcrc_tblk));
  return LCRC_OK;
}

// ---- writer side: batch seal ----
int lcrc_batch_seal(lcrc_ctx* ctx, uint8_t* base, uint64_t base_len, const lcrc_desc* descs, size_t n,
                    uint32_t* out_crc, void* stream) {
  TkScope tk_scope(ctx);
  if (!ctx || (n && (!descs || !base))) return LCRC_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  if (n == 0) return LCRC_OK;
  hipStream_t st = pick_stream(ctx, stream);
  uint32_t* crc = out_crc;
  if (!crc) {
    if ((rc = ctx->tbl_crcs.ensure(n))) return rc;
    crc = ctx->tbl_crcs.p;
  }
  if ((rc = lcrc_batch(ctx, base, base_len, descs, n, crc, nullptr, st))) return rc;
  HIPCHK(lcrc_launch_store_crc(base, base_len, (const lcrc_desc_dev*)descs, crc, n, st));
  return LCRC_OK;
}

// ---- device memory helpers ----
int lcrc_dev_alloc(int device, size_t bytes, void** out) {
  if (!out) return LCRC_EINVAL;
  *out = nullptr;
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipMalloc(out, bytes ? bytes : 1));
  return LCRC_OK;
}
int lcrc_dev_free(void* p) {
  if (p) HIPCHK(hipFree(p));
  return LCRC_OK;
}
int lcrc_host_alloc_pinned(size_t bytes, void** out) {
  if (!out) return LCRC_EINVAL;
  HIPCHK(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
  return LCRC_OK;
}
int lcrc_host_free_pinned(void* p) {
  if (p) HIPCHK(hipHostFree(p));
  return LCRC_OK;
}
int lcrc_memcpy_h2d(void* dst, const void* src, size_t bytes) {
  HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return LCRC_OK;
}
int lcrc_memcpy_d2h(void* dst, const void* src, size_t bytes) {
  HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return LCRC_OK;
}
int lcrc_memset_d(void* dst, int value, size_t bytes) {
  // finished when this returns (a fill left queued on the null stream is not ordered before the contexts'
  // non-blocking streams)
  HIPCHK(hipMemsetAsync(dst, value, bytes, nullptr));
  HIPCHK(hipStreamSynchronize(nullptr));
  return LCRC_OK;
}
int lcrc_device_sync(void) {
  HIPCHK(hipDeviceSynchronize());
  return LCRC_OK;
}
int lcrc_graph_begin(lcrc_ctx* ctx) {
  if (!ctx) return LCRC_EINVAL;
  int rc = set_device(ctx);
  if (rc) return rc;
  // the queue lanes (lcrc_batch_queue, lcrc_wal_scan_queue) exist before the capture starts: a first-ever queued
  // call inside the capture then creates no stream
  if ((rc = ensure_lanes(ctx))) return rc;
  HIPCHK(hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
  return LCRC_OK;
}
int lcrc_graph_end(lcrc_ctx* ctx, void** graph_exec) {
  if (!ctx || !graph_exec) return LCRC_EINVAL;
  *graph_exec = nullptr;
  hipGraph_t g = nullptr;
  HIPCHK(hipStreamEndCapture(ctx->stream, &g));
  hipGraphExec_t ge = nullptr;
  hipError_t e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) return fail_hip(e, "hipGraphInstantiate");
  *graph_exec = (void*)ge;
  return LCRC_OK;
}
int lcrc_graph_launch(lcrc_ctx* ctx, void* graph_exec) {
  if (!ctx || !graph_exec) return LCRC_EINVAL;
  HIPCHK(hipGraphLaunch((hipGraphExec_t)graph_exec, ctx->stream));
  return LCRC_OK;
}
int lcrc_graph_destroy(void* graph_exec) {
  if (graph_exec) HIPCHK(hipGraphExecDestroy((hipGraphExec_t)graph_exec));
  return LCRC_OK;
}

int lcrc_timer_start(lcrc_ctx* ctx) {
  if (!ctx) return LCRC_EINVAL;
  ctx->tk_armed0 = false;
  HIPCHK(hipEventRecord(ctx->t0, ctx->stream));
  return LCRC_OK;
}
int lcrc_timer_stop(lcrc_ctx* ctx, float* ms) {
  if (!ctx || !ms) return LCRC_EINVAL;
  if (ctx->tk_stop) {  // kernel-carried: the events are the first and last launches' own start and end
    const bool any = ctx->tk_any && ctx->tk_end;
    ctx->tk_start = ctx->tk_stop = ctx->tk_any = ctx->tk_end = ctx->tk_armed0 = false;
    if (!any) return LCRC_EINVAL;
  } else {
    // start carried by a launch (edge 0), stop recorded here: a start that no launch recorded leaves t0 stale
    const bool stale = ctx->tk_armed0 && !ctx->tk_any;
    ctx->tk_start = ctx->tk_any = ctx->tk_armed0 = false;
    if (stale) {
      g_last_error = "lcrc_timer_stop: edge 0 was armed but no launch recorded the start event";
      return LCRC_EINVAL;
    }
    HIPCHK(hipEventRecord(ctx->t1, ctx->stream));
  }
  HIPCHK(hipEventSynchronize(ctx->t1));
  HIPCHK(hipEventElapsedTime(ms, ctx->t0, ctx->t1));
  return LCRC_OK;
}
// Fast-path launches carry the timer's events themselves (hipExtLaunchKernelGGL): edge 0 -- the next launch
// records t0 at its start; edge 1 -- the launches from the next one on record t1 at their end (the last one
// wins); edge 2 -- disarm. No marker packet between launches, no host latency before the first kernel. Ended by
// lcrc_timer_stop.
int lcrc_timer_kernels(lcrc_ctx* ctx, int edge) {
  if (!ctx || edge < 0 || edge > 2) return LCRC_EINVAL;
  if (edge == 2) {  // disarm
    ctx->tk_start = ctx->tk_stop = ctx->tk_any = ctx->tk_end = ctx->tk_armed0 = false;
  } else if (edge == 0) {
    ctx->tk_start = true;
    ctx->tk_any = false;
    ctx->tk_armed0 = true;
  } else {
    ctx->tk_stop = true;
    ctx->tk_end = false;
  }
  return LCRC_OK;
}
// Kernel-carried timing over several contexts (one stream each, same device): from `first`'s start event to
// `last`'s stop event. The caller arms edge 0 on the context of the first timed launch and edge 1 on every
// context before its last timed launch, then takes the largest span over the contexts. Waits for `last`'s
// stop event; the timers stay armed until lcrc_timer_stop (or lcrc_timer_kernels) resets them.
int lcrc_timer_span(lcrc_ctx* first, lcrc_ctx* last, float* ms) {
  if (!first || !last || !ms || first->device != last->device) return LCRC_EINVAL;
  if (!first->tk_any || !last->tk_stop || !last->tk_end) return LCRC_EINVAL;
  HIPCHK(hipEventSynchronize(last->t1));
  HIPCHK(hipEventElapsedTime(ms, first->t0, last->t1));
  return LCRC_OK;
}

}  // extern "C"
