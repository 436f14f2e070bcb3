// Prototype: fixed-size block CRC (slice-by-4, LDS tables replicated x32, lane windows of S bytes,
// lane-tree combine with per-level shift tables). Measures GB/s and checks vs a CPU CRC.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>
#include <chrono>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

static const uint32_t POLY_C = 0x82F63B78u;

// ---------------- host tables ----------------
struct Op { uint32_t col[32]; };
static uint32_t op_apply(const Op& o, uint32_t v) { uint32_t r = 0; for (int i = 0; i < 32; ++i) if (v >> i & 1) r ^= o.col[i]; return r; }
static Op op_mul(const Op& a, const Op& b) { Op r; for (int i = 0; i < 32; ++i) r.col[i] = op_apply(a, b.col[i]); return r; }
static Op op_zero_bytes(uint32_t poly, uint64_t n) {
  Op bit; bit.col[0] = poly; for (int i = 1; i < 32; ++i) bit.col[i] = 1u << (i - 1);
  Op byte = bit; for (int i = 0; i < 3; ++i) byte = op_mul(byte, byte);
  Op r; for (int i = 0; i < 32; ++i) r.col[i] = 1u << i;
  Op p = byte;
  while (n) { if (n & 1) r = op_mul(p, r); p = op_mul(p, p); n >>= 1; }
  return r;
}
static void make_slice4(uint32_t poly, uint32_t* T /*4*256*/) {
  for (int b = 0; b < 256; ++b) { uint32_t c = b; for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (poly & (0u - (c & 1))); T[b] = c; }
  for (int t = 1; t < 4; ++t) for (int b = 0; b < 256; ++b) T[t * 256 + b] = (T[(t - 1) * 256 + b] >> 8) ^ T[T[(t - 1) * 256 + b] & 0xff];
}
static void make_shift(uint32_t poly, uint64_t nbytes, uint32_t* Z /*4*256*/) {
  Op o = op_zero_bytes(poly, nbytes);
  for (int k = 0; k < 4; ++k) for (int b = 0; b < 256; ++b) Z[k * 256 + b] = op_apply(o, (uint32_t)b << (8 * k));
}
static uint32_t cpu_crc(const uint32_t* T, const uint8_t* p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = (c >> 8) ^ T[(c ^ p[i]) & 0xff];
  return c ^ 0xFFFFFFFFu;
}

// ---------------- device ----------------
#define REP 32
template <int S, int L>
__global__ void __launch_bounds__(1024) k_crc_fixed(const uint8_t* __restrict__ data, uint32_t nblocks,
                                                     const uint32_t* __restrict__ gt, uint32_t* __restrict__ out) {
  constexpr int G = L / S;          // lanes per block
  constexpr int LEVELS = __builtin_ctz(G);
  constexpr int BPW = 64 / G;       // blocks per wave-task
  extern __shared__ uint32_t lds[];
  uint32_t* tz = lds + 4 * 256 * REP;  // tree tables, LEVELS*4*256
  for (int i = threadIdx.x; i < 4 * 256 * REP; i += blockDim.x) lds[i] = gt[i >> 5];
  for (int i = threadIdx.x; i < LEVELS * 4 * 256; i += blockDim.x) tz[i] = gt[4 * 256 + i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int g = lane & (G - 1);
  const uint32_t laneoff = (lane & 31) * 4;
  const char* lb = (const char*)lds;
  const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
  const uint32_t wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint32_t ntasks = (nblocks + BPW - 1) / BPW;
  for (uint32_t t = wave; t < ntasks; t += nwaves) {
    uint32_t blk = t * BPW + (lane / G);
    bool valid = blk < nblocks;
    const u32x4* w = (const u32x4*)(data + (size_t)(valid ? blk : 0) * L + (size_t)g * S);
    u32x4 v[S / 16];
#pragma unroll
    for (int j = 0; j < S / 16; ++j) v[j] = __builtin_nontemporal_load(w + j);
    __builtin_amdgcn_sched_barrier(0);
    uint32_t r = (g == 0) ? 0xFFFFFFFFu : 0u;
#pragma unroll
    for (int j = 0; j < S / 16; ++j) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t x = r ^ v[j][q];
        uint32_t a0 = ((x << 7) & 0x7f80u) | laneoff;
        uint32_t a1 = ((x >> 1) & 0x7f80u) | laneoff;
        uint32_t a2 = ((x >> 9) & 0x7f80u) | laneoff;
        uint32_t a3 = ((x >> 17) & 0x7f80u) | laneoff;
        uint32_t t3 = *(const uint32_t*)(lb + a0 + 3 * 32768);
        uint32_t t2 = *(const uint32_t*)(lb + a1 + 2 * 32768);
        uint32_t t1 = *(const uint32_t*)(lb + a2 + 1 * 32768);
        uint32_t t0 = *(const uint32_t*)(lb + a3);
        r = t0 ^ t1 ^ t2 ^ t3;
      }
    }
#pragma unroll
    for (int m = 0; m < LEVELS; ++m) {
      uint32_t partner = __shfl_down(r, 1 << m, 64);
      const uint32_t* z = tz + m * 1024;
      uint32_t sh = z[r & 0xff] ^ z[256 + ((r >> 8) & 0xff)] ^ z[512 + ((r >> 16) & 0xff)] ^ z[768 + (r >> 24)];
      if ((g & ((2 << m) - 1)) == 0) r = sh ^ partner;
    }
    if (g == 0 && valid) out[blk] = r ^ 0xFFFFFFFFu;
  }
}

template <typename F>
static float time_it(F f, int iters) {
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  f(0); (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int i = 0; i < iters; ++i) f(i);
  (void)hipEventRecord(b); (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b);
  return ms / iters;
}

template <int S>
static int run(uint8_t* buf, size_t NB, int NBUF, const std::vector<uint8_t>& host0, const uint32_t* T, uint32_t* dout, int ncu) {
  constexpr int L = 4096, G = L / S, LEVELS = __builtin_ctz(G);
  std::vector<uint32_t> gt(4 * 256 + LEVELS * 1024);
  make_slice4(POLY_C, gt.data());
  for (int m = 0; m < LEVELS; ++m) make_shift(POLY_C, (uint64_t)S << m, gt.data() + 1024 + m * 1024);
  uint32_t* dgt; CK(hipMalloc(&dgt, gt.size() * 4));
  CK(hipMemcpy(dgt, gt.data(), gt.size() * 4, hipMemcpyHostToDevice));
  size_t lds = (4 * 256 * REP + LEVELS * 1024) * 4;
  CK(hipFuncSetAttribute((const void*)k_crc_fixed<S, L>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  uint32_t nblocks = NB / L;
  k_crc_fixed<S, L><<<ncu, 1024, lds>>>(buf, nblocks, dgt, dout);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> got(nblocks);
  CK(hipMemcpy(got.data(), dout, nblocks * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (uint32_t b = 0; b < nblocks; b += 97) if (got[b] != cpu_crc(T, host0.data() + (size_t)b * L, L)) ++bad;
  if (got[nblocks - 1] != cpu_crc(T, host0.data() + (size_t)(nblocks - 1) * L, L)) ++bad;
  float ms = time_it([&](int i) { k_crc_fixed<S, L><<<ncu, 1024, lds>>>(buf + (i % NBUF) * NB, nblocks, dgt, dout); }, 40);
  printf("crc S=%3d G=%2d: %s  %.3f ms  %.1f GB/s (%.1f%% of 8TB/s)\n", S, G, bad ? "BAD" : "ok", ms, NB / ms / 1e6, NB / ms / 1e6 / 80.0);
  (void)hipFree(dgt);
  return 0;
}

__global__ void k_fill(uint8_t* p, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t nth = (size_t)gridDim.x * blockDim.x;
  for (; i < n / 8; i += nth) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull + 0x5EED;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; z ^= z >> 31;
    ((uint64_t*)p)[i] = z;
  }
}

int main() {
  const size_t NB = 256ull << 20;
  const int NBUF = 4;
  uint8_t* buf; CK(hipMalloc(&buf, NB * NBUF));
  uint32_t* dout; CK(hipMalloc(&dout, (NB / 4096) * 4));
  k_fill<<<4096, 256>>>(buf, NB * NBUF);
  CK(hipDeviceSynchronize());
  std::vector<uint8_t> host0(NB);
  CK(hipMemcpy(host0.data(), buf, NB, hipMemcpyDeviceToHost));
  uint32_t T[1024]; make_slice4(POLY_C, T);
  // sanity: check value
  printf("cpu crc32c(123456789)=%08x\n", cpu_crc(T, (const uint8_t*)"123456789", 9));
  int ncu = 0; (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  run<64>(buf, NB, NBUF, host0, T, dout, ncu);
  run<128>(buf, NB, NBUF, host0, T, dout, ncu);
  run<256>(buf, NB, NBUF, host0, T, dout, ncu);
  return 0;
}
