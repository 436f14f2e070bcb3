// Memory-skeleton probe for k_windows: the same region/half-tile load structure with the walk replaced by
// an xor fold, so the load pattern, depth, workgroup shape and ticketing can be varied in isolation.
//   PAT 0: k_windows' pattern -- lane (k, c) loads region byte 2048 j + 256 k + 128 h + 16 c
//   PAT 1: contiguous         -- lane l loads region byte 1024 (8 h + j) + 16 l
//   REFILL 0: a half is refilled while it is consumed (up to 16 loads in flight per wave)
//   REFILL 1: a half is refilled after the OTHER half has been consumed (up to 8 in flight)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);          \
      return 1;                                                                \
    }                                                                          \
  } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int REGION = 16384;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const uint8_t* base, uint64_t t, uint64_t nreg) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (t < nreg ? t : 0) * REGION), (short)0,
                                           t < nreg ? REGION : 0, 0x00020000);
}

template <int PAT>
__device__ __forceinline__ uint32_t voff(uint32_t lane, int h, int j) {
  if (PAT == 0) return 2048u * j + 256u * (lane & 7) + 128u * h + 16u * (lane >> 3);
  return 1024u * (8 * h + j) + 16u * lane;
}

//   ASSIGN 0: contiguous share per workgroup, LDS tickets; 1: per-wave grid stride (static);
//   2: per-workgroup grid stride (region b + G v), LDS tickets
template <int PAT, int THREADS, int REFILL, int WORK, int ASSIGN = 0>
__global__ void __launch_bounds__(THREADS) k_skel(const uint8_t* __restrict__ base, uint64_t nreg, uint32_t* out) {
  __shared__ uint32_t ticket;
  const uint32_t lane = __lane_id();
  const uint64_t per = (nreg + gridDim.x - 1) / gridDim.x;
  const uint64_t lo = (uint64_t)blockIdx.x * per;
  const uint64_t cnt = lo < nreg ? (nreg - lo < per ? nreg - lo : per) : 0;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr uint32_t W = THREADS / 64;
  const uint64_t gw = (uint64_t)blockIdx.x * W + wv, nw = (uint64_t)gridDim.x * W;
  uint32_t mine = 0;
  auto region = [&](uint32_t v) -> uint64_t {
    if (ASSIGN == 1) return gw + (uint64_t)v * nw < nreg ? gw + (uint64_t)v * nw : ~0ull;
    if (ASSIGN == 2) return blockIdx.x + (uint64_t)v * gridDim.x < nreg ? blockIdx.x + (uint64_t)v * gridDim.x : ~0ull;
    return v < cnt ? lo + v : ~0ull;
  };
  auto take = [&]() -> uint64_t {
    if (ASSIGN == 1) return region(++mine);
    uint32_t v = 0;
    if (lane == 0) v = atomicAdd(&ticket, 1u);
    return region(__builtin_amdgcn_readfirstlane(v));
  };
  uint64_t t = ASSIGN == 1 ? region(0) : region(wv);
  u32x4 va[8], vb[8];
  {
    auto rs = rsrc(base, t, nreg);
#pragma unroll
    for (int j = 0; j < 8; ++j) va[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff<PAT>(lane, 0, j), 0, 2);
#pragma unroll
    for (int j = 0; j < 8; ++j) vb[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff<PAT>(lane, 1, j), 0, 2);
  }
  if (threadIdx.x == 0) ticket = THREADS / 64;
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  uint64_t tn = take();
  uint32_t acc = 0;
  auto consume = [&](u32x4(&v)[8], int h, __amdgpu_buffer_rsrc_t rs, bool refill) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint32_t x = v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
#pragma unroll
      for (int w = 0; w < WORK; ++w) x = __builtin_amdgcn_perm(x, x * 0x9E3779B9u, 0x05040302u) ^ (x >> 3);
      acc ^= x;
      if (refill) v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff<PAT>(lane, h, j), 0, 2);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  while (t != ~0ull) {
    auto rsn = rsrc(base, tn, nreg);
    if (REFILL == 0) {
      consume(va, 0, rsn, true);
      const uint64_t tnn = take();
      consume(vb, 1, rsn, true);
      t = tn;
      tn = tnn;
    } else {
      consume(va, 0, rsn, false);
#pragma unroll
      for (int j = 0; j < 8; ++j) va[j] = __builtin_amdgcn_raw_buffer_load_b128(rsn, voff<PAT>(lane, 0, j), 0, 2);
      const uint64_t tnn = take();
      consume(vb, 1, rsn, false);
#pragma unroll
      for (int j = 0; j < 8; ++j) vb[j] = __builtin_amdgcn_raw_buffer_load_b128(rsn, voff<PAT>(lane, 1, j), 0, 2);
      t = tn;
      tn = tnn;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_fill(uint8_t* p, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t nth = (size_t)gridDim.x * blockDim.x;
  for (; i < n / 8; i += nth) ((uint64_t*)p)[i] = i * 0x9E3779B97F4A7C15ull;
}

template <typename F>
static float best_ms(F f, int iters) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float best = 1e9;
  for (int rep = 0; rep < 3; ++rep) {
    for (int i = 0; i < 3; ++i) f(i);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    for (int i = 0; i < iters; ++i) f(i);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    if (ms / iters < best) best = ms / iters;
  }
  return best;
}

int main() {
  const size_t NB = 256ull << 20;
  const int NBUF = 4;
  uint8_t* buf;
  CK(hipMalloc(&buf, NB * NBUF));
  uint32_t* out;
  CK(hipMalloc(&out, 4096));
  k_fill<<<4096, 256>>>(buf, NB * NBUF);
  CK(hipDeviceSynchronize());
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const uint64_t nreg = NB / REGION;
  auto rep = [&](const char* name, float ms) { printf("%-40s %7.1f us  %7.1f GB/s\n", name, ms * 1e3, NB / ms / 1e6); };
#define RUN(PAT, TH, WPC, RF, WK, AS)                                                                        \
  rep("pat" #PAT " thr" #TH " wg/cu" #WPC " refill" #RF " work" #WK " assign" #AS,                            \
      best_ms([&](int i) { k_skel<PAT, TH, RF, WK, AS><<<ncu * WPC, TH>>>(buf + (i % NBUF) * NB, nreg, out); }, 50));
  RUN(0, 512, 1, 0, 0, 0)
  RUN(0, 512, 1, 0, 0, 1)
  RUN(0, 512, 1, 0, 0, 2)
  RUN(0, 512, 1, 1, 0, 0)
  RUN(0, 512, 1, 1, 0, 1)
  RUN(1, 512, 1, 0, 0, 1)
  RUN(1, 512, 1, 1, 0, 1)
  RUN(0, 512, 2, 0, 0, 0)
  RUN(0, 512, 2, 0, 0, 1)
  RUN(0, 256, 4, 0, 0, 0)
  RUN(0, 256, 4, 0, 0, 1)
  RUN(0, 512, 1, 0, 8, 0)
  RUN(0, 512, 1, 0, 8, 1)
  RUN(0, 512, 1, 0, 0, 0)
  return 0;
}
