// Microbenchmark: the k_windows streaming skeleton (1024-thread workgroups, one per CU, two register
// buffers of 8 x 16 B per lane, refill-while-consuming) with different per-instruction address patterns
// and an artificial dependent VALU delay standing in for the CRC walk.
//   pattern 0: buffer = one contiguous 8 KiB tile; instruction j reads bytes [1024 j, 1024 j + 1024)
//   pattern 1: 16 KiB region, buffer h reads half h of every 256 B: 2048 j + 256 k + 128 h + 16 c
//   pattern 2: as 1, but the first 8 KiB (buffer a) and second 8 KiB (buffer b) are separate
//              contiguous tiles of the same region (instruction j: 1024 j + 16 lane' (+8192))
// Usage: probe_pattern  -> prints one line per (pattern, delay, 256 MiB launch)
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const uint8_t* base, uint64_t span, uint64_t off, uint32_t n) {
  uint32_t nrec = 0;
  if (off < span) nrec = (span - off) < n ? (uint32_t)(span - off) : n;
  return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (off < span ? off : 0)), (short)0, (int)nrec, 0x00020000);
}

__device__ __forceinline__ uint32_t consume(u32x4 (&v)[8], int delay) {
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
  for (int i = 0; i < delay; ++i) acc = acc * 0x9E3779B1u + 0x7F4A7C15u;
  return acc;
}

template <int P>
__global__ void __launch_bounds__(1024) k_pat(const uint8_t* __restrict__ base, uint64_t span, int delay,
                                              uint32_t* out) {
  const uint32_t lane = __lane_id();
  const uint64_t nwaves = (uint64_t)gridDim.x * 16;
  uint64_t t = (uint64_t)blockIdx.x * 16 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nreg = span / 16384;
  uint32_t offa[8], offb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (P != 2) {
      offa[j] = 2048 * j + 256 * (lane & 7) + 16 * (lane >> 3);
      offb[j] = offa[j] + 128;
    } else {
      offa[j] = 1024 * j + 16 * (8 * (lane & 7) + (lane >> 3));
      offb[j] = offa[j] + 8192;
    }
  }
  u32x4 va[8], vb[8];
  {
    auto rs = rsrc(base, span, t * 16384, 16384);
#pragma unroll
    for (int j = 0; j < 8; ++j) va[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, offa[j], 0, 2);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 8; ++j) vb[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, offb[j], 0, 2);
  }
  uint32_t acc = 0;
  uint32_t pf = 0;
  for (; t < nreg; t += nwaves) {
    auto rs = rsrc(base, span, (t + nwaves) * 16384, P == 5 ? 0 : 16384);
    if (P == 7) {
      auto rp = rsrc(base, span, (t + 2 * nwaves) * 16384, 16384);
      pf ^= __builtin_amdgcn_raw_buffer_load_b32(rp, lane * 128, 0, 0);
      pf ^= __builtin_amdgcn_raw_buffer_load_b32(rp, 8192 + lane * 128, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    acc ^= consume(va, delay);
    if (P != 6) {
#pragma unroll
      for (int j = 0; j < 8; ++j) va[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, offa[j], 0, 2);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) va[j] += acc;
    }
    __builtin_amdgcn_sched_barrier(0);
    acc ^= consume(vb, delay);
    if (P != 6) {
#pragma unroll
      for (int j = 0; j < 8; ++j) vb[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, offb[j], 0, 2);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) vb[j] += acc;
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  acc ^= pf;
  if (acc == 0x12345678u) out[lane] = acc;
}

// pattern 3: 512-thread workgroups (2 waves per SIMD, up to 256 VGPRs), four buffers: region t's halves
// in a0/b0, region t + n's in a1/b1; each refill targets the region two steps ahead
__global__ void __launch_bounds__(512) k_pat4(const uint8_t* __restrict__ base, uint64_t span, int delay,
                                              uint32_t* out) {
  const uint32_t lane = __lane_id();
  const uint64_t nwaves = (uint64_t)gridDim.x * 8;
  uint64_t t = (uint64_t)blockIdx.x * 8 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nreg = span / 16384;
  uint32_t offa[8], offb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    offa[j] = 2048 * j + 256 * (lane & 7) + 16 * (lane >> 3);
    offb[j] = offa[j] + 128;
  }
  u32x4 a0[8], b0[8], a1[8], b1[8];
  {
    auto rs = rsrc(base, span, t * 16384, 16384);
#pragma unroll
    for (int j = 0; j < 8; ++j) a0[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, offa[j], 0, 2);
#pragma unroll
    for (int j = 0; j < 8; ++j) b0[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, offb[j], 0, 2);
    __builtin_amdgcn_sched_barrier(0);
    rs = rsrc(base, span, (t + nwaves) * 16384, 16384);
#pragma unroll
    for (int j = 0; j < 8; ++j) a1[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, offa[j], 0, 2);
#pragma unroll
    for (int j = 0; j < 8; ++j) b1[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, offb[j], 0, 2);
  }
  uint32_t acc = 0;
  for (; t < nreg; t += 2 * nwaves) {
    auto rs = rsrc(base, span, (t + 2 * nwaves) * 16384, 16384);
    __builtin_amdgcn_sched_barrier(0);
    acc ^= consume(a0, delay);
#pragma unroll
    for (int j = 0; j < 8; ++j) a0[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, offa[j], 0, 2);
    __builtin_amdgcn_sched_barrier(0);
    acc ^= consume(b0, delay);
#pragma unroll
    for (int j = 0; j < 8; ++j) b0[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, offb[j], 0, 2);
    __builtin_amdgcn_sched_barrier(0);
    rs = rsrc(base, span, (t + 3 * nwaves) * 16384, 16384);
    acc ^= consume(a1, delay);
#pragma unroll
    for (int j = 0; j < 8; ++j) a1[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, offa[j], 0, 2);
    __builtin_amdgcn_sched_barrier(0);
    acc ^= consume(b1, delay);
#pragma unroll
    for (int j = 0; j < 8; ++j) b1[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, offb[j], 0, 2);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (acc == 0x12345678u) out[lane] = acc;
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
  uint32_t* out; CK(hipMalloc(&out, 4096));
  k_fill<<<4096, 256>>>(buf, NB * NBUF);
  CK(hipDeviceSynchronize());
  int ncu = 0; hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int delay : {0, 50, 100, 150}) {
    for (int p : {1, 5, 6, 7, 3}) {
      auto launch = [&](int i) {
        const uint8_t* bp = buf + (i % NBUF) * NB;
        if (p == 0) k_pat<0><<<ncu, 1024>>>(bp, NB, delay, out);
        else if (p == 1) k_pat<1><<<ncu, 1024>>>(bp, NB, delay, out);
        else if (p == 2) k_pat<2><<<ncu, 1024>>>(bp, NB, delay, out);
        else if (p == 3) k_pat4<<<ncu, 512>>>(bp, NB, delay, out);
        else if (p == 5) k_pat<5><<<ncu, 1024>>>(bp, NB, delay, out);
        else if (p == 6) k_pat<6><<<ncu, 1024>>>(bp, NB, delay, out);
        else if (p == 7) k_pat<7><<<ncu, 1024>>>(bp, NB, delay, out);
        else k_pat4<<<2 * ncu, 512>>>(bp, NB, delay, out);
      };
      for (int i = 0; i < 5; ++i) launch(i);
      float best = 1e9;
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(a);
        for (int i = 0; i < 50; ++i) launch(i);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        if (ms / 50 < best) best = ms / 50;
      }
      printf("pattern %d delay %4d: %7.1f us  %7.1f GB/s\n", p, delay, best * 1000, NB / best / 1e6);
    }
  }
  CK(hipGetLastError());
  return 0;
}
