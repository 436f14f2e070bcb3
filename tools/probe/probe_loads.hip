// Microbenchmark: HBM read patterns relevant to the batched CRC kernel.
//  A) fully coalesced 16 B/lane streaming read
//  B) lane-contiguous windows of S bytes (lane l reads [l*S, l*S+S) of a wave tile)
//  C) unaligned raw-buffer dwordx4 loads (correctness)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) k_coalesced(const u32x4* __restrict__ p, size_t n16, uint32_t* out) {
  size_t tid = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t nth = (size_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  size_t i = tid;
  for (; i + 3 * nth < n16; i += 4 * nth) {
    u32x4 a = __builtin_nontemporal_load(p + i);
    u32x4 b = __builtin_nontemporal_load(p + i + nth);
    u32x4 c = __builtin_nontemporal_load(p + i + 2 * nth);
    u32x4 d = __builtin_nontemporal_load(p + i + 3 * nth);
    acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
  }
  for (; i < n16; i += nth) { u32x4 a = p[i]; acc ^= a.x ^ a.y ^ a.z ^ a.w; }
  if (acc == 0x12345678u) out[tid & 1023] = acc;
}

template <int S>
__global__ void __launch_bounds__(256) k_window(const uint8_t* __restrict__ p, size_t nbytes, uint32_t* out) {
  // each wave owns tiles of 64*S bytes; lane reads its S-byte window
  const int lane = threadIdx.x & 63;
  size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
  size_t ntiles = nbytes / (64 * S);
  uint32_t acc = 0;
  for (size_t t = wave; t < ntiles; t += nwaves) {
    const u32x4* w = (const u32x4*)(p + t * (64 * S) + (size_t)lane * S);
    u32x4 v[S / 16];
#pragma unroll
    for (int j = 0; j < S / 16; ++j) v[j] = __builtin_nontemporal_load(w + j);
#pragma unroll
    for (int j = 0; j < S / 16; ++j) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
  }
  if (acc == 0x12345678u) out[lane] = acc;
}

__global__ void k_unaligned(const uint8_t* p, uint32_t size, uint32_t* out) {
  int lane = threadIdx.x;  // 64 lanes, offset = lane
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)size, 0x00020000);
  u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 7 + 1, 0, 0);
  out[lane * 4 + 0] = v.x; out[lane * 4 + 1] = v.y; out[lane * 4 + 2] = v.z; out[lane * 4 + 3] = v.w;
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

template <typename F>
static float time_it(F f, int iters) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  f(0);
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < iters; ++i) f(i);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / iters;
}

int main() {
  const size_t NB = 256ull << 20;  // 256 MiB per buffer
  const int NBUF = 4;
  uint8_t* buf; CK(hipMalloc(&buf, NB * NBUF + 4096));
  uint32_t* out; CK(hipMalloc(&out, 1 << 20));
  k_fill<<<4096, 256>>>(buf, NB * NBUF);
  CK(hipDeviceSynchronize());
  int ncu = 0; hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  printf("CUs %d\n", ncu);
  for (int blocks : {1024, 2048, 4096, 8192}) {
    float ms = time_it([&](int i) { k_coalesced<<<blocks, 256>>>((const u32x4*)(buf + (i % NBUF) * NB), NB / 16, out); }, 40);
    printf("coalesced  grid %5d: %.3f ms  %.1f GB/s\n", blocks, ms, NB / ms / 1e6);
  }
  for (int blocks : {1024, 2048, 4096}) {
    float ms = time_it([&](int i) { k_window<64><<<blocks, 256>>>(buf + (i % NBUF) * NB, NB, out); }, 40);
    printf("window S=64  grid %5d: %.3f ms  %.1f GB/s\n", blocks, ms, NB / ms / 1e6);
    ms = time_it([&](int i) { k_window<128><<<blocks, 256>>>(buf + (i % NBUF) * NB, NB, out); }, 40);
    printf("window S=128 grid %5d: %.3f ms  %.1f GB/s\n", blocks, ms, NB / ms / 1e6);
    ms = time_it([&](int i) { k_window<256><<<blocks, 256>>>(buf + (i % NBUF) * NB, NB, out); }, 40);
    printf("window S=256 grid %5d: %.3f ms  %.1f GB/s\n", blocks, ms, NB / ms / 1e6);
  }
  // unaligned check
  k_unaligned<<<1, 64>>>(buf, 1 << 20, out);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> got(256);
  std::vector<uint8_t> host(1024);
  CK(hipMemcpy(got.data(), out, 1024, hipMemcpyDeviceToHost));
  CK(hipMemcpy(host.data(), buf, 1024, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int w = 0; w < 4; ++w) {
      uint32_t e; memcpy(&e, host.data() + l * 7 + 1 + 4 * w, 4);
      if (e != got[l * 4 + w]) ++bad;
    }
  printf("unaligned buffer_load_b128: %s (%d bad dwords)\n", bad ? "MISMATCH" : "ok", bad);
  return 0;
}
