// Read-bandwidth ceiling probe on MI355X: which load form streams HBM fastest?
//   global_load_dwordx4 (plain / nt), buffer_load_dwordx4 (aux 0 / nt), loads in flight per lane,
//   LDS-DMA (global_load_lds_dwordx4) into a per-wave LDS ring.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <algorithm>
#include <hip/hip_ext.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// persistent grid-stride, each wave reads chunks of 1 KiB * DEPTH per iteration
template <int DEPTH, bool NT>
__global__ void __launch_bounds__(256) k_global(const u32x4* __restrict__ p, size_t n16, uint32_t* out) {
  const size_t lane = threadIdx.x & 63;
  const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  uint32_t acc = 0;
  for (size_t c = wave; c * 64 * DEPTH < n16; c += nw) {
    const u32x4* q = p + c * 64 * DEPTH + lane;
    u32x4 v[DEPTH];
#pragma unroll
    for (int j = 0; j < DEPTH; ++j) v[j] = NT ? __builtin_nontemporal_load(q + 64 * j) : q[64 * j];
#pragma unroll
    for (int j = 0; j < DEPTH; ++j) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int DEPTH, int AUX>
__global__ void __launch_bounds__(256) k_buffer(const uint8_t* __restrict__ p, size_t nbytes, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63;
  const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  const size_t chunk = 1024 * DEPTH;
  uint32_t acc = 0;
  for (size_t c = wave; c * chunk < nbytes; c += nw) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(p + c * chunk), (short)0, (int)chunk, 0x00020000);
    u32x4 v[DEPTH];
#pragma unroll
    for (int j = 0; j < DEPTH; ++j) v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, j * 1024 + lane * 16, 0, AUX);
#pragma unroll
    for (int j = 0; j < DEPTH; ++j) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// double-buffered buffer loads (like k_windows): loads for chunk c+1 issued before consuming chunk c
template <int DEPTH, int AUX, int THREADS>
__global__ void __launch_bounds__(THREADS) k_buffer_db(const uint8_t* __restrict__ p, size_t nbytes, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63;
  const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  const size_t chunk = 1024 * DEPTH;
  const size_t nch = nbytes / chunk;
  uint32_t acc = 0;
  u32x4 a[DEPTH], b[DEPTH];
  size_t c = wave;
  auto ld = [&](u32x4 (&v)[DEPTH], size_t cc) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(p + (cc < nch ? cc : 0) * chunk), (short)0,
                                                                 cc < nch ? (int)chunk : 0, 0x00020000);
#pragma unroll
    for (int j = 0; j < DEPTH; ++j) v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, j * 1024 + lane * 16, 0, AUX);
  };
  ld(a, c);
  while (c < nch) {
    ld(b, c + nw);
#pragma unroll
    for (int j = 0; j < DEPTH; ++j) acc ^= a[j].x ^ a[j].y ^ a[j].z ^ a[j].w;
    if (c + nw >= nch) break;
    ld(a, c + 2 * nw);
#pragma unroll
    for (int j = 0; j < DEPTH; ++j) acc ^= b[j].x ^ b[j].y ^ b[j].z ^ b[j].w;
    c += 2 * nw;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// LDS-DMA stream: each wave owns a ring of RING x 1 KiB slots; waits with counted vmcnt.
template <int RING, int AUX>
__global__ void __launch_bounds__(256) k_glds(const uint8_t* __restrict__ p, size_t nbytes, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint32_t ring[4][RING * 256];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t w = threadIdx.x >> 6;
  const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  const size_t chunk = 1024 * RING;
  uint32_t acc = 0;
  for (size_t c = wave; c * chunk < nbytes; c += nw) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(p + c * chunk), (short)0, (int)chunk, 0x00020000);
#pragma unroll
    for (int j = 0; j < RING; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)&ring[w][j * 256], 16,
                                               lane * 16 + j * 1024, 0, 0, AUX);
    __builtin_amdgcn_s_waitcnt(0x0F70 & ~0x0F00);  // vmcnt(0)
    acc ^= ring[w][lane];
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

// one isolated launch at a time, timed by events carried by the launch itself (start of the first
// wave to end of the last): the single-launch floor of a plain streaming read, to set beside k_windows
template <typename F>
static float single_us(F f) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float v[12];
  for (int rep = 0; rep < 15; ++rep) {
    (void)hipDeviceSynchronize();
    f(rep, a, b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    if (rep >= 3) v[rep - 3] = ms * 1e3f;
  }
  std::sort(v, v + 12);
  return (v[5] + v[6]) / 2;
}

int main(int argc, char** argv) {
  const size_t NB = 256ull << 20;
  const int NBUF = 4;
  uint8_t* buf;
  CK(hipMalloc(&buf, NB * NBUF));
  uint32_t* out;
  CK(hipMalloc(&out, 4096));
  k_fill<<<4096, 256>>>(buf, NB * NBUF);
  CK(hipDeviceSynchronize());
  auto rep = [&](const char* name, float ms) { printf("%-36s %7.1f us  %7.1f GB/s\n", name, ms * 1e3, NB / ms / 1e6); };
  if (argc > 1) {  // buffers rotated as in bench.py's single launches (1 GiB in all, past the MALL)
    for (int g : {256, 512, 1024, 2048, 4096}) {
      char nm[64];
      snprintf(nm, 64, "single buffer d8 nt g%d", g);
      rep(nm, 1e-3f * single_us([&](int i, hipEvent_t a, hipEvent_t b) {
            hipExtLaunchKernelGGL(k_buffer<8, 2>, dim3(g), dim3(256), 0, 0, a, b, 0,
                                  (const uint8_t*)(buf + (i % NBUF) * NB), NB, out); }));
      snprintf(nm, 64, "single buffer d16 nt g%d", g);
      rep(nm, 1e-3f * single_us([&](int i, hipEvent_t a, hipEvent_t b) {
            hipExtLaunchKernelGGL(k_buffer<16, 2>, dim3(g), dim3(256), 0, 0, a, b, 0,
                                  (const uint8_t*)(buf + (i % NBUF) * NB), NB, out); }));
      snprintf(nm, 64, "single global d8 nt g%d", g);
      rep(nm, 1e-3f * single_us([&](int i, hipEvent_t a, hipEvent_t b) {
            hipExtLaunchKernelGGL(k_global<8, true>, dim3(g), dim3(256), 0, 0, a, b, 0,
                                  (const u32x4*)(buf + (i % NBUF) * NB), NB / 16, out); }));
      snprintf(nm, 64, "single same-buffer buffer d8 nt g%d", g);
      rep(nm, 1e-3f * single_us([&](int, hipEvent_t a, hipEvent_t b) {
            hipExtLaunchKernelGGL(k_buffer<8, 2>, dim3(g), dim3(256), 0, 0, a, b, 0, (const uint8_t*)buf, NB, out); }));
    }
    return 0;
  }
  for (int g : {1024, 2048, 4096}) {
    char nm[64];
    snprintf(nm, 64, "global d4 plain g%d", g);
    rep(nm, best_ms([&](int i) { k_global<4, false><<<g, 256>>>((const u32x4*)(buf + (i % NBUF) * NB), NB / 16, out); }, 50));
    snprintf(nm, 64, "global d4 nt g%d", g);
    rep(nm, best_ms([&](int i) { k_global<4, true><<<g, 256>>>((const u32x4*)(buf + (i % NBUF) * NB), NB / 16, out); }, 50));
    snprintf(nm, 64, "global d8 nt g%d", g);
    rep(nm, best_ms([&](int i) { k_global<8, true><<<g, 256>>>((const u32x4*)(buf + (i % NBUF) * NB), NB / 16, out); }, 50));
    snprintf(nm, 64, "buffer d8 aux0 g%d", g);
    rep(nm, best_ms([&](int i) { k_buffer<8, 0><<<g, 256>>>(buf + (i % NBUF) * NB, NB, out); }, 50));
    snprintf(nm, 64, "buffer d8 nt g%d", g);
    rep(nm, best_ms([&](int i) { k_buffer<8, 2><<<g, 256>>>(buf + (i % NBUF) * NB, NB, out); }, 50));
    snprintf(nm, 64, "buffer d16 nt g%d", g);
    rep(nm, best_ms([&](int i) { k_buffer<16, 2><<<g, 256>>>(buf + (i % NBUF) * NB, NB, out); }, 50));
    snprintf(nm, 64, "glds ring8 nt g%d", g);
    rep(nm, best_ms([&](int i) { k_glds<8, 2><<<g, 256>>>(buf + (i % NBUF) * NB, NB, out); }, 50));
    snprintf(nm, 64, "glds ring16 nt g%d", g);
    rep(nm, best_ms([&](int i) { k_glds<16, 2><<<g, 256>>>(buf + (i % NBUF) * NB, NB, out); }, 50));
  }
  rep("buffer_db d8 nt 1024thr g256", best_ms([&](int i) { k_buffer_db<8, 2, 1024><<<256, 1024>>>(buf + (i % NBUF) * NB, NB, out); }, 50));
  rep("buffer_db d8 aux0 1024thr g256", best_ms([&](int i) { k_buffer_db<8, 0, 1024><<<256, 1024>>>(buf + (i % NBUF) * NB, NB, out); }, 50));
  rep("buffer_db d16 nt 1024thr g256", best_ms([&](int i) { k_buffer_db<16, 2, 1024><<<256, 1024>>>(buf + (i % NBUF) * NB, NB, out); }, 50));
  rep("buffer_db d8 nt 256thr g1024", best_ms([&](int i) { k_buffer_db<8, 2, 256><<<1024, 256>>>(buf + (i % NBUF) * NB, NB, out); }, 50));
  rep("buffer_db d8 nt 256thr g2048", best_ms([&](int i) { k_buffer_db<8, 2, 256><<<2048, 256>>>(buf + (i % NBUF) * NB, NB, out); }, 50));
  // the same stream over 1 GiB per launch (launch overhead amortized)
  rep("buffer d8 nt g2048 (1 GiB/launch)/4", best_ms([&](int i) { k_buffer<8, 2><<<2048, 256>>>(buf, NB * 4, out); }, 20) / 4);
  return 0;
}
