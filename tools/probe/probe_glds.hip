// Does global_load_lds_dwordx4 (LDS-DMA, 16 B per lane) accept an unaligned per-lane global source on gfx950?
// Each lane loads 16 B from src + 17 * lane + shift into LDS (wave-uniform base + 16 * lane); the kernel copies LDS
// out and the host compares with the bytes at those addresses.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>

__global__ void k(const uint8_t* src, uint8_t* out, int shift) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[64 * 16];
  const int lane = threadIdx.x;
  __builtin_amdgcn_global_load_lds((const void*)(src + 17 * lane + shift), (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_s_barrier();
  for (int i = 0; i < 16; ++i) out[16 * lane + i] = lds[16 * lane + i];
}

int main() {
  uint8_t h[2048];
  for (int i = 0; i < 2048; ++i) h[i] = (uint8_t)(i * 7 + 3);
  uint8_t *d, *o;
  if (hipMalloc(&d, 2048) || hipMalloc(&o, 1024)) return 1;
  if (hipMemcpy(d, h, 2048, hipMemcpyHostToDevice)) return 1;
  int bad_total = 0;
  for (int shift = 0; shift < 16; ++shift) {
    k<<<1, 64>>>(d, o, shift);
    uint8_t r[1024];
    if (hipMemcpy(r, o, 1024, hipMemcpyDeviceToHost)) return 1;
    int bad = 0;
    for (int l = 0; l < 64; ++l)
      if (memcmp(r + 16 * l, h + 17 * l + shift, 16)) ++bad;
    printf("shift %2d: %d of 64 lanes wrong\n", shift, bad);
    bad_total += bad;
  }
  printf("glds unaligned: %s\n", bad_total ? "NOT exact" : "exact");
  return 0;
}
