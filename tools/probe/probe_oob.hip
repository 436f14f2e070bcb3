// Buffer range-check granularity of raw_buffer_load_b128 on gfx950: which dwords of a 16 B load come back
// when num_records cuts the access (at byte granularity, and with an unaligned base).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void k(const uint8_t* p, uint32_t* out, int nrec, int shift) {
  auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(p + shift), (short)0, nrec, 0x00020000);
  u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, 0, 0, 0);
  if (threadIdx.x == 0) {
    out[0] = v.x;
    out[1] = v.y;
    out[2] = v.z;
    out[3] = v.w;
  }
}

int main() {
  uint8_t h[64];
  for (int i = 0; i < 64; ++i) h[i] = (uint8_t)(0x10 + i);
  uint8_t* d;
  uint32_t* o;
  if (hipMalloc(&d, 64) || hipMalloc(&o, 16)) return 1;
  if (hipMemcpy(d, h, 64, hipMemcpyHostToDevice)) return 1;
  for (int shift : {0, 1, 2}) {
    for (int nrec : {1, 2, 3, 4, 5, 7, 8, 9, 12, 13, 15, 16}) {
      k<<<1, 64>>>(d, o, nrec, shift);
      uint32_t r[4];
      if (hipMemcpy(r, o, 16, hipMemcpyDeviceToHost)) return 1;
      printf("shift %d nrec %2d: %08x %08x %08x %08x\n", shift, nrec, r[0], r[1], r[2], r[3]);
    }
  }
  return 0;
}
