// VALU issue-rate microbenchmark on gfx950: cycles per wave64 instruction per SIMD for the ops the CRC
// walk uses, with WPS waves per SIMD (1024-thread workgroup = 4 waves/SIMD per 256 threads... grid sized
// to one workgroup per CU). Cycles from s_memtime around the loop (shader clock).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int OP>
__device__ __forceinline__ void body(uint32_t (&r)[8], uint32_t s) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if constexpr (OP == 0) r[i] = __builtin_amdgcn_perm(r[i], s, 0x0C060104u);
    else if constexpr (OP == 1) r[i] = r[i] ^ (s + i);
    else if constexpr (OP == 2) r[i] = __builtin_amdgcn_bitop3_b32(r[i], s, r[(i + 1) & 7], 0x96);
    else if constexpr (OP == 3) r[i] = (uint32_t)__builtin_amdgcn_update_dpp((int)r[i], (int)r[(i + 3) & 7], 0x118, 0xF, 0xC, false);
    else if constexpr (OP == 4) { if (i & 1) { auto q = __builtin_amdgcn_permlane16_swap(r[i - 1], r[i], false, false); r[i - 1] = q[0]; r[i] = q[1]; } }
    else if constexpr (OP == 5) r[i] = __float_as_uint(__uint_as_float(r[i]) * 1.0001f + 0.5f);
    else if constexpr (OP == 6) { uint32_t x; asm volatile("v_add_u32 %0, %1, %2" : "=v"(x) : "v"(r[i]), "v"(s)); r[i] = x; }
  }
}

template <int OP>
__global__ void __launch_bounds__(1024) k(uint32_t* out, int iters, unsigned long long* cyc) {
  uint32_t r[8];
  for (int i = 0; i < 8; ++i) r[i] = threadIdx.x * 7 + i;
  uint32_t s = blockIdx.x;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) body<OP>(r, s + it);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t a = 0;
  for (int i = 0; i < 8; ++i) a ^= r[i];
  if (a == 0x1234567u) out[0] = a;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int OP>
static void run(const char* name, int threads, uint32_t* out, unsigned long long* cyc, int ncu) {
  const int iters = 4096;
  k<OP><<<ncu, threads>>>(out, iters, cyc);
  (void)hipDeviceSynchronize();
  unsigned long long c;
  (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  const int wps = threads / 256;  // waves per SIMD (4 SIMDs per CU)
  const double instrs = (double)iters * 8 * (OP == 4 ? 0.5 : 1.0);
  printf("%-14s waves/SIMD=%d : %.2f cycles per wave-instruction per SIMD\n", name, wps, (double)c / (instrs * wps));
}

int main() {
  uint32_t* out;
  unsigned long long* cyc;
  CK(hipMalloc(&out, 64));
  CK(hipMalloc(&cyc, 8));
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  for (int th : {256, 512, 1024}) {
    run<0>("v_perm_b32", th, out, cyc, ncu);
    run<1>("v_xor/add", th, out, cyc, ncu);
    run<2>("v_bitop3_b32", th, out, cyc, ncu);
    run<3>("v_mov_dpp", th, out, cyc, ncu);
    run<4>("permlane16swp", th, out, cyc, ncu);
    run<5>("v_fma_f32", th, out, cyc, ncu);
    run<6>("v_add_u32", th, out, cyc, ncu);
  }
  return 0;
}
