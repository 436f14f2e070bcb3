// Microbenchmark: back-to-back launch cost of (nearly) empty kernels of different shapes, with and
// without a large static LDS allocation.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int T>
__global__ void __launch_bounds__(T) k_empty(uint32_t* out, int flag) {
  if (flag == 12345) out[threadIdx.x] = blockIdx.x;
}
template <int T>
__global__ void __launch_bounds__(T) k_lds(uint32_t* out, int flag) {
  __shared__ uint32_t big[152 * 256];
  big[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (flag == 12345) out[threadIdx.x] = big[(threadIdx.x + 1) % T];
}

template <typename F>
float timeit(F f) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 10; ++i) f();
  float best = 1e9;
  for (int r = 0; r < 3; ++r) {
    (void)hipEventRecord(a);
    for (int i = 0; i < 200; ++i) f();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    if (ms / 200 < best) best = ms / 200;
  }
  return best * 1000;
}

int main() {
  uint32_t* out;
  CK(hipMalloc(&out, 1 << 20));
  printf("empty 1x64        %6.2f us\n", timeit([&] { k_empty<64><<<1, 64>>>(out, 0); }));
  printf("empty 256x1024    %6.2f us\n", timeit([&] { k_empty<1024><<<256, 1024>>>(out, 0); }));
  printf("empty 1024x256    %6.2f us\n", timeit([&] { k_empty<256><<<1024, 256>>>(out, 0); }));
  printf("empty 4096x64     %6.2f us\n", timeit([&] { k_empty<64><<<4096, 64>>>(out, 0); }));
  printf("lds152 1x1024     %6.2f us\n", timeit([&] { k_lds<1024><<<1, 1024>>>(out, 0); }));
  printf("lds152 256x1024   %6.2f us\n", timeit([&] { k_lds<1024><<<256, 1024>>>(out, 0); }));
  printf("lds152 256x512    %6.2f us\n", timeit([&] { k_lds<512><<<256, 512>>>(out, 0); }));
  CK(hipGetLastError());
  return 0;
}
