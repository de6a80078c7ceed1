// ds_read_u8_d16 / ds_read_u8_d16_hi into one VGPR, both in flight (probe)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k(uint32_t* out, int mode)
{
  __shared__ uint8_t t[256];
  t[threadIdx.x] = (uint8_t)(threadIdx.x * 7 + 1);
  __syncthreads();
  const uint32_t a0 = threadIdx.x & 255, a1 = (threadIdx.x + 3) & 255;
  const uint32_t base = (uint32_t)(uintptr_t)t;
  uint32_t r;
  if (mode == 0) {
    asm volatile("ds_read_u8_d16 %0, %1\n\tds_read_u8_d16_hi %0, %2\n\ts_waitcnt lgkmcnt(0)" : "=&v"(r) : "v"(a0 + base), "v"(a1 + base) : "memory");
  } else {
    uint32_t x = 0;
    asm volatile("ds_read_u8_d16 %0, %1\n\ts_waitcnt lgkmcnt(0)\n\tds_read_u8_d16_hi %0, %2\n\ts_waitcnt lgkmcnt(0)" : "+v"(x) : "v"(a0 + base), "v"(a1 + base) : "memory");
    r = x;
  }
  out[threadIdx.x] = r;
  out[256 + threadIdx.x] = base;
}
int main()
{
  uint32_t* d;
  hipMalloc(&d, 4096);
  uint32_t h[512];
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, d, mode);
    hipMemcpy(h, d, 2048, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) {
      const uint32_t want = (uint8_t)(i * 7 + 1) | ((uint32_t)(uint8_t)(((i + 3) & 255) * 7 + 1) << 16);
      if (h[i] != want) { if (bad < 4) printf("mode %d lane %d got %08x want %08x\n", mode, i, h[i], want); ++bad; }
    }
    printf("mode %d: %d bad, lds base %u\n", mode, bad, h[256]);
  }
  return 0;
}
