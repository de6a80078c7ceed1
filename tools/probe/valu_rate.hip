// valu_rate.hip -- probe: issue cost of the integer VALU instructions the
// U-mode kernel (xc_kernel.hip xu_kernel) is made of, per SIMD, at 1 and 8
// waves per SIMD.  Each lane runs 8 independent chains of one instruction
// kind; cycles per wave-instruction = SIMD cycles / (waves per SIMD x
// instructions per wave), with cycles from s_memtime inside the kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHAINS 8
template <int K>
__device__ __forceinline__ uint32_t op(uint32_t a, uint32_t b)
{
  if constexpr (K == 0) return __builtin_amdgcn_perm(a, b, 0x05010400u);
  if constexpr (K == 1) return __builtin_amdgcn_alignbit(a, b, 9);
  if constexpr (K == 2) return a & b & 0x70707070u;  // v_bitop3_b32 (constant in an SGPR)
  if constexpr (K == 3) return a + b;
  if constexpr (K == 4) return __builtin_popcount(a) + b;
  if constexpr (K == 5) return __builtin_amdgcn_udot4(a, 0x03020100u, b, false);
  if constexpr (K == 6) return __builtin_amdgcn_update_dpp(b, a, 0x130, 0xf, 0xf, false);
  if constexpr (K == 7) return (a << 3) + b;  // v_lshl_add_u32
  if constexpr (K == 8) return (a << 8) | b;  // v_lshl_or_b32
  if constexpr (K == 9) return a >> 7;        // v_lshrrev_b32 (dependent chain per lane: 8 chains)
  if constexpr (K == 10) return (a | b) | (a >> 3);  // v_or3_b32 (+ shift)
  if constexpr (K == 11) return __builtin_amdgcn_ubfe(a, 8, 16) ^ b;  // v_bfe_u32 (+ xor)
  if constexpr (K == 12) return (a & 0x00ff00ffu) | (b & 0xff00ff00u);  // v_bfi_b32 or bitop3
  if constexpr (K == 13) return a - b;  // v_sub_u32
  if constexpr (K == 14) return a + b + 0x1234567u;  // v_add3_u32
  if constexpr (K == 15) return (a & b) | 0x01010101u;  // v_and_or_b32
  if constexpr (K == 16) { uint32_t r; asm volatile("v_lshl_or_b32 %0, %1, 8, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
  if constexpr (K == 17) { uint32_t r; asm volatile("v_or3_b32 %0, %1, %2, %1" : "=v"(r) : "v"(a), "v"(b)); return r; }
  if constexpr (K == 18) { uint32_t r; asm volatile("v_lshlrev_b32 %0, 3, %1" : "=v"(r) : "v"(a)); return r ^ b; }
  if constexpr (K == 19) { uint32_t r; asm volatile("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(256u), "v"(b)); return r; }
  if constexpr (K == 20) { uint32_t r; asm volatile("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
  return a;
}

template <int K>
__global__ __launch_bounds__(256) void probe(uint32_t* out, int iters, unsigned long long* cyc)
{
  uint32_t v[CHAINS];
  for (int c = 0; c < CHAINS; ++c) v[c] = threadIdx.x * 7 + c + blockIdx.x;
  const uint32_t b = blockIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int c = 0; c < CHAINS; ++c) v[c] = op<K>(v[c], v[(c + 1) % CHAINS]);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t x = 0;
  for (int c = 0; c < CHAINS; ++c) x ^= v[c];
  if (x == 0x12345678u) out[threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int K>
void run(const char* name, int waves_per_simd)
{
  uint32_t* out;
  unsigned long long* cyc;
  hipMalloc(&out, 4096);
  hipMalloc(&cyc, 8);
  const int cus = 256, iters = 4096;
  const int blocks = cus * waves_per_simd;  // 4 waves (256 threads) per block: one per SIMD
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  probe<K><<<blocks, 256>>>(out, 64, cyc);
  hipEventRecord(e0);
  probe<K><<<blocks, 256>>>(out, iters, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long c = 0;
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  // instructions per wave (the body; the xor of the operand is hoisted or counted below)
  const double inst = (double)iters * 8 * CHAINS;
  const double waves_per_simd_d = waves_per_simd;
  // wall-clock cycles at the measured memtime rate of wave 0 are not the SIMD's;
  // report ns per wave-instruction per SIMD and memtime ticks per instruction of one wave
  const double ns_per = ms * 1e6 / (inst * waves_per_simd_d);
  printf("%-10s waves/SIMD %d: %.3f ns per wave-instr per SIMD (x 2.1 GHz = %.2f cyc); wave0 %.2f ticks/instr\n", name,
         waves_per_simd, ns_per, ns_per * 2.1, (double)c / inst);
  hipFree(out);
  hipFree(cyc);
}

int main()
{
  for (int w : {8}) {
    run<0>("v_perm", w);
    run<1>("alignbit", w);
    run<2>("bitop3", w);
    run<3>("add", w);
    run<4>("bcnt", w);
    run<5>("dot4", w);
    run<6>("dpp", w);
    run<7>("lshl_add", w);
    run<8>("lshl_or", w);
    run<9>("lshr", w);
    run<10>("or3+lshr", w);
    run<11>("bfe+xor", w);
    run<12>("bfi", w);
    run<13>("sub", w);
    run<14>("add3", w);
    run<15>("and_or", w);
    run<16>("lshl_or(asm)", w);
    run<17>("or3(asm)", w);
    run<18>("lshl+xor", w);
    run<19>("mad_u24(asm)", w);
    run<20>("mul_u24(asm)", w);
  }
  return 0;
}
