// valu_rate3.hip -- probe (round 6, second pass; valu_rate2.hip was the first): issue cost per wave-instruction per SIMD
// of the integer VALU forms a U-mode rewrite could use instead of the
// half-rate v_perm / v_alignbit / v_lshl_or (valu_rate.hip measured those):
// SDWA byte inserts and byte selects, v_bitop3 with three VGPR sources, the
// single-VGPR shifts and masks, packed 16-bit ops.  Each lane runs 8
// independent chains of one instruction (inline asm, so the compiler neither
// folds nor splits it); 8 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHAINS 8
template <int K>
__device__ __forceinline__ uint32_t op(uint32_t a, uint32_t b)
{
  uint32_t r = a;
  if constexpr (K == 0) asm volatile("v_lshlrev_b32 %0, 2, %1" : "=v"(r) : "v"(a));
  if constexpr (K == 1) asm volatile("v_lshlrev_b32 %0, 7, %1" : "=v"(r) : "v"(a));
  if constexpr (K == 2) asm volatile("v_lshrrev_b32 %0, 2, %1" : "=v"(r) : "v"(a));
  if constexpr (K == 3) asm volatile("v_lshrrev_b32 %0, 7, %1" : "=v"(r) : "v"(a));
  if constexpr (K == 4) asm volatile("v_and_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  if constexpr (K == 5) asm volatile("v_or_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  if constexpr (K == 6) asm volatile("v_and_b32 %0, 63, %1" : "=v"(r) : "v"(a));
  if constexpr (K == 7) asm volatile("v_and_b32 %0, %1, %2" : "=v"(r) : "s"(0xfcfcfcfcu), "v"(a));
  if constexpr (K == 8) asm volatile("v_and_b32 %0, %1, %2" : "=v"(r) : "s"(0xfcfcfcfcu), "v"(b));
  if constexpr (K == 9) asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "s"(0x01010101u), "v"(a));
  if constexpr (K == 10) asm volatile("v_xor_b32 %0, %1, %2" : "=v"(r) : "s"(0x01010101u), "v"(a));
  if constexpr (K == 11) asm volatile("v_lshlrev_b32 %0, %1, %2" : "=v"(r) : "v"(b), "v"(a));
  if constexpr (K == 12) asm volatile("v_lshrrev_b32 %0, %1, %2" : "=v"(r) : "v"(b), "v"(a));
  if constexpr (K == 13) asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xec" : "=v"(r) : "v"(a), "v"(b), "v"(a + 0u));
  if constexpr (K == 14) asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(b ^ 5u));
  if constexpr (K == 15) asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(a ^ 0x0c0c0c0cu));
  if constexpr (K == 16) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(a));
  if constexpr (K == 17) asm volatile("v_add_u32_dpp %0, %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(a), "v"(b));
  if constexpr (K == 18) asm volatile("v_lshlrev_b16 %0, 2, %1" : "=v"(r) : "v"(a));
  if constexpr (K == 19) asm volatile("v_not_b32 %0, %1" : "=v"(r) : "v"(a));
  if constexpr (K == 20) asm volatile("v_sub_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  if constexpr (K == 21) asm volatile("v_lshrrev_b32 %0, 8, %1\n v_and_b32 %0, %2, %0" : "=&v"(r) : "v"(a), "s"(0xffffu));
  if constexpr (K == 22) asm volatile("v_and_b32 %0, %2, %1\n v_lshrrev_b32 %0, 8, %0" : "=&v"(r) : "v"(a), "s"(0xffffu));
  if constexpr (K == 23) asm volatile("v_lshlrev_b32 %0, 8, %1\n v_or_b32 %0, %0, %2" : "=&v"(r) : "v"(a), "v"(b));
  if constexpr (K == 24) asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xec" : "=v"(r) : "v"(a), "v"(b), "v"(0x00ff00ffu));
  if constexpr (K == 25) asm volatile("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(0x5555555555555555ull));
  if constexpr (K == 26) asm volatile("v_add_co_u32 %0, vcc, %1, %2\n v_addc_co_u32 %0, vcc, %0, %2, vcc" : "=&v"(r) : "v"(a), "v"(b) : "vcc");
  if constexpr (K == 27) asm volatile("v_max_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

template <int K>
__global__ __launch_bounds__(256) void probe(uint32_t* out, int iters, unsigned long long* cyc)
{
  uint32_t v[CHAINS];
  for (int c = 0; c < CHAINS; ++c) v[c] = threadIdx.x * 7 + c + blockIdx.x;
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
void run(const char* name, int waves_per_simd, int ninst = 1)
{
  uint32_t* out;
  unsigned long long* cyc;
  hipMalloc(&out, 4096);
  hipMalloc(&cyc, 8);
  const int cus = 256, iters = 4096;
  const int blocks = cus * waves_per_simd;
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
  const double inst = (double)iters * 8 * CHAINS * ninst;
  const double ns_per = ms * 1e6 / (inst * waves_per_simd);
  printf("%-22s waves/SIMD %d: %.3f ns per wave-instr per SIMD (x 2.1 GHz = %.2f cyc)\n", name, waves_per_simd, ns_per,
         ns_per * 2.1);
  hipFree(out);
  hipFree(cyc);
}

int main()
{
  const int w = 8;
  run<0>("v_lshlrev 2", w);
  run<1>("v_lshlrev 7", w);
  run<2>("v_lshrrev 2", w);
  run<3>("v_lshrrev 7", w);
  run<4>("v_and vv", w);
  run<5>("v_or vv", w);
  run<6>("v_and inline", w);
  run<7>("v_and sv (self)", w);
  run<8>("v_and sv (other)", w);
  run<9>("v_add sv", w);
  run<10>("v_xor sv", w);
  run<11>("v_lshlrev vv", w);
  run<12>("v_lshrrev vv", w);
  run<13>("bitop3 vvv(a,b,a)", w);
  run<14>("bitop3 vvv distinct", w);
  run<15>("v_perm vvv", w);
  run<16>("v_mov dpp", w);
  run<17>("v_add dpp", w);
  run<18>("v_lshlrev_b16", w);
  run<19>("v_not", w);
  run<20>("v_sub vv", w);
  run<21>("lshr;and(s) pair", w, 2);
  run<22>("and(s);lshr pair", w, 2);
  run<23>("lshl;or pair", w, 2);
  run<24>("bitop3 vv+vconst", w);
  run<25>("v_cndmask s", w);
  run<26>("add_co;addc pair", w, 2);
  run<27>("v_max_u32", w);
  return 0;
}
