// Write rate of the OFFSETS record stores by store shape (calibration probe).
// Each one-wave block writes its own contiguous run of records, in rounds of
// `per` records, to two arrays as the expansion does: starts (u64) and lengths
// (u32), 12 bytes a record, 1e9 records.
//   shape 0: 8 B / 4 B per lane (the expansion's stores today)
//   shape 1: 16 B per lane for both arrays (2 starts, 4 lengths a lane)
//   shape 2: shape 1 but rounds not aligned to 4 records (head/tail lanes narrow)
//   shape 3: a plain linear 16-B-per-lane fill of the same 12 GB
//   shape 4: shape 0 with non-temporal stores
// hipcc --offload-arch=gfx950 -O3 store_shape.hip -o store_shape
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); exit(1); } } while (0)

template <int SHAPE>
__global__ __launch_bounds__(64) void k(uint64_t* st, uint32_t* ln, uint64_t nrec, uint64_t per_blk, uint32_t per)
{
  const uint32_t lane = threadIdx.x;
  const uint64_t b0 = (uint64_t)blockIdx.x * per_blk;
  if (b0 >= nrec) return;
  const uint64_t b1 = b0 + per_blk < nrec ? b0 + per_blk : nrec;
  if constexpr (SHAPE == 3) {
    // 12 bytes a record as plain 16-B lanes over the block's share of both arrays
    uint4* s4 = reinterpret_cast<uint4*>(st + b0);
    for (uint64_t i = lane; i < (b1 - b0) / 2; i += 64) s4[i] = make_uint4(i, 0, i, 0);
    uint4* l4 = reinterpret_cast<uint4*>(ln + b0);
    for (uint64_t i = lane; i < (b1 - b0) / 4; i += 64) l4[i] = make_uint4(i, i, i, i);
    return;
  }
  for (uint64_t r = b0; r < b1; r += per) {
    const uint32_t R = (uint32_t)(b1 - r < per ? b1 - r : per);
    if constexpr (SHAPE == 0) {
      for (uint32_t t = lane; t < R; t += 64) st[r + t] = r + t;
      for (uint32_t t = lane; t < R; t += 64) ln[r + t] = (uint32_t)t;
    } else if constexpr (SHAPE == 4) {
      // shape 0 with non-temporal stores
      for (uint32_t t = lane; t < R; t += 64) __builtin_nontemporal_store((uint64_t)(r + t), &st[r + t]);
      for (uint32_t t = lane; t < R; t += 64) __builtin_nontemporal_store((uint32_t)t, &ln[r + t]);
    } else {
      // head records up to 4-alignment of r, then 16-B lanes, then the tail
      const uint32_t h = SHAPE == 1 ? 0u : (uint32_t)((4 - (r & 3)) & 3);
      const uint32_t hh = h < R ? h : R;
      if (lane < hh) {
        st[r + lane] = r + lane;
        ln[r + lane] = lane;
      }
      const uint64_t a = r + hh;
      const uint32_t body = (R - hh) & ~3u;
      uint4* s4 = reinterpret_cast<uint4*>(st + a);
      for (uint32_t t = lane; t < body / 2; t += 64) s4[t] = make_uint4((uint32_t)(a + 2 * t), 0, (uint32_t)(a + 2 * t + 1), 0);
      uint4* l4 = reinterpret_cast<uint4*>(ln + a);
      for (uint32_t t = lane; t < body / 4; t += 64) l4[t] = make_uint4(t, t, t, t);
      const uint32_t tl = R - hh - body;
      if (lane < tl) {
        st[a + body + lane] = a + body + lane;
        ln[a + body + lane] = lane;
      }
    }
  }
}

int main(int argc, char** argv)
{
  const uint64_t nrec = 1000000000ull;
  const uint32_t nblk = argc > 1 ? atoi(argv[1]) : 65536;
  uint64_t* st;
  uint32_t* ln;
  CK(hipMalloc(&st, nrec * 8 + 64));
  CK(hipMalloc(&ln, nrec * 4 + 64));
  const uint64_t per_blk = ((nrec + nblk - 1) / nblk + 3) & ~3ull;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int shape = 0; shape < 5; ++shape) {
    for (uint32_t per : {476u, 475u}) {
      if ((shape == 1 && per & 3) || (shape >= 3 && per != 476u)) continue;
      float best = 1e9f;
      for (int rep = 0; rep < 6; ++rep) {
        CK(hipEventRecord(a));
        switch (shape) {
          case 0: hipLaunchKernelGGL(k<0>, dim3(nblk), dim3(64), 0, 0, st, ln, nrec, per_blk, per); break;
          case 1: hipLaunchKernelGGL(k<1>, dim3(nblk), dim3(64), 0, 0, st, ln, nrec, per_blk, per); break;
          case 2: hipLaunchKernelGGL(k<2>, dim3(nblk), dim3(64), 0, 0, st, ln, nrec, per_blk, per); break;
          case 3: hipLaunchKernelGGL(k<3>, dim3(nblk), dim3(64), 0, 0, st, ln, nrec, per_blk, per); break;
          default: hipLaunchKernelGGL(k<4>, dim3(nblk), dim3(64), 0, 0, st, ln, nrec, per_blk, per); break;
        }
        CK(hipGetLastError());
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (rep && ms < best) best = ms;
      }
      printf("shape %d per %u blocks %u: %.3f ms = %.2f TB/s\n", shape, per, nblk, best, nrec * 12.0 / best / 1e9);
    }
  }
  return 0;
}
