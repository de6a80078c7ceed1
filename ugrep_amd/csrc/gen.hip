// gen.hip -- device generator of the synthetic corpora of SURVEY.md §8(d).
//
// The corpus is a sequence of independent 64-byte cells; cell c is a pure
// function of (seed, c), so every GPU generates any slice of one logical
// stream in parallel (one thread per cell).  The byte-level specification is
// documented with the kinds in include/ugpu.h; tests check it against the host
// restatement in oracle/gen.h.
#include "scan_kernels.hpp"

namespace ugpu {

namespace {

constexpr int kCell = 64;

__device__ __forceinline__ uint64_t sm64(uint64_t& s)
{
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ int put_utf8(uint8_t* out, int pos, uint32_t cp)
{
  if (cp < 0x80) {
    if (pos + 1 > kCell) return 0;
    out[pos] = (uint8_t)cp;
    return 1;
  }
  if (cp < 0x800) {
    if (pos + 2 > kCell) return 0;
    out[pos] = (uint8_t)(0xC0 | (cp >> 6));
    out[pos + 1] = (uint8_t)(0x80 | (cp & 0x3F));
    return 2;
  }
  if (pos + 3 > kCell) return 0;
  out[pos] = (uint8_t)(0xE0 | (cp >> 12));
  out[pos + 1] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F));
  out[pos + 2] = (uint8_t)(0x80 | (cp & 0x3F));
  return 3;
}

__device__ __forceinline__ uint8_t ident_char(uint32_t sl, bool first)
{
  // [A-Z][a-z]_ then (rest only) [0-9]
  uint32_t k = first ? sl % 53 : sl % 63;
  if (k < 26) return (uint8_t)('A' + k);
  if (k < 52) return (uint8_t)('a' + k - 26);
  if (k == 52) return '_';
  return (uint8_t)('0' + k - 53);
}

__device__ void cell_bytes(int kind, uint64_t seed, uint64_t cell, uint8_t* out)
{
  const char planted[] = "acdeghijklmnopqrstuvwxyz";
  const char ops[] = "(){};,=+-*/<>.";
  const char punct[] = ".,;:!?";
  uint64_t s = seed ^ (cell * 0xD1B54A32D192ED03ull);
  const uint64_t x = sm64(s);
  int pos = 0;
  if (kind == 1 || kind == 2) {
    while (pos < kCell) {
      uint64_t r = sm64(s);
      int wl = 1 + (int)(r % 10);
      uint64_t r2 = sm64(s);
      for (int i = 0; i < wl && pos < kCell; ++i) {
        uint32_t sl = (uint32_t)((r2 >> (6 * i)) & 63);
        out[pos++] = kind == 1 ? (uint8_t)('a' + sl % 26) : (uint8_t)planted[sl % 24];
      }
      if (pos < kCell) out[pos++] = ' ';
    }
    if (kind == 2 && ((x >> 1) & 63) == 0) {
      uint32_t off = (uint32_t)((x >> 8) % 61);
      uint32_t wsel = (uint32_t)((x >> 16) % 3);
      out[off] = wsel == 0 ? 'f' : 'b';
      out[off + 1] = wsel == 0 ? 'o' : 'a';
      out[off + 2] = wsel == 0 ? 'o' : (wsel == 1 ? 'r' : 'z');
    }
    if (x & 1) out[kCell - 1] = '\n';
    return;
  }
  if (kind == 3) {
    while (pos < kCell) {
      uint64_t r = sm64(s);
      uint32_t t = (uint32_t)(r % 100);
      if (t < 55) {
        int len = 1 + (int)((r >> 8) % 16);
        uint64_t r2 = sm64(s);
        uint64_t r3 = sm64(s);
        for (int i = 0; i < len && pos < kCell; ++i) {
          uint32_t sl = (uint32_t)((i < 10 ? (r2 >> (6 * i)) : (r3 >> (6 * (i - 10)))) & 63);
          out[pos++] = ident_char(sl, i == 0);
        }
      } else if (t < 65) {
        int len = 1 + (int)((r >> 8) % 6);
        uint64_t r2 = sm64(s);
        for (int i = 0; i < len && pos < kCell; ++i) out[pos++] = (uint8_t)('0' + ((r2 >> (6 * i)) & 63) % 10);
      } else if (t < 90) {
        out[pos++] = (uint8_t)ops[(r >> 8) % 14];
      } else {
        out[pos++] = ' ';
      }
      if (t < 65 && pos < kCell && ((r >> 16) & 1)) out[pos++] = ' ';
    }
    if (x & 1) out[kCell - 1] = '\n';
    return;
  }
  // kind 4: UTF-8 words
  while (pos < kCell) {
    uint64_t r = sm64(s);
    uint32_t t = (uint32_t)(r % 100);
    bool stop = false;
    if (t < 90) {
      int len = 1 + (int)((r >> 8) % 8);
      uint64_t r2 = sm64(s);
      for (int i = 0; i < len; ++i) {
        uint32_t sl = (uint32_t)((r2 >> (7 * i)) & 127);
        uint32_t cp;
        if (t < 40) {
          cp = (sl & 64) ? 'A' + sl % 26 : 'a' + sl % 26;
        } else if (t < 55) {
          cp = 0xC0 + (sl & 63);
          if (cp == 0xD7 || cp == 0xF7) cp = 0xE9;
        } else if (t < 70) {
          cp = 0x3B1 + sl % 25;
        } else if (t < 80) {
          cp = 0x430 + (sl & 31);
        } else {
          cp = 0x4E00 + ((uint32_t)((r2 >> (7 * i)) & 0xFFFF) % 0x5000);
        }
        int n = put_utf8(out, pos, cp);
        if (n == 0) break;
        pos += n;
      }
    } else if (t < 95) {
      if ((r >> 8) & 1) {
        int n = put_utf8(out, pos, 0x20AC);
        if (n == 0)
          stop = true;
        else
          pos += n;
      } else {
        out[pos++] = (uint8_t)punct[(r >> 9) % 6];
      }
    }
    if (stop) break;
    if (pos < kCell) out[pos++] = ' ';
  }
  while (pos < kCell) out[pos++] = ' ';
  if ((x & 1) && out[kCell - 1] < 0x80) out[kCell - 1] = '\n';
}

__global__ void gen_kernel(int kind, uint64_t seed, uint64_t off, uint8_t* dbuf, uint64_t len, uint64_t c0,
                           uint64_t ncell)
{
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ncell) return;
  const uint64_t cell = c0 + i;
  uint8_t b[kCell];
  cell_bytes(kind, seed, cell, b);
  const uint64_t cs = cell * kCell;
  const uint64_t end = off + len;
  const uint64_t a = cs < off ? off : cs;
  const uint64_t z = cs + kCell > end ? end : cs + kCell;
  uint8_t* dst = dbuf + (a - off);
  if (a == cs && z == cs + kCell && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    uint4* d = reinterpret_cast<uint4*>(dst);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint4 v;
      v.x = b[16 * k] | (b[16 * k + 1] << 8) | (b[16 * k + 2] << 16) | ((uint32_t)b[16 * k + 3] << 24);
      v.y = b[16 * k + 4] | (b[16 * k + 5] << 8) | (b[16 * k + 6] << 16) | ((uint32_t)b[16 * k + 7] << 24);
      v.z = b[16 * k + 8] | (b[16 * k + 9] << 8) | (b[16 * k + 10] << 16) | ((uint32_t)b[16 * k + 11] << 24);
      v.w = b[16 * k + 12] | (b[16 * k + 13] << 8) | (b[16 * k + 14] << 16) | ((uint32_t)b[16 * k + 15] << 24);
      d[k] = v;
    }
  } else {
    for (uint64_t p = a; p < z; ++p) dbuf[p - off] = b[p - cs];
  }
}

}  // namespace

hipError_t launch_gen(int kind, uint64_t seed, uint64_t off, uint8_t* dbuf, uint64_t len, hipStream_t stream)
{
  if (len == 0) return hipSuccess;
  const uint64_t c0 = off / kCell;
  const uint64_t c1 = (off + len + kCell - 1) / kCell;
  const uint64_t n = c1 - c0;
  const uint64_t per = 256ull * 65535ull * 64ull;  // stay under the grid-x limit per launch
  for (uint64_t s = 0; s < n; s += per) {
    const uint64_t m = n - s < per ? n - s : per;
    const uint64_t blocks = (m + 255) / 256;
    hipLaunchKernelGGL(gen_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, kind, seed, off, dbuf, len, c0 + s, m);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace ugpu
