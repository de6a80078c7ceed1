// exit_probe_dl.cpp -- exit_probe.cpp's calls through a dlopen()ed
// libugrep_amd.so (RTLD_NOW | RTLD_LOCAL, never closed), the way the drop-in
// adapter loads the device half (integration/reflex_gpu_matcher.h GpuEngine).
//   exit_probe_dl LIBDIR FILE PATTERN
#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ugpu.h"

template <class F>
static F sym(void* h, const char* n)
{
  return reinterpret_cast<F>(dlsym(h, n));
}

int main(int argc, char** argv)
{
  if (argc < 4) return 2;
  FILE* f = std::fopen(argv[2], "rb");
  if (!f) return 2;
  std::vector<unsigned char> data;
  unsigned char buf[1 << 16];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) data.insert(data.end(), buf, buf + n);
  std::fclose(f);
  uint32_t* opc = nullptr;
  uint32_t nop = 0;
  if (ugpu_compile(argv[3], std::strlen(argv[3]), UGPU_RX_REFLEX, &opc, &nop) != UGPU_OK) return 3;
  void* h = dlopen((std::string(argv[1]) + "/libugrep_amd.so").c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!h) return 8;
  auto warmup = sym<decltype(&ugpu_warmup)>(h, "ugpu_warmup");
  auto dfa_create = sym<decltype(&ugpu_dfa_create)>(h, "ugpu_dfa_create");
  auto dfa_destroy = sym<decltype(&ugpu_dfa_destroy)>(h, "ugpu_dfa_destroy");
  auto stream_create = sym<decltype(&ugpu_stream_create)>(h, "ugpu_stream_create");
  auto stream_feed = sym<decltype(&ugpu_stream_feed)>(h, "ugpu_stream_feed");
  auto stream_destroy = sym<decltype(&ugpu_stream_destroy)>(h, "ugpu_stream_destroy");
  auto result_free = sym<decltype(&ugpu_result_free)>(h, "ugpu_result_free");
  if (warmup(0) != UGPU_OK) return 4;
  ugpu_dfa* d = nullptr;
  if (dfa_create(opc, nop, 0, &d) != UGPU_OK) return 5;
  ugpu_opc_free(opc);
  uint64_t total = 0;
  ugpu_stream* st = nullptr;
  if (stream_create(d, 0, &st) != UGPU_OK) return 6;
  const size_t chunk = 2u << 20;
  for (size_t off = 0; off < data.size(); off += chunk) {
    const size_t len = data.size() - off < chunk ? data.size() - off : chunk;
    ugpu_result* r = nullptr;
    if (stream_feed(st, data.data() + off, len, off + len >= data.size() ? 1 : 0, UGPU_MODE_OFFSETS, &r) != UGPU_OK)
      return 7;
    for (uint64_t i = 0; i < r->count; ++i) total += r->start[i] + r->len[i];
    result_free(r);
  }
  stream_destroy(st);
  if (!(argc > 4 && std::strcmp(argv[4], "keep") == 0)) dfa_destroy(d);
  std::printf("%llu\n", (unsigned long long)total);
  return 0;
}
