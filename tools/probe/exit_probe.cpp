// exit_probe.cpp -- the drop-in adapter's stream calls without ugrep: compile
// a pattern, warm the device, feed a file in 2 MiB chunks as ugpu_stream_feed
// (OFFSETS), free the results, the stream and the table, exit.  Used to tell
// whether ugrep_gpu's rare exit abort ("corrupted double-linked list") comes
// from the engine and the HIP runtime or from ugrep and the adapter.
//   exit_probe FILE PATTERN [cleanup]
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ugpu.h"

int main(int argc, char** argv)
{
  if (argc < 3) return 2;
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<unsigned char> data;
  unsigned char buf[1 << 16];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) data.insert(data.end(), buf, buf + n);
  std::fclose(f);
  uint32_t* opc = nullptr;
  uint32_t nop = 0;
  if (ugpu_compile(argv[2], std::strlen(argv[2]), UGPU_RX_REFLEX, &opc, &nop) != UGPU_OK) return 3;
  if (ugpu_warmup(0) != UGPU_OK) return 4;
  ugpu_dfa* d = nullptr;
  if (ugpu_dfa_create(opc, nop, 0, &d) != UGPU_OK) return 5;
  ugpu_opc_free(opc);
  uint64_t total = 0;
  for (int rep = 0; rep < 2; ++rep) {
    ugpu_stream* st = nullptr;
    if (ugpu_stream_create(d, 0, &st) != UGPU_OK) return 6;
    const size_t chunk = 2u << 20;
    for (size_t off = 0; off < data.size(); off += chunk) {
      const size_t len = data.size() - off < chunk ? data.size() - off : chunk;
      const int fin = off + len >= data.size() ? 1 : 0;
      ugpu_result* r = nullptr;
      if (ugpu_stream_feed(st, data.data() + off, len, fin, UGPU_MODE_OFFSETS, &r) != UGPU_OK) return 7;
      for (uint64_t i = 0; i < r->count; ++i) total += r->start[i] + r->len[i];
      ugpu_result_free(r);
    }
    ugpu_stream_destroy(st);
  }
  ugpu_dfa_destroy(d);
  std::printf("%llu\n", (unsigned long long)total);
  return 0;
}
