// Start-up cost of the engine in a fresh process (what every ugrep_gpu run
// pays once): device discovery, table build + upload, the first stream feed
// and the first whole-buffer records scan, each timed separately.
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>
#include "ugpu.h"

static double ms(std::chrono::steady_clock::time_point a)
{
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
}

int main()
{
  auto t = std::chrono::steady_clock::now();
  int n = 0;
  int rc = ugpu_device_count(&n);
  std::printf("device_count rc=%d n=%d %.1f ms\n", rc, n, ms(t));
  t = std::chrono::steady_clock::now();
  rc = ugpu_select_device(0);
  std::printf("select_device rc=%d %.1f ms\n", rc, ms(t));
  const char* rx = "foo|bar|baz";
  uint32_t* opc = NULL;
  uint32_t nop = 0;
  t = std::chrono::steady_clock::now();
  rc = ugpu_compile(rx, std::strlen(rx), 0, &opc, &nop);
  std::printf("compile rc=%d %.1f ms\n", rc, ms(t));
  ugpu_dfa* d = NULL;
  t = std::chrono::steady_clock::now();
  rc = ugpu_dfa_create(opc, nop, 0, &d);
  std::printf("dfa_create rc=%d %.1f ms\n", rc, ms(t));
  std::vector<uint8_t> buf(1 << 16);
  for (size_t i = 0; i < buf.size(); ++i) buf[i] = "xyfoo bar\n"[i % 10];
  for (int k = 0; k < 3; ++k) {
    ugpu_stream* st = NULL;
    ugpu_result* res = NULL;
    t = std::chrono::steady_clock::now();
    rc = ugpu_stream_create(d, 0, &st);
    const double c = ms(t);
    t = std::chrono::steady_clock::now();
    rc |= ugpu_stream_feed(st, buf.data(), buf.size(), 1, UGPU_MODE_OFFSETS, &res);
    std::printf("stream %d: create %.2f ms feed rc=%d %.2f ms count=%llu\n", k, c, rc, ms(t),
                (unsigned long long)(res ? res->count : 0));
    ugpu_stream_destroy(st);
    ugpu_records* r = NULL;
    t = std::chrono::steady_clock::now();
    rc = ugpu_find_records(d, buf.data(), buf.size(), 0, &r);
    uint64_t cnt = 0, dg = 0, dc = 0;
    rc |= ugpu_records_drain(r, &cnt, &dg, &dc);
    std::printf("records %d: rc=%d %.2f ms count=%llu\n", k, rc, ms(t), (unsigned long long)cnt);
    ugpu_records_free(r);
  }
  return 0;
}
