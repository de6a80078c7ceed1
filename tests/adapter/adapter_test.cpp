// adapter_test.cpp -- TEST INFRASTRUCTURE (GPU box): the drop-in adapter
// reflex::GpuMatcher (integration/reflex_gpu_matcher.h) against the reference
// reflex::Matcher, both linked in one binary (the reference libreflex compiled
// from its sources by oracle/Makefile into oracle/_ref/).  The adapter is built
// exactly as ugrep would build it -- GpuMatcher(pattern, Input(), options) --
// and compiles its tables from the Pattern's public operator[](0): this file
// reads no private member.
//
// For every case line "MODE<TAB>REGEX<TAB>INPUT" of the spec file:
//   0. plain loop   : while (m.find()) -> (first, size, accept) sequences equal
//   1. -c loop      : while (m.find()) { ++n; m.skip('\n'); }  (src/ugrep.cpp:10583)
//   2. skip(' ')    : cur_ moved to arbitrary positions between finds
//   3. re-buffer    : new bytes at the same address and size, second loop
//   4. stream       : input() from a std::istream (GPU stream feeds of
//                     UGPU_ADAPTER_CHUNK bytes, set small here), plain loop
//   5. stream -c    : the same with skip('\n') after each hit
//   in every loop lineno(), columno() after each hit and at_end() at the end agree
// Then the slow-pipe case: stdin is a non-blocking pipe (as ugrep sets it,
// src/ugrep.cpp:3956-3966) whose writer stalls after its first line; the first
// match must be reported before the writer continues, as the reference does.
// INPUT as in oracle/ref_harness.cpp (file:, gen:, hex:).  Prints one line
// per case; exit status 1 if any case differs.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <fstream>
#include <thread>
#include <sstream>
#include <string>
#include <vector>

#include <reflex/matcher.h>

#include "gen.h"
#include "reflex_gpu_matcher.h"

static std::string build_regex(const std::string& mode, const std::string& rx)
{
  // as src/ugrep.cpp:8574-8604, :8849 (see oracle/ref_harness.cpp)
  std::string regex = rx;
  if (mode == "F" && !regex.empty())
  {
    size_t from = 0, to;
    while ((to = regex.find("\\E", from)) != std::string::npos)
    {
      regex.insert(to + 2, "\\\\E\\Q");
      from = to + 7;
    }
    regex.insert(0, "\\Q").append("\\E");
  }
  regex.insert(0, "(?m)");
  return reflex::Matcher::convert(regex, reflex::convert_flag::notnewline | reflex::convert_flag::unicode);
}

static std::vector<char> load_input(const std::string& spec)
{
  std::vector<char> buf;
  if (spec.compare(0, 5, "file:") == 0)
  {
    std::string rest = spec.substr(5);
    size_t total = 0;
    size_t c = rest.rfind(':');
    if (c != std::string::npos && c > 0 && rest.find_first_not_of("0123456789", c + 1) == std::string::npos)
    {
      total = strtoull(rest.c_str() + c + 1, NULL, 10);
      rest = rest.substr(0, c);
    }
    std::ifstream f(rest.c_str(), std::ios::binary);
    std::vector<char> data((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (total == 0)
      total = data.size();
    buf.resize(total);
    for (size_t i = 0; i < total && !data.empty(); ++i)
      buf[i] = data[i % data.size()];
  }
  else if (spec.compare(0, 4, "gen:") == 0)
  {
    int kind;
    unsigned long long seed, off, len;
    if (sscanf(spec.c_str() + 4, "%d:%llu:%llu:%llu", &kind, &seed, &off, &len) == 4)
    {
      buf.resize(len);
      gen_fill(kind, seed, off, reinterpret_cast<uint8_t*>(buf.data()), len);
    }
  }
  else if (spec.compare(0, 4, "hex:") == 0)
  {
    std::string h = spec.substr(4);
    for (size_t i = 0; i + 1 < h.size(); i += 2)
      buf.push_back(static_cast<char>(strtoul(h.substr(i, 2).c_str(), NULL, 16)));
  }
  buf.push_back('\0');  // ugrep passes size+1 (src/ugrep.cpp:3939)
  return buf;
}

struct Hit {
  size_t first, size, accept, lineno, columno;
  bool operator!=(const Hit& o) const
  {
    return first != o.first || size != o.size || accept != o.accept || lineno != o.lineno || columno != o.columno;
  }
};

// loop kind: 0 plain, 1 skip('\n') after each hit, 2 skip(' ') after every other
// hit, 3 plain loop, then new bytes at the same address and size handed over
// with buffer() and a second plain loop (ugrep re-buffers one reused std::string
// per line, src/ugrep.cpp:733-740; buffer() is non-virtual, absmatcher.h:542);
// 4, 5: kinds 0, 1 on a stream; 6: a tokenizer loop, scan() until it fails,
// then input() past one byte (the position of each failure recorded as a hit
// of size 0, accept 0); 7: matches() of the whole buffer
static bool buffer_kind(int kind) { return kind < 4 || kind >= 6; }

template <class M>
static std::vector<Hit> run(M& m, std::vector<char>& buf, int kind, bool& at_end)
{
  std::vector<Hit> out;
  if (kind == 6)
  {
    m.buffer(buf.data(), buf.size());
    for (;;)
    {
      while (m.scan())
        out.push_back(Hit{m.first(), m.size(), m.accept(), m.lineno(), m.columno()});
      if (m.at_end())
        break;
      out.push_back(Hit{m.first(), 0, 0, m.lineno(), m.columno()});
      if (m.input() == EOF)
        break;
    }
    at_end = m.at_end();
    return out;
  }
  if (kind == 7)
  {
    m.buffer(buf.data(), buf.size());
    const size_t r = m.matches();
    out.push_back(Hit{r, r ? m.size() : 0, m.accept(), 0, 0});
    at_end = m.at_end();
    return out;
  }
  for (int pass = 0; pass < (kind == 3 ? 2 : 1); ++pass)
  {
    if (kind < 4)
    {
      if (pass == 1 && buf.size() > 2)  // rotate the data bytes in place, keep the NUL
        std::rotate(buf.begin(), buf.begin() + (buf.size() - 1) / 3, buf.end() - 1);
      m.buffer(buf.data(), buf.size());
    }
    while (m.find())
    {
      out.push_back(Hit{m.first(), m.size(), m.accept(), m.lineno(), m.columno()});
      if (kind == 1 || kind == 5)
        m.skip('\n');
      else if (kind == 2 && (out.size() & 1))
        m.skip(' ');
    }
  }
  at_end = m.at_end();
  return out;
}

// The writer sends one line with a match, then waits (up to 5 s) until the
// reader has reported it, then sends the rest.  Returns 1 on failure.
static int slow_pipe()
{
  const std::string part1 = "alpha foo beta\n", part2 = "gamma bar delta baz\n";
  int fds[2];
  if (pipe(fds) != 0)
    return 1;
  const int saved = dup(0);
  dup2(fds[0], 0);
  close(fds[0]);
  fcntl(0, F_SETFL, fcntl(0, F_GETFL) | O_NONBLOCK);
  clearerr(stdin);
  std::atomic<bool> got_first(false);
  bool timely = false;
  std::thread writer([&] {
    (void)!write(fds[1], part1.data(), part1.size());
    for (int i = 0; i < 500 && !got_first.load(); ++i)
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    timely = got_first.load();
    (void)!write(fds[1], part2.data(), part2.size());
    close(fds[1]);
  });
  reflex::Pattern pat(build_regex("re", "foo|bar|baz"), "r");
  reflex::GpuMatcher gpu(pat, reflex::Input(stdin), NULL);
  gpu.gpu_min_bytes(0);
  gpu.gpu_sparse_max(1 << 30);
  std::vector<size_t> got;
  while (gpu.find())
  {
    got.push_back(gpu.first());
    got_first = true;
  }
  writer.join();
  dup2(saved, 0);
  close(saved);
  clearerr(stdin);
  const std::vector<size_t> want = {6, 21, 31};
  const bool ok = timely && got == want && gpu.gpu_scans() > 0;
  printf("%s gpu slow-pipe: first match before the writer continued: %s, %zu matches, gpu scans %zu\n",
         ok ? "ok" : "FAIL", timely ? "yes" : "no", got.size(), gpu.gpu_scans());
  return ok ? 0 : 1;
}

int main(int argc, char** argv)
{
  if (argc < 2)
  {
    fprintf(stderr, "usage: adapter_test SPECFILE\n");
    return 2;
  }
  setenv("UGPU_ADAPTER_CHUNK", "100000", 0);  // many stream feeds per input
  setenv("UGPU_ADAPTER_WARM", "0", 0);         // the first GPU input waits for the device (no CPU answers meanwhile)
  std::ifstream spec(argv[1]);
  std::string line;
  int bad = 0, n = 0;
  while (std::getline(spec, line))
  {
    if (line.empty() || line[0] == '#')
      continue;
    size_t t1 = line.find('\t'), t2 = line.find('\t', t1 + 1);
    std::string mode = line.substr(0, t1);
    const std::string rx = line.substr(t1 + 1, t2 - t1 - 1), in = line.substr(t2 + 1);
    // mode suffix W: Matcher option W (ugrep -w) on both sides
    const bool word = mode.size() > 1 && mode[mode.size() - 1] == 'W';
    if (word)
      mode.erase(mode.size() - 1);
    const char* opt = word ? "W" : NULL;
    reflex::Pattern pat(build_regex(mode, rx), "r");
    std::vector<char> a = load_input(in), b = a;
    const std::string text(a.data(), a.size() - 1);  // (stream input: no NUL)
    for (int kind = 0; kind < 8; ++kind)
    {
      std::istringstream sa(text), sb(text);
      reflex::Matcher cpu(pat, buffer_kind(kind) ? reflex::Input() : reflex::Input(sa), opt);
      reflex::GpuMatcher gpu(pat, buffer_kind(kind) ? reflex::Input() : reflex::Input(sb), opt);
      gpu.gpu_min_bytes(0);  // parity on every size and pattern (the dispatch policy is measured separately)
      gpu.gpu_sparse_max(1 << 30);
      const bool ready = gpu.gpu_ready();
      bool ea = false, eb = false;
      std::vector<Hit> ra = run(cpu, a, kind, ea), rb = run(gpu, b, kind, eb);
      size_t diff = 0;
      while (diff < ra.size() && diff < rb.size() && !(ra[diff] != rb[diff]))
        ++diff;
      const bool ok = ra.size() == rb.size() && diff == ra.size() && ea == eb;
      printf("%s %s kind=%d /%s/%s %s: cpu %zu gpu %zu matches, gpu scans %zu%s\n", ok ? "ok" : "FAIL",
             ready ? "gpu" : "cpu-only", kind, rx.c_str(), word ? "W" : "", in.substr(0, 40).c_str(), ra.size(),
             rb.size(), gpu.gpu_scans(), ready ? "" : " (engine: unsupported table)");
      if (!ok)
      {
        ++bad;
        if (diff < ra.size() && diff < rb.size())
          printf("  first difference at #%zu: cpu (%zu,%zu,%zu,%zu,%zu) gpu (%zu,%zu,%zu,%zu,%zu)\n", diff,
                 ra[diff].first, ra[diff].size, ra[diff].accept, ra[diff].lineno, ra[diff].columno, rb[diff].first,
                 rb[diff].size, rb[diff].accept, rb[diff].lineno, rb[diff].columno);
      }
      // the GPU path must actually have served supported tables (option W on
      // streams stays on the CPU by design)
      if (ready && gpu.gpu_scans() == 0 && !ra.empty() && !(word && kind >= 4 && kind <= 5))
      {
        printf("FAIL gpu matcher fell back to the CPU for /%s/ kind=%d\n", rx.c_str(), kind);
        ++bad;
      }
      ++n;
    }
  }
  bad += slow_pipe();
  ++n;
  printf("%d cases, %d failed\n", n, bad);
  return bad ? 1 : 0;
}
