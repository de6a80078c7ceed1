// reflex_gpu_matcher.h -- drop-in FIND matcher for ugrep: a reflex::Matcher
// whose FIND over a fully buffered input is served by the MI355X engine
// (include/ugpu.h).  This is the reference-side binding of INTEGRATION.md;
// it includes the reference's <reflex/matcher.h>.
//
// Override point: virtual size_t Matcher::match(Method)
// (include/reflex/matcher.h:1321, called by AbstractMatcher::find
// include/reflex/absmatcher.h:276-280, :1401; ugrep's loop
// `while (matcher->find())` src/ugrep.cpp:10544).
//
// FIND on a buffer() input (include/reflex/absmatcher.h:542-591: eof_ set,
// own_ clear) runs one whole-buffer GPU scan from cur_ at the first call and
// then pops one (start, len, accept) record per call, leaving the matcher in
// the state lib/matcher.cpp:682-746 leaves after a hit:
//   txt_ = buf_ + start, len_ = len, cap_ = accept, cur_ = pos_ = start + len,
//   got_ = buf_[cur_-1] (set_current, absmatcher.h:1571-1580)
// and after exhaustion cap_ = len_ = 0, cur_ = pos_ = end_.
//
// Between finds the caller may move cur_ (skip('\n') for -c, --range, context
// modes: src/ugrep.cpp:10583, :3989).  The FIND chain passes through every
// position that is not strictly inside a match, so the remaining records are
// exact whenever the new cur_ is not inside one; otherwise (and for a new
// buffer) the scan is re-run from cur_.
//
// Option W (ugrep -w, src/ugrep.cpp:8616-8618) is served from a second table
// handle created with UGPU_PAT_WORD (wdfa).  Everything else -- SCAN/SPLIT/
// MATCH, streaming input(), options A/N, tables the engine rejects (anchors,
// \b, lookahead: UGPU_UNSUPPORTED) -- stays on the CPU matcher, unchanged.
#ifndef REFLEX_GPU_MATCHER_H
#define REFLEX_GPU_MATCHER_H

#include <reflex/matcher.h>

#include "ugpu.h"

namespace reflex {

class GpuMatcher : public Matcher {
 public:
  /// dfa: ugpu_dfa_create(pattern's opc_ words, 0) or NULL (CPU only); wdfa:
  /// the same words with UGPU_PAT_WORD, used when opt has W; not owned.
  GpuMatcher(const Pattern& pattern, const ugpu_dfa* dfa, const char* opt = NULL, const ugpu_dfa* wdfa = NULL)
      : Matcher(pattern, Input(), opt), dfa_(opt_.W ? wdfa : dfa)
  {
  }
  ~GpuMatcher() { ugpu_result_free(gres_); }

  /// Number of whole-buffer GPU scans issued so far (for tests).
  size_t gpu_scans() const { return scans_; }

 protected:
  virtual size_t match(Method method)
  {
    if (method != Const::FIND || dfa_ == NULL || own_ || !eof_ || opt_.A || opt_.N)
      return Matcher::match(method);
    // buffer() and reset() are non-virtual and rewind cur_ without telling this
    // class (absmatcher.h:542-591), and the caller may hand over new bytes at
    // the same address and size (ugrep re-buffers one std::string per line,
    // src/ugrep.cpp:733-740): any cursor behind the one this class last left
    // means the records may be stale, so scan again
    if (gres_ == NULL || gbuf_ != buf_ || gend_ != end_ || cur_ < gcur_ || inside_match())
      if (!rescan())
        return Matcher::match(method);
    while (gi_ < gres_->count && gres_->start[gi_] < cur_)
      ++gi_;
    if (gi_ >= gres_->count)
    {
      set_current(end_);
      txt_ = buf_ + end_;
      len_ = 0;
      gcur_ = cur_;
      return cap_ = 0;
    }
    const size_t start = static_cast<size_t>(gres_->start[gi_]);
    txt_ = buf_ + start;
    len_ = gres_->len[gi_];
    cap_ = gres_->cap[gi_];
    set_current(start + len_);
    gcur_ = cur_;
    ++gi_;
    return cap_;
  }

 private:
  // cur_ lies strictly inside a match of the current record set
  bool inside_match()
  {
    size_t i = gi_ > 0 ? gi_ - 1 : 0;
    while (i < gres_->count && gres_->start[i] + gres_->len[i] <= cur_)
      ++i;
    return i < gres_->count && gres_->start[i] < cur_;
  }
  bool rescan()
  {
    ugpu_result_free(gres_);
    gres_ = NULL;
    if (ugpu_find_all(dfa_, reinterpret_cast<const uint8_t*>(buf_), end_, cur_, UGPU_MODE_OFFSETS, &gres_) != UGPU_OK)
    {
      dfa_ = NULL;  // engine unavailable for this input: stay on the CPU matcher
      return false;
    }
    ++scans_;
    gbuf_ = buf_;
    gend_ = end_;
    gcur_ = cur_;
    gi_ = 0;
    return true;
  }

  const ugpu_dfa* dfa_;
  ugpu_result* gres_ = NULL;
  const char* gbuf_ = NULL;
  // gcur_: the cursor this class left behind (after the scan or the last hit)
  size_t gend_ = 0, gcur_ = 0, gi_ = 0, scans_ = 0;
};

}  // namespace reflex

#endif
