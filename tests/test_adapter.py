"""GPU: the drop-in C++ adapter reflex::GpuMatcher (integration/reflex_gpu_matcher.h)
against the reference reflex::Matcher on the same inputs, both linked into
tests/adapter/build/adapter_test (built with the reference headers in the
development container; see tests/adapter/Makefile).  Each case compares the
plain find() loop, the -c loop with skip('\\n'), and a loop that moves cur_
with skip(' ') between finds, including lineno()/columno() after each hit."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "adapter", "build", "adapter_test")
SPEC = os.path.join(ROOT, "tests", "adapter", "cases.tsv")


@pytest.mark.gpu
def test_reflex_gpu_matcher_drop_in():
    if not os.path.exists(EXE):
        pytest.skip("adapter_test not built (needs the reference headers at build time: make -C tests/adapter)")
    r = subprocess.run([EXE, SPEC], cwd=ROOT, capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert " 0 failed" in out
    # supported tables really ran on the GPU engine
    assert sum(1 for ln in out.splitlines() if ln.startswith("ok gpu")) >= 30, out[-3000:]
