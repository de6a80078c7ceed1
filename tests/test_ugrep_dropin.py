"""ugrep itself with the drop-in adapter: oracle/_ref/ugrep_gpu is ugrep's own
sources (compiled where they lie, oracle/Makefile) with reflex::GpuMatcher at
its two Matcher construction sites (src/ugrep.cpp:8902, :8920) -- the only
change -- linked with the reference libreflex and libugrep_amd.so.

Cases: a subset of the reference's CLI suite tests/verify.sh (Hello loops over
24 output modes and -F/-G/-w/-x variants, -iwco over UTF-8/16/32 and Latin-1
input, --bool queries), each expected output pinned by the SHA-256 of the
reference's own golden file tests/out/*.out (tests/golden/verify_cases.json,
tools/gen_verify_golden.py; inputs copied to tests/golden/verify/).

CPU test: the reference build oracle/_ref/ugrep reproduces every golden (pins
the harness).  GPU test: ugrep_gpu with UGPU_ADAPTER_MIN_BYTES=0 and no sparse
limit (every input on the GPU, the suite's files are tiny) reproduces them too, and the engine
really served the FIND calls (adapter statistics on stderr)."""
import hashlib
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CWD = os.path.join(ROOT, "tests", "golden", "verify")
SPEC = json.load(open(os.path.join(ROOT, "tests", "golden", "verify_cases.json")))


def _run_all(exe, env):
    env = dict(env, **SPEC["env"])
    env.pop("UGREP_COLORS", None)
    bad, scans = [], 0
    for c in SPEC["cases"]:
        r = subprocess.run([exe] + c["args"], cwd=CWD, env=env, capture_output=True, timeout=60,
                           input=open(os.path.join(CWD, c["stdin"]), "rb").read() if c["stdin"] else None)
        h = hashlib.sha256(r.stdout).hexdigest()
        if h != c["sha256"]:
            bad.append((c["args"], c["expect"], len(r.stdout), c["size"]))
        for ln in r.stderr.decode(errors="replace").splitlines():
            if ln.startswith("[ugpu-adapter] scans="):
                scans += int(ln.split("=")[1])
    return bad, scans


def test_fixture_size():
    assert len(SPEC["cases"]) > 150


def test_reference_ugrep_reproduces_goldens():
    exe = os.path.join(ROOT, "oracle", "_ref", "ugrep")
    if not os.path.exists(exe):
        pytest.skip("reference ugrep not built (make -C oracle ref, build container)")
    bad, _ = _run_all(exe, dict(os.environ))
    assert not bad, bad[:5]


@pytest.mark.gpu
def test_dropin_ugrep_reproduces_goldens():
    exe = os.path.join(ROOT, "oracle", "_ref", "ugrep_gpu")
    if not os.path.exists(exe):
        pytest.skip("ugrep_gpu not built (make -C oracle ref, build container)")
    env = dict(os.environ, UGPU_ADAPTER_MIN_BYTES="0", UGPU_ADAPTER_SPARSE_MAX="1000000", UGPU_ADAPTER_STATS="1")
    bad, scans = _run_all(exe, env)
    assert not bad, bad[:5]
    assert scans > 100, scans
