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
the harness).  GPU test: ugrep_gpu with UGPU_ADAPTER_MIN_BYTES=0 (every input on the GPU,
the suite's files are tiny) and the default device queue reproduces them too,
and the engine really served the FIND calls (adapter statistics on stderr)."""
import hashlib
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CWD = os.path.join(ROOT, "tests", "golden", "verify")
SPEC = json.load(open(os.path.join(ROOT, "tests", "golden", "verify_cases.json")))


def _stats(stderr):
    """The adapter's per-matcher statistics lines (UGPU_ADAPTER_STATS=1):
    scans, FIND calls answered from GPU records, FIND calls the CPU matcher
    answered, whether the engine took the table, and the CPU calls by reason."""
    out = []
    for ln in stderr.decode(errors="replace").splitlines():
        if ln.startswith("[ugpu-adapter] "):
            kv = dict(f.split("=", 1) for f in ln.split()[1:])
            why = {} if kv["cpu_why"] == "-" else {k: int(v) for k, v in (w.split(":") for w in kv["cpu_why"].split(","))}
            out.append(dict(scans=int(kv["scans"]), gpu=int(kv["gpu_finds"]), cpu=int(kv["cpu_finds"]),
                            table=kv["table"], why=why))
    return out


def _run_all(exe, env, workers=8):
    """Every case, `workers` ugrep processes at a time (each its own GPU
    context on the GPU run: well under the box's per-card process limit)."""
    from concurrent.futures import ThreadPoolExecutor
    env = dict(env, **SPEC["env"])
    env.pop("UGREP_COLORS", None)

    def one(c):
        r = subprocess.run([exe] + c["args"], cwd=CWD, env=env, capture_output=True, timeout=120,
                           input=open(os.path.join(CWD, c["stdin"]), "rb").read() if c["stdin"] else None)
        return c, r

    bad, ledger = [], []
    with ThreadPoolExecutor(workers) as ex:
        for c, r in ex.map(one, SPEC["cases"]):
            h = hashlib.sha256(r.stdout).hexdigest()
            if h != c["sha256"]:
                bad.append((c["args"], c["expect"], len(r.stdout), c["size"]))
            ledger.append(dict(expect=c["expect"], args=c["args"], matchers=_stats(r.stderr)))
    return bad, ledger


# CPU answers that are by design: line anchors the reference's match predictor
# decides (anchored tables without option N or with anchors inside the regex:
# tests/test_anchor.py), and inputs of prefiltered tables that found the
# device queue's slots taken, or that came while the devices warmed up (the
# CPU matcher scans them meanwhile; both are timing, so these reasons are left
# out of the ledger)
BY_DESIGN = {"anchor_predictor", "sparse_limit", "warmup", "cold"}
TIMING = {"sparse_limit", "warmup", "cold"}
LEDGER = os.path.join(ROOT, "tests", "golden", "dropin_fallbacks.json")


def test_fixture_size():
    assert len(SPEC["cases"]) > 150


def test_reference_ugrep_reproduces_goldens():
    exe = os.path.join(ROOT, "oracle", "_ref", "ugrep")
    if not os.path.exists(exe):
        pytest.skip("reference ugrep not built (make -C oracle ref, build container)")
    bad, _ = _run_all(exe, dict(os.environ))
    assert not bad, bad[:5]


def test_fallback_ledger_is_consistent():
    """The committed ledger of cases in which the CPU matcher answered FIND
    calls names a reason for each, and only reasons of the adapter."""
    if not os.path.exists(LEDGER):
        pytest.skip("no ledger yet")
    led = json.load(open(LEDGER))
    known = {"method", "option_A", "anchor_predictor", "table", "sparse_limit", "partial", "small", "engine", "warmup", "cold"}
    expects = {c["expect"] for c in SPEC["cases"]}
    for e, why in led["cpu_cases"].items():
        assert e in expects, e
        assert why and set(why) <= known, (e, why)


def test_dropin_default_policy_never_touches_a_device():
    """ugrep_gpu with the adapter's default policy on the suite's small inputs:
    the CPU matcher answers (reason "small"), decided on the host -- the
    tables are planned by ugpu_dfa_plan_host, no HIP call is made, so this runs
    in a container without a GPU and no FIND call falls back for "engine"."""
    exe = os.path.join(ROOT, "oracle", "_ref", "ugrep_gpu")
    if not os.path.exists(exe):
        pytest.skip("ugrep_gpu not built (make -C oracle ref, build container)")
    env = dict(os.environ, UGPU_ADAPTER_STATS="1")
    for k in ("UGPU_ADAPTER_MIN_BYTES", "UGPU_ADAPTER_SPARSE_MAX"):
        env.pop(k, None)
    bad, ledger = _run_all(exe, env)
    assert not bad, bad[:5]
    why = {}
    for c in ledger:
        for m in c["matchers"]:
            assert m["scans"] == 0, (c["expect"], m)
            for k in m["why"]:
                why[k] = why.get(k, 0) + 1
    assert "engine" not in why, why
    assert why.get("small", 0) > 100, why


def test_dropin_links_no_hip_runtime():
    """ugrep_gpu links the engine's host half only
    (libugpu_host.so); the device half and the HIP runtime are dlopen()ed at
    the first input the adapter's policy sends to a GPU, so a CPU-served run
    does not pay for loading them."""
    exe = os.path.join(ROOT, "oracle", "_ref", "ugrep_gpu")
    if not os.path.exists(exe):
        pytest.skip("ugrep_gpu not built (make -C oracle ref, build container)")
    out = subprocess.run(["readelf", "-d", exe], capture_output=True, check=True).stdout.decode()
    needed = [ln.split("[")[1].split("]")[0] for ln in out.splitlines() if "(NEEDED)" in ln]
    assert "libugpu_host.so" in needed, needed
    assert not any("ugrep_amd" in n or "amdhip" in n or "hsa" in n for n in needed), needed
    host = os.path.join(ROOT, "ugrep_amd", "libugpu_host.so")
    out = subprocess.run(["readelf", "-d", host], capture_output=True, check=True).stdout.decode()
    assert "amdhip" not in out and "hsa-runtime" not in out


@pytest.mark.gpu
def test_dropin_ugrep_reproduces_goldens():
    exe = os.path.join(ROOT, "oracle", "_ref", "ugrep_gpu")
    if not os.path.exists(exe):
        pytest.skip("ugrep_gpu not built (make -C oracle ref, build container)")
    # every input on the GPU (the suite's files are tiny), the device queue
    # at its default size; the first GPU input waits for the device warm-up
    # (by default the CPU matcher answers meanwhile, and these inputs would be
    # done before the device is)
    env = dict(os.environ, UGPU_ADAPTER_MIN_BYTES="0", UGPU_ADAPTER_STATS="1", UGPU_ADAPTER_WARM="0")
    env.pop("UGPU_ADAPTER_SPARSE_MAX", None)
    bad, ledger = _run_all(exe, env)
    assert not bad, bad[:5]
    # attribution: per case, which FIND calls the GPU answered and why the CPU
    # answered the others
    cpu_cases, served, leaks = {}, 0, []
    for c in ledger:
        why = {}
        for m in c["matchers"]:
            for k, v in m["why"].items():
                if k not in TIMING:
                    why[k] = why.get(k, 0) + v
            # a table the engine accepted: every FIND call not excluded by design ran on the GPU
            if m["table"] == "gpu" and set(m["why"]) - BY_DESIGN:
                leaks.append((c["expect"], m))
        if any(m["gpu"] for m in c["matchers"]):
            served += 1
        if why:
            cpu_cases[c["expect"]] = sorted(why)
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "dropin_ledger.json"), "w") as f:
        json.dump(dict(served_by_gpu=served, cases=len(ledger), cpu_cases=cpu_cases, detail=ledger), f, indent=1)
    assert not leaks, leaks[:5]
    assert served > 100, served
    if os.path.exists(LEDGER):  # the committed list of cases the CPU (partly) answered, and why
        want = json.load(open(LEDGER))
        diff = sorted(k for k in set(cpu_cases) | set(want["cpu_cases"]) if cpu_cases.get(k) != want["cpu_cases"].get(k))
        assert not diff, [(k, cpu_cases.get(k), want["cpu_cases"].get(k)) for k in diff[:10]]
        assert served == want["served_by_gpu"]


# word-boundary searches: ugrep_gpu against the reference
# build on the same files, byte for byte; the finite patterns are served by the
# GPU, a boundary after a loop stays on the CPU matcher (reason
# anchor_predictor: the reference's match predictor decides there)
WORDB_CMDS = [(["-co", r"\bdolor\b"], True), (["-on", r"\<con"], True), (["-c", r"um\>"], True),
              (["-co", r"\Bor\B"], True), (["-io", r"\b(lorem|ipsum|sit)\b"], True), (["-o", r"\<(in|ut)\>"], True),
              (["-co", r"\w+\b"], False)]


# negative patterns (ugrep -N: (?^...) alternatives, REDO accepts)
NEG_CMDS = [(["-co", "-N", "dolor", "-e", r"dolor\w*"], True), (["-on", "-N", "sit", "-e", r"s[a-z]+"], True),
            (["-c", "-N", "con", "-N", "in", "-e", r"[a-z]+"], True), (["-o", "-U", "-N", "ad", "-e", r"a[a-z]"], True),
            (["-co", "-N", "lorem", "-e", r"\w+"], True)]


# lookahead X(?=Y): the native compiler emits the
# reference's TAIL/HEAD words (tests/test_lookahead_compile.py), so these
# commands go to the GPU's lookahead walk; Unicode and -U, -i, -c/-o/-n
# (-J1: one worker takes both files, so the second file does not meet the
# device warming up for the first -- reason "warmup", timing -- and every FIND
# call of every command is the GPU's)
LOOK_CMDS = [(["-J1", "-co", "dolor(?= sit)"], True), (["-J1", "-on", r"[a-z]+(?=,)"], True),
             (["-J1", "-o", r"\w+(?=\.)"], True), (["-J1", "-c", r"(?:lorem|ipsum)(?= )"], True),
             (["-J1", "-o", "-U", r"in(?=c|t)"], True), (["-J1", "-co", "-i", r"ut(?= [a-z]+)"], True),
             (["-J1", "-o", r"[A-Z]\w*(?= [a-z])"], True)]


# word boundaries inside a leading or trailing group (the compiler distributes
# the group, tests/test_asgroup.py); line anchors in such groups compile too
# but stay with the reference's match predictor (reason anchor_predictor)
ASGROUP_CMDS = [(["-J1", "-co", r"(\bdolor|amet,)"], True), (["-J1", "-on", r"(\<in|ut\>)"], True),
                (["-J1", "-o", r"(\bsit|\bamet)\b"], True), (["-J1", "-co", r"(^|, )[a-z]+"], False)]


@pytest.mark.gpu
def test_dropin_assertion_groups(tmp_path):
    _dropin_ledger(tmp_path, ASGROUP_CMDS, "dropin_asgroup_ledger.json")


# lookahead under option W (ugrep -w; tests/test_lookahead_w.py)
LOOK_W_CMDS = [(["-J1", "-cow", "dolor(?= sit)"], True), (["-J1", "-onw", r"[a-z]+(?=,)"], True),
               (["-J1", "-ow", r"\w+(?=\.)"], True)]


@pytest.mark.gpu
def test_dropin_lookahead_word_on_gpu(tmp_path):
    _dropin_ledger(tmp_path, LOOK_W_CMDS, "dropin_lookahead_w_ledger.json")


@pytest.mark.gpu
def test_dropin_lookahead_on_gpu(tmp_path):
    """ugrep lookahead commands served by the GPU, byte-equal to the reference build."""
    _dropin_ledger(tmp_path, LOOK_CMDS, "dropin_lookahead_ledger.json")


@pytest.mark.gpu
def test_dropin_word_boundaries_on_gpu(tmp_path):
    _dropin_ledger(tmp_path, WORDB_CMDS, "dropin_wordb_ledger.json")


# negative patterns under option W (ugrep -w -N; REDO accepts skip at_we,
# tests/test_redo_w.py)
NEG_W_CMDS = [(["-J1", "-cow", "-N", "dolor", "-e", r"dolor\w*"], True),
              (["-J1", "-ow", "-N", "sit", "-e", r"s[a-z]+"], True),
              (["-J1", "-cw", "-N", "lorem", "-e", r"\w+"], True)]


@pytest.mark.gpu
def test_dropin_negative_patterns_word_on_gpu(tmp_path):
    _dropin_ledger(tmp_path, NEG_W_CMDS, "dropin_redo_w_ledger.json")


@pytest.mark.gpu
def test_dropin_negative_patterns_on_gpu(tmp_path):
    """ugrep -N commands served by the GPU (REDO accepts),
    byte-equal to the reference build."""
    _dropin_ledger(tmp_path, NEG_CMDS, "dropin_redo_ledger.json")


def _dropin_ledger(tmp_path, cmds, ledger_name):
    exe_gpu = os.path.join(ROOT, "oracle", "_ref", "ugrep_gpu")
    exe_ref = os.path.join(ROOT, "oracle", "_ref", "ugrep")
    if not (os.path.exists(exe_gpu) and os.path.exists(exe_ref)):
        pytest.skip("ugrep builds missing (make -C oracle ref, build container)")
    import numpy as np
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import gen
    lorem = open(os.path.join(CWD, "lorem.utf8.txt"), "rb").read()
    (tmp_path / "lorem1m.txt").write_bytes((lorem * (1 + (1 << 20) // len(lorem)))[:1 << 20])
    (tmp_path / "words.txt").write_bytes(np.asarray(gen(4, 5, 0, 3 << 20)).tobytes())
    files = ["lorem1m.txt", "words.txt"]
    env = dict(os.environ, UGPU_ADAPTER_MIN_BYTES="0", UGPU_ADAPTER_STATS="1", UGPU_ADAPTER_WARM="0")
    ledger = []
    for args, on_gpu in cmds:
        ref = subprocess.run([exe_ref, "--sort"] + args + files, cwd=tmp_path, capture_output=True, timeout=120, env=env)
        got = subprocess.run([exe_gpu, "--sort"] + args + files, cwd=tmp_path, capture_output=True, timeout=120, env=env)
        assert ref.returncode == got.returncode, args
        assert got.stdout == ref.stdout, (args, len(got.stdout), len(ref.stdout))
        st = _stats(got.stderr)
        gpu_finds = sum(m["gpu"] for m in st)
        ledger.append(dict(args=args, out_bytes=len(ref.stdout), gpu_finds=gpu_finds,
                           cpu_finds=sum(m["cpu"] for m in st), why=[m["why"] for m in st if m["why"]]))
        if on_gpu:
            # (matchers ugrep built but never ran show table "none"; a FIND
            # call past a file's last record may go to the CPU matcher)
            assert gpu_finds > 0 and not any(m["table"] == "unsupported" for m in st), (args, st)
            assert not any({"anchor_predictor", "table", "engine"} & set(m["why"]) for m in st), (args, st)
        else:
            assert gpu_finds == 0 and any("anchor_predictor" in m["why"] for m in st), (args, st)
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, ledger_name), "w") as f:
        json.dump(ledger, f, indent=1)


@pytest.mark.gpu
def test_dropin_workers_wait_for_warmup(tmp_path):
    """with the default warm-up policy, workers that meet the
    device warming wait for it, so no FIND call goes to the reference matcher
    (reason "warmup"), and the output equals the reference build's."""
    exe_gpu = os.path.join(ROOT, "oracle", "_ref", "ugrep_gpu")
    exe_ref = os.path.join(ROOT, "oracle", "_ref", "ugrep")
    if not (os.path.exists(exe_gpu) and os.path.exists(exe_ref)):
        pytest.skip("ugrep builds missing (make -C oracle ref, build container)")
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import gen
    files = []
    for k in range(4):
        p = tmp_path / ("c3_%d.txt" % k)
        p.write_bytes(gen(3, 1, k << 23, 8 << 20).tobytes())
        files.append(p.name)
    env = dict(os.environ, UGPU_ADAPTER_MIN_BYTES="0", UGPU_ADAPTER_STATS="1")
    env.pop("UGPU_ADAPTER_WARM", None)
    args = ["--sort", "-co", "-J4", "[A-Za-z_][A-Za-z0-9_]*"] + files
    ref = subprocess.run([exe_ref] + args, cwd=tmp_path, capture_output=True, timeout=120, env=env)
    got = subprocess.run([exe_gpu] + args, cwd=tmp_path, capture_output=True, timeout=120, env=env)
    assert got.returncode == ref.returncode and got.stdout == ref.stdout
    st = _stats(got.stderr)
    assert sum(m["gpu"] for m in st) > 0, st
    assert not any("warmup" in m["why"] for m in st), st
    assert sum(m["cpu"] for m in st) == 0, st


@pytest.mark.gpu
def test_dropin_exit_releases_nothing_after_teardown(tmp_path):
    """ugrep keeps its matcher in a global unique_ptr (src/ugrep.cpp:4491), so
    the adapter releases its last stream and tables from a static destructor,
    after the engine's pools and the HIP runtime were torn down.  Before the
    engine's exit guard (engine.hip exit_guard_arm) about 1 run in 20 of this
    command aborted at exit ("corrupted double-linked list", rc 134); 280 runs
    after it exited cleanly (profiles/r06_exit_abort.txt).  Here: 25 runs,
    every one exits 0 with the reference build's output."""
    exe_gpu = os.path.join(ROOT, "oracle", "_ref", "ugrep_gpu")
    exe_ref = os.path.join(ROOT, "oracle", "_ref", "ugrep")
    if not (os.path.exists(exe_gpu) and os.path.exists(exe_ref)):
        pytest.skip("ugrep builds missing (make -C oracle ref, build container)")
    lorem = open(os.path.join(CWD, "lorem.utf8.txt"), "rb").read()
    (tmp_path / "lorem1m.txt").write_bytes((lorem * (1 + (1 << 20) // len(lorem)))[:1 << 20])
    env = dict(os.environ, UGPU_ADAPTER_MIN_BYTES="0", UGPU_ADAPTER_STATS="1", UGPU_ADAPTER_WARM="0")
    args = ["--sort", "-J1", "-o", r"\w+", "lorem1m.txt"]
    ref = subprocess.run([exe_ref] + args, cwd=tmp_path, capture_output=True, timeout=120, env=env)
    assert ref.returncode == 0
    for i in range(25):
        got = subprocess.run([exe_gpu] + args, cwd=tmp_path, capture_output=True, timeout=120, env=env)
        assert got.returncode == 0, (i, got.returncode, got.stderr[-400:])
        assert got.stdout == ref.stdout
        st = _stats(got.stderr)
        assert sum(m["gpu"] for m in st) > 0, st
