"""Test-side loader of the oracle restatement (oracle/_build/liboracle.so).

Test infrastructure only: used by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker, never by the product path.
"""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
LIB = os.path.join(ORACLE_DIR, "_build", "liboracle.so")
GOLDEN = os.path.join(REPO, "tests", "golden")


def _load():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR, "restate"])
    L = ctypes.CDLL(LIB)
    V, U64 = ctypes.c_void_p, ctypes.c_uint64
    P64 = ctypes.POINTER(ctypes.c_uint64)
    L.orc_dfa_build.argtypes = [V, ctypes.c_uint32, ctypes.POINTER(V)]
    L.orc_dfa_build.restype = ctypes.c_int
    L.orc_dfa_free.argtypes = [V]
    L.orc_dfa_nstates.argtypes = [V]
    L.orc_dfa_nstates.restype = ctypes.c_uint32
    L.orc_find.argtypes = [V, V, U64, U64, U64, P64, P64, V, U64]
    L.orc_find.restype = U64
    L.orc_find_mt.argtypes = [V, V, U64, ctypes.c_int, P64, P64]
    L.orc_find_mt.restype = U64
    L.orc_find_w.argtypes = [V, V, U64, U64, P64, P64, V, U64]
    L.orc_find_w.restype = U64
    L.orc_find_a.argtypes = [V, V, U64, U64, ctypes.c_int, P64, P64, V, U64]
    L.orc_find_a.restype = U64
    L.orc_dfa_anchored.argtypes = [V]
    L.orc_dfa_anchored.restype = ctypes.c_int
    L.orc_chain_exit.argtypes = [V, V, U64, U64, U64]
    L.orc_chain_exit.restype = U64
    L.orc_gen.argtypes = [ctypes.c_int, U64, U64, V, U64]
    L.orc_isutf8.argtypes = [V, U64]
    L.orc_isutf8.restype = ctypes.c_int
    L.orc_utf8_first_bad.argtypes = [V, U64]
    L.orc_utf8_first_bad.restype = U64
    L.orc_init_window.argtypes = [V, U64]
    L.orc_init_window.restype = ctypes.c_int64
    return L


L = _load()


_DFA_CACHE = {}


def oracle_dfa(opc):
    """OracleDfa of opc, cached (tests build the same tables many times)."""
    key = bytes(np.ascontiguousarray(np.asarray(opc, dtype=np.uint32)).tobytes())
    d = _DFA_CACHE.get(key)
    if d is None:
        d = _DFA_CACHE[key] = OracleDfa(opc)
    return d


def range_totals(opc, host, lo, hi):
    """(count, digest, dcap, exit) of the FIND chain entering at lo over the
    whole of host, counting the matches that start before hi; exit is the end
    of the last such match when it runs past hi, else hi.  (The scanners'
    ugpu_scan(lo, hi) totals; numpy sums wrap mod 2**64 like the digests.)"""
    o = oracle_dfa(opc)
    if o.anchored:
        _, _, _, lst = o.find(host, start=lo, want_list=True)
        a = np.asarray(lst, dtype=np.uint64).reshape(-1, 3)
        st, ln, cp = a[:, 0], a[:, 1], a[:, 2]
    else:
        st, ln, cp = o.find_arrays(host, start=lo)
    k = int(np.searchsorted(st, np.uint64(hi), side="left"))
    ex = hi
    if not k:
        return 0, 0, 0, ex
    s, l, c = st[:k], ln[:k], cp[:k]
    with np.errstate(over="ignore"):
        dg = int((s * np.uint64(31) + l).sum(dtype=np.uint64))
        dc = int(((s + np.uint64(1)) * c).sum(dtype=np.uint64))
    end = int(s[-1]) + int(l[-1])
    if end > hi:
        ex = end
    return k, dg, dc, ex


class OracleDfa:
    def __init__(self, opc):
        self.opc = np.ascontiguousarray(np.asarray(opc, dtype=np.uint32))
        h = ctypes.c_void_p()
        self.rc = L.orc_dfa_build(self.opc.ctypes.data, len(self.opc), ctypes.byref(h))
        self.h = h if self.rc == 0 else None

    @property
    def supported(self):
        return self.rc == 0

    def nstates(self):
        return L.orc_dfa_nstates(self.h)

    @property
    def anchored(self):
        if self.h is None:
            raise ValueError("the oracle refused this table (rc %d)" % self.rc)
        return bool(L.orc_dfa_anchored(self.h))

    def find(self, data, start=0, bias=0, want_list=False, nul=False):
        """FIND over data[start:] (orc_find; orc_find_a for tables with ^/$
        edges or with option N, nul=True): (count, digest, dcap, list|None)."""
        buf = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
        if nul or self.anchored:
            assert bias == 0
            dg, dc = ctypes.c_uint64(), ctypes.c_uint64()
            cnt = L.orc_find_a(self.h, buf.ctypes.data, buf.size, start, int(nul), ctypes.byref(dg), ctypes.byref(dc),
                               None, 0)
            lst = None
            if want_list:
                arr = np.zeros(3 * max(cnt, 1), np.uint64)
                L.orc_find_a(self.h, buf.ctypes.data, buf.size, start, int(nul), None, None, arr.ctypes.data, cnt)
                lst = arr[:3 * cnt].reshape(-1, 3).tolist()
            return cnt, dg.value, dc.value, lst
        dg, dc = ctypes.c_uint64(), ctypes.c_uint64()
        cnt = L.orc_find(self.h, buf.ctypes.data, buf.size, start, bias, ctypes.byref(dg), ctypes.byref(dc), None, 0)
        lst = None
        if want_list:
            arr = np.zeros(3 * max(cnt, 1), np.uint64)
            L.orc_find(self.h, buf.ctypes.data, buf.size, start, bias, None, None, arr.ctypes.data, cnt)
            lst = arr[:3 * cnt].reshape(-1, 3).tolist()
        return cnt, dg.value, dc.value, lst

    def find_arrays(self, data, start=0):
        """FIND over data[start:] as numpy arrays (start, len, cap) of uint64,
        for match lists too long for Python lists."""
        buf = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
        cnt = L.orc_find(self.h, buf.ctypes.data, buf.size, start, 0, None, None, None, 0)
        arr = np.zeros(3 * max(cnt, 1), np.uint64)
        L.orc_find(self.h, buf.ctypes.data, buf.size, start, 0, None, None, arr.ctypes.data, cnt)
        a = arr[:3 * cnt].reshape(-1, 3)
        return a[:, 0], a[:, 1], a[:, 2]

    def find_w(self, data, start=0, want_list=False):
        """FIND with option W (ugrep -w, orc_find_w): (count, digest, dcap, list|None)."""
        buf = _u8(data)
        dg, dc = ctypes.c_uint64(), ctypes.c_uint64()
        cnt = L.orc_find_w(self.h, buf.ctypes.data, buf.size, start, ctypes.byref(dg), ctypes.byref(dc), None, 0)
        lst = None
        if want_list:
            arr = np.zeros(3 * max(cnt, 1), np.uint64)
            L.orc_find_w(self.h, buf.ctypes.data, buf.size, start, None, None, arr.ctypes.data, cnt)
            lst = arr[:3 * cnt].reshape(-1, 3).tolist()
        return cnt, dg.value, dc.value, lst

    def find_mt(self, buf, threads):
        dg, dc = ctypes.c_uint64(), ctypes.c_uint64()
        cnt = L.orc_find_mt(self.h, buf.ctypes.data, buf.size, threads, ctypes.byref(dg), ctypes.byref(dc))
        return cnt, dg.value, dc.value

    def chain_exit(self, buf, x, e):
        return L.orc_chain_exit(self.h, buf.ctypes.data, buf.size, x, e)

    def __del__(self):
        if getattr(self, "h", None):
            L.orc_dfa_free(self.h)


def gen(kind, seed, off, length):
    buf = np.zeros(length, np.uint8)
    L.orc_gen(kind, seed, off, buf.ctypes.data, length)
    return buf


def _u8(data):
    return np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data)


def isutf8(data):
    """reflex::isutf8 restated (lib/simd.cpp:391-418)."""
    b = _u8(data)
    return bool(L.orc_isutf8(b.ctypes.data, b.size))


def utf8_first_bad(data):
    """First failing position (len for a cut-off sequence) or None when valid."""
    b = _u8(data)
    r = L.orc_utf8_first_bad(b.ctypes.data, b.size)
    return None if r == b.size + 1 else int(r)


def first_nul(data):
    b = _u8(data)
    z = np.flatnonzero(b == 0)
    return int(z[0]) if z.size else None


def is_binary(data, null_data=False, nul_only=False, init_window=False):
    """ugrep's is_binary (src/ugrep.cpp:699-711), with init_is_binary's trim
    (:3998-4015) when init_window."""
    b = _u8(data)
    n = b.size
    if init_window:
        w = L.orc_init_window(b.ctypes.data, n)
        if w < 0:
            return True
        n = int(w)
    if null_data:
        return False
    if nul_only:
        return first_nul(b[:n]) is not None
    return not isutf8(b[:n])


def case_input(inp):
    """Bytes of a golden-case input description."""
    t = inp["type"]
    if t == "hex":
        return np.frombuffer(bytes.fromhex(inp["hex"]), np.uint8)
    if t == "file":
        data = open(os.path.join(GOLDEN, inp["name"]), "rb").read()
        total = inp.get("total")
        if total:
            reps = -(-total // len(data))
            data = (data * reps)[:total]
        return np.frombuffer(data, np.uint8)
    if t == "gen":
        return gen(inp["kind"], inp["seed"], inp["off"], inp["len"])
    raise ValueError(t)
