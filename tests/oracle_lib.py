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
    L.orc_chain_exit.argtypes = [V, V, U64, U64, U64]
    L.orc_chain_exit.restype = U64
    L.orc_gen.argtypes = [ctypes.c_int, U64, U64, V, U64]
    return L


L = _load()


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

    def find(self, data, start=0, bias=0, want_list=False):
        buf = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
        dg, dc = ctypes.c_uint64(), ctypes.c_uint64()
        cnt = L.orc_find(self.h, buf.ctypes.data, buf.size, start, bias, ctypes.byref(dg), ctypes.byref(dc), None, 0)
        lst = None
        if want_list:
            arr = np.zeros(3 * max(cnt, 1), np.uint64)
            L.orc_find(self.h, buf.ctypes.data, buf.size, start, bias, None, None, arr.ctypes.data, cnt)
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
