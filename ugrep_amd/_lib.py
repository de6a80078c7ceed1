"""ctypes binding of the in-tree engine library libugrep_amd.so (include/ugpu.h).

The product path is the HIP engine only: if the library is missing this module
raises ImportError instead of falling back to any CPU implementation.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# UGPU_LIB selects an in-tree build variant (benchmarking experiments only)
LIB_PATH = os.path.join(HERE, os.path.basename(os.environ.get("UGPU_LIB", "libugrep_amd.so")))
HEADER = os.path.join(os.path.dirname(HERE), "include", "ugpu.h")

UGPU_OK = 0
UGPU_UNSUPPORTED = 1
UGPU_INVAL = 2
UGPU_NOMEM = 3
UGPU_DEVICE = 4
UGPU_HALO = 5
UGPU_CAPACITY = 6

SHAPE_FINITE, SHAPE_WORD_COND, SHAPE_ONE_ACCEPT, SHAPE_LOOP_NEEDLE, SHAPE_LOOKAHEAD = 1, 2, 4, 8, 16

MODE_COUNT = 0
MODE_OFFSETS = 1

GEN_WORDS, GEN_PLANTED, GEN_CODE, GEN_UTF8 = 1, 2, 3, 4

BIN_NULL_DATA, BIN_NUL_ONLY, BIN_INIT_WINDOW = 1, 2, 4

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_u16p = ctypes.POINTER(ctypes.c_uint16)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_u64p = ctypes.POINTER(ctypes.c_uint64)


class DfaInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in
                ("states", "classes", "row", "format", "table_bytes", "prefilter_ppm", "first_bytes", "accepting",
                 "kernel", "contexts", "shape")]


class Totals(ctypes.Structure):
    _fields_ = [("count", ctypes.c_uint64), ("digest", ctypes.c_uint64), ("dcap", ctypes.c_uint64),
                ("entry", ctypes.c_uint64), ("exit", ctypes.c_uint64), ("flags", ctypes.c_uint32),
                ("fix_rounds", ctypes.c_uint32)]


class Result(ctypes.Structure):
    _fields_ = [("count", ctypes.c_uint64), ("digest", ctypes.c_uint64), ("dcap", ctypes.c_uint64),
                ("start", c_u64p), ("len", c_u32p), ("cap", c_u32p)]


class UgpuError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("ugpu error %d: %s" % (code, msg))
        self.code = code


class Unsupported(UgpuError):
    pass


def _torch_runtime_first():
    """One HIP runtime per process.  The engine library links libamdhip64 by
    soname; when PyTorch-ROCm is importable, load it first so that the engine
    binds to the runtime torch uses (device buffers and streams are shared with
    torch tensors).  Loading the engine first would bring in /opt/rocm's runtime
    and torch's own beside it, and the first of them to initialise can leave
    the other without a device ("no ROCm-capable device is detected")."""
    if os.environ.get("UGPU_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def _load():
    _torch_runtime_first()
    if not os.path.exists(LIB_PATH):
        raise ImportError("libugrep_amd.so not built (%s); run __graft_entry__.build() or make -C ugrep_amd"
                          % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    V = ctypes.c_void_p
    P = ctypes.POINTER
    sig = {
        "ugpu_dfa_create": (ctypes.c_int, [c_u32p, ctypes.c_uint32, ctypes.c_uint32, P(V)]),
        "ugpu_dfa_destroy": (ctypes.c_int, [V]),
        "ugpu_dfa_info_get": (ctypes.c_int, [V, P(DfaInfo)]),
        "ugpu_dfa_plan_host": (ctypes.c_int, [c_u32p, ctypes.c_uint32, ctypes.c_uint32, P(DfaInfo)]),
        "ugpu_tables_build_host": (ctypes.c_int, [c_u32p, ctypes.c_uint32, P(DfaInfo), c_u16p, ctypes.c_uint32,
                                                  c_u8p, c_u32p, ctypes.c_uint32, c_u32p, c_u32p]),
        "ugpu_tables_prefilter_host": (ctypes.c_int, [c_u32p, ctypes.c_uint32, c_u8p, P(ctypes.c_int)]),
        "ugpu_tables_transducer_host": (ctypes.c_int, [c_u32p, ctypes.c_uint32, c_u16p, ctypes.c_uint32,
                                                       P(ctypes.c_int)]),
        "ugpu_tables_immediate_host": (ctypes.c_int, [c_u32p, ctypes.c_uint32, c_u8p, ctypes.c_uint32, c_u32p,
                                                      c_u8p, P(ctypes.c_int)]),
        "ugpu_tables_gap_host": (ctypes.c_int, [c_u32p, ctypes.c_uint32, c_u16p, ctypes.c_uint32, c_u8p,
                                                P(ctypes.c_int)]),
        "ugpu_tables_equivalent_host": (ctypes.c_int, [c_u32p, ctypes.c_uint32, c_u32p, ctypes.c_uint32,
                                                       P(ctypes.c_int)]),
        "ugpu_tables_context_host": (ctypes.c_int, [c_u32p, ctypes.c_uint32, c_u32p, ctypes.c_uint32,
                                                    P(ctypes.c_int), P(ctypes.c_int)]),
        "ugpu_scanner_context": (ctypes.c_int, [V, ctypes.c_int]),
        "ugpu_tables_xc_host": (ctypes.c_int, [c_u32p, ctypes.c_uint32, c_u8p, P(ctypes.c_int)]),
        "ugpu_tables_xu_host": (ctypes.c_int, [c_u32p, ctypes.c_uint32, c_u8p, c_u32p, P(ctypes.c_int)]),
        "ugpu_tables_dom_host": (ctypes.c_int, [c_u32p, ctypes.c_uint32, c_u32p, ctypes.c_uint32,
                                                P(ctypes.c_uint32), P(ctypes.c_int)]),
        "ugpu_find_all": (ctypes.c_int, [V, V, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, P(P(Result))]),
        "ugpu_find_all_multi": (ctypes.c_int, [V, V, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int,
                                               P(P(Result))]),
        "ugpu_result_free": (ctypes.c_int, [P(Result)]),
        "ugpu_scanner_create": (ctypes.c_int, [V, P(V)]),
        "ugpu_scanner_create_ex": (ctypes.c_int, [V, ctypes.c_uint32, P(V)]),
        "ugpu_scanner_destroy": (ctypes.c_int, [V]),
        "ugpu_scanner_stage": (ctypes.c_int, [V, ctypes.c_int]),
        "ugpu_scan": (ctypes.c_int, [V, V, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                     ctypes.c_uint64, V]),
        "ugpu_scan_totals": (ctypes.c_int, [V, P(Totals)]),
        "ugpu_scan_offsets": (ctypes.c_int, [V, V, V, V, ctypes.c_uint64, V]),
        "ugpu_chain_fix": (ctypes.c_int, [V, V, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                          ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, P(Totals), V]),
        "ugpu_scan_kernel_ms": (ctypes.c_int, [V, P(ctypes.c_float)]),
        "ugpu_gen": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, V, ctypes.c_uint64, V]),
        "ugpu_stream_create": (ctypes.c_int, [V, ctypes.c_uint64, P(V)]),
        "ugpu_stream_destroy": (ctypes.c_int, [V]),
        "ugpu_stream_feed": (ctypes.c_int, [V, V, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32, P(P(Result))]),
        "ugpu_stream_settled": (ctypes.c_uint64, [V]),
        "ugpu_stream_reserve": (ctypes.c_int, [V, ctypes.c_int, ctypes.c_uint64]),
        "ugpu_lines": (ctypes.c_int, [V, ctypes.c_uint64, V, ctypes.c_uint64, V, P(ctypes.c_uint64),
                                      P(ctypes.c_uint64), V]),
        "ugpu_check_utf8": (ctypes.c_int, [V, ctypes.c_uint64, P(ctypes.c_uint64), V]),
        "ugpu_find_nul": (ctypes.c_int, [V, ctypes.c_uint64, P(ctypes.c_uint64), V]),
        "ugpu_is_binary": (ctypes.c_int, [V, ctypes.c_uint64, ctypes.c_uint32, P(ctypes.c_int), V]),
        "ugpu_compile": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32, P(c_u32p),
                                        P(ctypes.c_uint32)]),
        "ugpu_opc_free": (None, [c_u32p]),
        "ugpu_compile_error": (ctypes.c_char_p, []),
        "ugpu_last_error": (ctypes.c_char_p, []),
        "ugpu_version": (ctypes.c_char_p, []),
        "ugpu_build_id": (ctypes.c_char_p, []),
        "ugpu_abi_version": (ctypes.c_int, []),
        "ugpu_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
        "ugpu_find_records": (ctypes.c_int, [V, V, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(V)]),
        "ugpu_find_records_ex": (ctypes.c_int, [V, V, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                                ctypes.POINTER(V)]),
        "ugpu_records_next": (ctypes.c_int, [V, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32),
                                             ctypes.POINTER(ctypes.c_uint32)]),
        "ugpu_records_totals": (ctypes.c_int, [V, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                               ctypes.POINTER(ctypes.c_uint64)]),
        "ugpu_records_free": (ctypes.c_int, [V]),
        "ugpu_records_drain": (ctypes.c_int, [V, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                              ctypes.POINTER(ctypes.c_uint64)]),
        "ugpu_select_device": (ctypes.c_int, [ctypes.c_int]),
        "ugpu_warmup": (ctypes.c_int, [ctypes.c_int]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()


def _source_hash():
    """tools/srchash.py's hash of the sources beside this package (None when
    they are not there, e.g. an installed copy)."""
    import hashlib
    repo = os.path.dirname(HERE)
    csrc = os.path.join(HERE, "csrc")
    hdr = os.path.join(repo, "include", "ugpu.h")
    if not os.path.isdir(csrc) or not os.path.exists(hdr):
        return None
    h = hashlib.sha256()
    files = sorted(os.path.join(csrc, f) for f in os.listdir(csrc)
                   if f.endswith((".hip", ".hpp", ".cpp", ".inc", ".h")))
    for f in files + [hdr]:
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_id():
    """(library build id, whether it matches the sources beside it): the id is
    "src:<hash> git:<commit>" (ugpu_build_id, ugrep_amd/Makefile)."""
    bid = lib.ugpu_build_id().decode()
    src = _source_hash()
    return bid, src is None or bid.startswith("src:%s " % src)


def _check_provenance():
    import warnings
    bid, ok = build_id()
    if not ok:
        warnings.warn("%s was not built from the sources beside it (%s, sources src:%s): rebuild with "
                      "make -C ugrep_amd" % (os.path.basename(LIB_PATH), bid, _source_hash()), RuntimeWarning)


if os.path.basename(LIB_PATH) == "libugrep_amd.so":  # (variant builds share the id of the default one)
    _check_provenance()


def check(rc):
    if rc != UGPU_OK:
        msg = lib.ugpu_last_error().decode(errors="replace")
        if rc == UGPU_UNSUPPORTED:
            raise Unsupported(rc, msg)
        raise UgpuError(rc, msg)
    return rc


def declared_symbols(header=HEADER):
    """Function names declared in include/ugpu.h."""
    import re
    txt = open(header).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(ugpu_\w+)\s*\(", txt, re.M)))
