"""Host-side mirror of the reference matcher interface for the FIND hot path.

    reflex::Pattern(const Opcode *code, ...)   include/reflex/pattern.h:151-159
    reflex::Matcher(pattern); m.buffer(base, size); while (m.find()) ...
        find  = AbstractMatcher::Operation, include/reflex/absmatcher.h:276-280, :1401
        first = absmatcher.h:901-905, size = :651-658, accept = :605-609

`Pattern` takes the compiled opcode words (Pattern::opc_) and uploads the dense
tables once; `Matcher` serves find() from one whole-buffer GPU scan, the way a
ugrep worker consumes matches from a mmap'd file (src/ugrep.cpp:3936-3940,
:10544).  Everything runs through the HIP engine (libugrep_amd.so); there is no
CPU fallback in this module: tables the engine does not support raise
`Unsupported`, as ugpu_dfa_create returns UGPU_UNSUPPORTED.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import BIN_INIT_WINDOW, BIN_NUL_ONLY, BIN_NULL_DATA, check, lib


def _as_u32(opc):
    a = np.ascontiguousarray(np.asarray(opc, dtype=np.uint32))
    return a, a.ctypes.data_as(_lib.c_u32p)


RX_FIXED = 1
RX_ICASE = 2
RX_REFLEX = 4
PAT_WORD = 1  # ugpu_dfa_create pattern_flags: option W
PAT_EMPTY = 2  # ugpu_dfa_create pattern_flags: option N (empty matches)


def compile_regex(regex, fixed=False, icase=False, reflex=False):
    """Opcode words (numpy u32) for `regex` from the native compiler
    (ugpu_compile, regex_compile.cpp): ugrep's default ERE in Unicode mode, as
    Matcher::convert(rx, notnewline|unicode) + Pattern(conv, "r") produce them
    (src/ugrep.cpp:8574-8578, lib/pattern.cpp:171-3063).  Syntax errors raise
    UgpuError(UGPU_INVAL) where the reference throws regex_error; constructs the
    GPU tables do not cover raise Unsupported.  reflex=True: `regex` is the
    RE/flex byte regex a Pattern holds after ugrep's conversion
    (Pattern::operator[](0), UGPU_RX_REFLEX), as the drop-in adapter passes it."""
    if isinstance(regex, str):
        regex = regex.encode("utf-8")
    words = _lib.c_u32p()
    n = ctypes.c_uint32()
    flags = (RX_FIXED if fixed else 0) | (RX_ICASE if icase else 0) | (RX_REFLEX if reflex else 0)
    rc = lib.ugpu_compile(regex, len(regex), flags, ctypes.byref(words), ctypes.byref(n))
    if rc != _lib.UGPU_OK:
        msg = lib.ugpu_compile_error().decode(errors="replace")
        raise (_lib.Unsupported if rc == _lib.UGPU_UNSUPPORTED else _lib.UgpuError)(rc, msg)
    try:
        return np.ctypeslib.as_array(words, shape=(n.value,)).copy()
    finally:
        lib.ugpu_opc_free(words)


def host_tables(opc):
    """Dense tables built on the host (no device needed): dict of numpy arrays."""
    a, p = _as_u32(opc)
    info = _lib.DfaInfo()
    check(lib.ugpu_tables_build_host(p, len(a), ctypes.byref(info), None, 0, None, None, 0, None, None))
    trans = np.zeros(info.states * info.row, np.uint16)
    cls = np.zeros(256, np.uint8)
    caps = np.zeros(info.states, np.uint32)
    start = ctypes.c_uint32()
    accb = ctypes.c_uint32()
    check(lib.ugpu_tables_build_host(p, len(a), ctypes.byref(info), trans.ctypes.data_as(_lib.c_u16p), len(trans),
                                     cls.ctypes.data_as(_lib.c_u8p), caps.ctypes.data_as(_lib.c_u32p), len(caps),
                                     ctypes.byref(start), ctypes.byref(accb)))
    return dict(info={f: getattr(info, f) for f, _ in _lib.DfaInfo._fields_}, trans=trans, cls=cls, caps=caps,
                start=start.value, accb=accb.value)


def host_context(opc):
    """(acap u32[states * 4], anchored, start_acc): the per-context accept
    indices acap[state * 4 + bol * 2 + eol] of the dense tables (tables.hpp)."""
    a, p = _as_u32(opc)
    info = _lib.DfaInfo()
    check(lib.ugpu_tables_build_host(p, len(a), ctypes.byref(info), None, 0, None, None, 0, None, None))
    acap = np.zeros(info.states * max(info.contexts, 4), np.uint32)
    an, sa = ctypes.c_int(), ctypes.c_int()
    check(lib.ugpu_tables_context_host(p, len(a), acap.ctypes.data_as(_lib.c_u32p), len(acap), ctypes.byref(an),
                                       ctypes.byref(sa)))
    return acap, bool(an.value), bool(sa.value)


def host_prefilter(opc):
    """(enabled, ft[20]) prefilter lookup tables built on the host (tables.hpp)."""
    a, p = _as_u32(opc)
    ft = np.zeros(20, np.uint8)
    en = ctypes.c_int()
    check(lib.ugpu_tables_prefilter_host(p, len(a), ft.ctypes.data_as(_lib.c_u8p), ctypes.byref(en)))
    return bool(en.value), ft


def host_plan(opc, word=False, empty=False):
    """The info dict Pattern(opc, word, empty).info() would report (kernel
    choice included), decided on the host without a device
    (ugpu_dfa_plan_host); raises like Pattern() for unsupported tables."""
    a, p = _as_u32(compile_regex(opc) if isinstance(opc, (str, bytes)) else opc)
    info = _lib.DfaInfo()
    check(lib.ugpu_dfa_plan_host(p, len(a), (PAT_WORD if word else 0) | (PAT_EMPTY if empty else 0),
                                 ctypes.byref(info)))
    return {f: getattr(info, f) for f, _ in _lib.DfaInfo._fields_}


def host_transducer(opc):
    """FIND transducer table (u16 numpy array, tables.hpp) or None when the DFA
    is not restart-local."""
    a, p = _as_u32(opc)
    t = host_tables(opc)
    x = np.zeros(t["info"]["states"] * t["info"]["row"], np.uint16)
    loc = ctypes.c_int()
    check(lib.ugpu_tables_transducer_host(p, len(a), x.ctypes.data_as(_lib.c_u16p), len(x), ctypes.byref(loc)))
    return x if loc.value else None


def host_immediate(opc):
    """Immediate transducer of xi_kernel: (xid table as uint8[rows, 256], sync byte) or None."""
    a, p = _as_u32(opc)
    rows, sb, imm = ctypes.c_uint32(), ctypes.c_uint8(), ctypes.c_int()
    check(lib.ugpu_tables_immediate_host(p, len(a), None, 0, ctypes.byref(rows), ctypes.byref(sb), ctypes.byref(imm)))
    if not imm.value:
        return None
    x = np.zeros(rows.value * 256, np.uint8)
    check(lib.ugpu_tables_immediate_host(p, len(a), x.ctypes.data_as(_lib.c_u8p), x.size, ctypes.byref(rows),
                                         ctypes.byref(sb), ctypes.byref(imm)))
    return x.reshape(rows.value, 256), sb.value


def host_gap(opc):
    """Gap transducer of xg_kernel: (xg table uint16[states*row], sync uint8[256]) or None."""
    a, p = _as_u32(opc)
    info = host_tables(opc)["info"]
    x = np.zeros(info["states"] * info["row"], np.uint16)
    sy = np.zeros(256, np.uint8)
    ok = ctypes.c_int()
    check(lib.ugpu_tables_gap_host(p, len(a), x.ctypes.data_as(_lib.c_u16p), x.size, sy.ctypes.data_as(_lib.c_u8p),
                                   ctypes.byref(ok)))
    return (x, sy) if ok.value else None


def host_equivalent(opc_a, opc_b):
    """True when two opcode tables accept the same strings with the same accept indices."""
    a, pa = _as_u32(opc_a)
    b, pb = _as_u32(opc_b)
    eq = ctypes.c_int(0)
    check(lib.ugpu_tables_equivalent_host(pa, len(a), pb, len(b), ctypes.byref(eq)))
    return bool(eq.value)


def host_xc(opc):
    """Byte classes of xc_kernel (two-state tables): cls uint8[256] = G << 7 | X << 6, or None."""
    a, p = _as_u32(opc)
    ok = ctypes.c_int(0)
    cls = np.zeros(256, np.uint8)
    check(lib.ugpu_tables_xc_host(p, len(a), cls.ctypes.data_as(_lib.c_u8p), ctypes.byref(ok)))
    return cls if ok.value else None


def host_xu(opc):
    """Code-point run tables of xc_kernel's U mode: (tab uint8[16896], bm3 uint32[2048]), or None."""
    a, p = _as_u32(opc)
    ok = ctypes.c_int(0)
    tab = np.zeros(256 + 64 * 256 + 256, np.uint8)  # (tables.hpp kXuTab)
    bm3 = np.zeros(2048, np.uint32)
    check(lib.ugpu_tables_xu_host(p, len(a), tab.ctypes.data_as(_lib.c_u8p), bm3.ctypes.data_as(_lib.c_u32p),
                                  ctypes.byref(ok)))
    return (tab, bm3) if ok.value else None


def host_dom(opc, want_all=False):
    """Dominated-restart bits of the dense tables (tables.hpp dom): a bool
    numpy array over state ids (ugpu_tables_build_host numbering), or None
    when they were not computed; want_all: (bits, dom_all)."""
    a, p = _as_u32(opc)
    n = ctypes.c_uint32(0)
    al = ctypes.c_int(0)
    check(lib.ugpu_tables_dom_host(p, len(a), None, 0, ctypes.byref(n), ctypes.byref(al)))
    bits = None
    if n.value:
        w = np.zeros(n.value, np.uint32)
        check(lib.ugpu_tables_dom_host(p, len(a), w.ctypes.data_as(_lib.c_u32p), n.value, ctypes.byref(n), None))
        bits = np.unpackbits(w.view(np.uint8), bitorder="little").astype(bool)
    return (bits, bool(al.value)) if want_all else bits


class Pattern:
    """Compiled pattern (opcode words) with its device tables."""

    def __init__(self, opc, word=False, empty=False):
        """opc: opcode words (or a regex for compile_regex).  word=True is
        Matcher option W (ugrep -w, reflex::Matcher(pat, input, "W"),
        src/ugrep.cpp:8616-8618): whole-buffer scans on wfind_kernel.
        empty=True is option N (ugrep -Y, -x): empty matches are reported."""
        if isinstance(opc, (str, bytes)):
            opc = compile_regex(opc)
        self.opc, p = _as_u32(opc)
        self.word = bool(word)
        self.empty = bool(empty)
        h = ctypes.c_void_p()
        check(lib.ugpu_dfa_create(p, len(self.opc), (PAT_WORD if word else 0) | (PAT_EMPTY if empty else 0),
                                  ctypes.byref(h)))
        self._h = h

    @property
    def handle(self):
        return self._h

    def info(self):
        info = _lib.DfaInfo()
        check(lib.ugpu_dfa_info_get(self._h, ctypes.byref(info)))
        return {f: getattr(info, f) for f, _ in _lib.DfaInfo._fields_}

    def close(self):
        if getattr(self, "_h", None):
            lib.ugpu_dfa_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _buffer_ptr(data):
    """(pointer, length, keepalive) of bytes / numpy / torch (host or device) data."""
    if isinstance(data, (bytes, bytearray, memoryview)):
        arr = np.frombuffer(bytes(data), dtype=np.uint8)
        return arr.ctypes.data, arr.size, arr
    if isinstance(data, np.ndarray):
        arr = np.ascontiguousarray(data.view(np.uint8).reshape(-1))
        return arr.ctypes.data, arr.size, arr
    if hasattr(data, "data_ptr"):  # torch tensor, host or device
        t = data.contiguous()
        return t.data_ptr(), t.numel() * t.element_size(), t
    raise TypeError("unsupported buffer type %r" % type(data))


class FindResult:
    def __init__(self, count, digest, dcap, start=None, length=None, cap=None):
        self.count, self.digest, self.dcap = count, digest, dcap
        self.start, self.length, self.cap = start, length, cap

    def triples(self):
        return [[int(s), int(l), int(c)] for s, l, c in zip(self.start, self.length, self.cap)]


def _take_result(res, offsets):
    try:
        r = res.contents
        if offsets and r.count:
            st = np.ctypeslib.as_array(r.start, shape=(r.count,)).copy()
            ln = np.ctypeslib.as_array(r.len, shape=(r.count,)).copy()
            cp = np.ctypeslib.as_array(r.cap, shape=(r.count,)).copy()
        else:
            st = np.zeros(0, np.uint64)
            ln = np.zeros(0, np.uint32)
            cp = np.zeros(0, np.uint32)
        return FindResult(r.count, r.digest, r.dcap, st, ln, cp)
    finally:
        lib.ugpu_result_free(res)


def find_all(pattern, data, start=0, offsets=True):
    """ugpu_find_all: every FIND match of `data` from position `start`."""
    ptr, n, keep = _buffer_ptr(data)
    res = ctypes.POINTER(_lib.Result)()
    check(lib.ugpu_find_all(pattern.handle, ctypes.c_void_p(ptr), n, start,
                            _lib.MODE_OFFSETS if offsets else _lib.MODE_COUNT, ctypes.byref(res)))
    out = _take_result(res, offsets)
    del keep
    return out


def find_all_multi(pattern, data, ndev=0, start=0, offsets=True):
    """ugpu_find_all_multi: as find_all, with [start, len) cut into ndev shards
    at arbitrary offsets, shard k on device k mod the visible devices (ndev 0:
    one per device), chains resolved across the cuts."""
    ptr, n, keep = _buffer_ptr(data)
    res = ctypes.POINTER(_lib.Result)()
    check(lib.ugpu_find_all_multi(pattern.handle, ctypes.c_void_p(ptr), n, start,
                                  _lib.MODE_OFFSETS if offsets else _lib.MODE_COUNT, ndev, ctypes.byref(res)))
    out = _take_result(res, offsets)
    del keep
    return out


class Records:
    """ugpu_find_records: the records of a buffer for a one-at-a-time consumer
    (pipelined H2D, scans and packed record copy-back; include/ugpu.h)."""

    def __init__(self, pattern, data, start=0, borrow=False):
        """borrow=True (UGPU_REC_BORROW): this object keeps `data` alive until
        close(), and the first records can be popped while the rest of the
        input is still on its way to the device."""
        ptr, n, keep = _buffer_ptr(data)
        h = ctypes.c_void_p()
        if borrow:
            check(lib.ugpu_find_records_ex(pattern.handle, ctypes.c_void_p(ptr), n, start, 1, ctypes.byref(h)))
            self._keep = (keep, data)
        else:
            check(lib.ugpu_find_records(pattern.handle, ctypes.c_void_p(ptr), n, start, ctypes.byref(h)))
            del keep
        self._h = h

    def next(self):
        """(start, len, cap) of the next record, or None."""
        s, ln, c = ctypes.c_uint64(), ctypes.c_uint32(), ctypes.c_uint32()
        rc = lib.ugpu_records_next(self._h, ctypes.byref(s), ctypes.byref(ln), ctypes.byref(c))
        if rc < 0:
            check(-rc)
        return (s.value, ln.value, c.value) if rc == 1 else None

    def triples(self):
        out = []
        while True:
            t = self.next()
            if t is None:
                return out
            out.append(list(t))

    def totals(self):
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        check(lib.ugpu_records_totals(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value

    def drain(self):
        """Pop every remaining record natively: (n, digest, dcap)."""
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        check(lib.ugpu_records_drain(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value

    def close(self):
        if getattr(self, "_h", None):
            lib.ugpu_records_free(self._h)
            self._h = None
        self._keep = None  # (a borrowed buffer outlives the pipeline)

    def __del__(self):
        self.close()


class Stream:
    """Streaming FIND over input fed in chunks (ugpu_stream):
    feed() returns the matches that became final, with absolute offsets."""

    def __init__(self, pattern, keep=0):
        self.pattern = pattern
        h = ctypes.c_void_p()
        check(lib.ugpu_stream_create(pattern.handle, keep, ctypes.byref(h)))
        self._h = h

    def feed(self, chunk, final=False, offsets=True, flush=False):
        """final: the input ends here; flush: more may follow, but settle every
        match the bytes so far decide (UGPU_FEED_FLUSH: an input that would block)."""
        ptr, n, keep = _buffer_ptr(chunk)
        res = ctypes.POINTER(_lib.Result)()
        check(lib.ugpu_stream_feed(self._h, ctypes.c_void_p(ptr), n, 1 if final else (2 if flush else 0),
                                   _lib.MODE_OFFSETS if offsets else _lib.MODE_COUNT, ctypes.byref(res)))
        out = _take_result(res, offsets)
        del keep
        return out

    def settled(self):
        return lib.ugpu_stream_settled(self._h)

    def close(self):
        if getattr(self, "_h", None):
            lib.ugpu_stream_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Matcher:
    """FIND over a fully buffered input: m = Matcher(pat, data); while m.find(): m.first(), m.size()."""

    def __init__(self, pattern, data=None):
        self.pattern = pattern
        self._data = None
        if data is not None:
            self.buffer(data)

    def buffer(self, data):
        """AbstractMatcher::buffer(base, size): whole input, cursor at 0 (absmatcher.h:542-591)."""
        self._data = data
        self._cur = 0
        self._from = 0
        self._res = None
        self._i = 0
        self._first = 0
        self._size = 0
        self._cap = 0
        return self

    def _inside_match(self):
        """The cursor lies strictly inside a record of the current scan."""
        r, i = self._res, max(self._i - 1, 0)
        while i < r.count and int(r.start[i]) + int(r.length[i]) <= self._cur:
            i += 1
        return i < r.count and int(r.start[i]) < self._cur

    def find(self):
        """Next match at or after the cursor; returns its accept index, 0 when exhausted.

        The FIND chain passes through every position that is not strictly
        inside one of its matches, so after skip_to() the remaining records
        stay exact unless the cursor landed inside a match; then (as the C++
        adapter, integration/reflex_gpu_matcher.h) the scan is re-run from the
        cursor."""
        if self._res is None or self._cur < self._from or self._inside_match():
            self._res = find_all(self.pattern, self._data, self._cur, offsets=True)
            self._from = self._cur
            self._i = 0
        r = self._res
        while self._i < r.count and int(r.start[self._i]) < self._cur:
            self._i += 1
        if self._i >= r.count:
            self._cap = 0
            self._size = 0
            return 0
        self._first = int(r.start[self._i])
        self._size = int(r.length[self._i])
        self._cap = int(r.cap[self._i])
        self._cur = self._first + self._size
        self._i += 1
        return self._cap

    def first(self):
        return self._first

    def size(self):
        return self._size

    def last(self):
        return self._first + self._size

    def accept(self):
        return self._cap

    def skip_to(self, pos):
        """Advance the cursor (the effect of skip('\\n') on cur_ between finds)."""
        self._cur = max(self._cur, pos)

    def __iter__(self):
        while self.find():
            yield self._first, self._size, self._cap


class Scanner:
    """Device-resident scans (ugpu_scanner): one per stream/thread."""

    def __init__(self, pattern, records=False):
        """records=True: scans will be followed by offsets() -- prefer kernels
        with their own record pass (UGPU_SCANNER_RECORDS)."""
        self.pattern = pattern
        h = ctypes.c_void_p()
        check(lib.ugpu_scanner_create_ex(pattern.handle, 1 if records else 0, ctypes.byref(h)))
        self._h = h

    def scan(self, dptr, lo, hi, read_end=None, at_eof=True, bias=0, stream=0):
        if read_end is None:
            read_end = hi
        check(lib.ugpu_scan(self._h, ctypes.c_void_p(dptr), lo, hi, read_end, 1 if at_eof else 0, bias,
                            ctypes.c_void_p(stream)))

    def totals(self):
        t = _lib.Totals()
        check(lib.ugpu_scan_totals(self._h, ctypes.byref(t)))
        return t

    def context(self, bol0):
        """ugpu_scanner_context: whether dbuf[0] begins a line (anchored tables)."""
        check(lib.ugpu_scanner_context(self._h, 1 if bol0 else 0))

    def stage(self, on=True):
        """Single-pass OFFSETS: COUNT scans stage the records of prefiltered tables."""
        check(lib.ugpu_scanner_stage(self._h, 1 if on else 0))

    def kernel_ms(self):
        ms = ctypes.c_float()
        check(lib.ugpu_scan_kernel_ms(self._h, ctypes.byref(ms)))
        return ms.value

    def offsets(self, d_start, d_len, d_cap, capacity, stream=0):
        """Write the last scan's records; d_cap 0/None: 12-byte records (tables
        with one accept index, info()["shape"] & SHAPE_ONE_ACCEPT)."""
        check(lib.ugpu_scan_offsets(self._h, ctypes.c_void_p(d_start), ctypes.c_void_p(d_len),
                                    ctypes.c_void_p(d_cap or None), capacity, ctypes.c_void_p(stream)))

    def chain_fix(self, dptr, lo, hi, read_end, at_eof, bias, old_entry, new_entry, stream=0):
        t = _lib.Totals()
        check(lib.ugpu_chain_fix(self._h, ctypes.c_void_p(dptr), lo, hi, read_end, 1 if at_eof else 0, bias,
                                 old_entry, new_entry, ctypes.byref(t), ctypes.c_void_p(stream)))
        return t

    def close(self):
        if getattr(self, "_h", None):
            lib.ugpu_scanner_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def lines(dptr, length, d_start=0, n=0, d_line=0, stream=0):
    """ugpu_lines over a 16-byte aligned device buffer: (newlines, matching_lines);
    fills d_line[i] with the 1-based line of d_start[i] when d_line is given."""
    nl = ctypes.c_uint64()
    ml = ctypes.c_uint64()
    check(lib.ugpu_lines(ctypes.c_void_p(dptr), length, ctypes.c_void_p(d_start), n, ctypes.c_void_p(d_line),
                         ctypes.byref(nl), ctypes.byref(ml), ctypes.c_void_p(stream)))
    return nl.value, ml.value


def check_utf8(dptr, length, stream=0):
    """reflex::isutf8 over device bytes (ugpu_check_utf8): None when valid,
    else the offset of the first failing byte (length for a cut-off sequence)."""
    r = ctypes.c_uint64()
    check(lib.ugpu_check_utf8(ctypes.c_void_p(dptr), length, ctypes.byref(r), ctypes.c_void_p(stream)))
    return None if r.value == 0xFFFFFFFFFFFFFFFF else r.value


def isutf8(dptr, length, stream=0):
    """reflex::isutf8(s, s + length) (lib/simd.cpp:169) on a device buffer."""
    return check_utf8(dptr, length, stream) is None


def find_nul(dptr, length, stream=0):
    """memchr(s, '\\0', length) on a device buffer: offset or None."""
    r = ctypes.c_uint64()
    check(lib.ugpu_find_nul(ctypes.c_void_p(dptr), length, ctypes.byref(r), ctypes.c_void_p(stream)))
    return None if r.value == 0xFFFFFFFFFFFFFFFF else r.value


def is_binary(dptr, length, null_data=False, nul_only=False, init_window=False, stream=0):
    """ugrep's is_binary (src/ugrep.cpp:699-711); init_window adds
    init_is_binary's trailing-sequence trim (:3998-4015)."""
    flags = (BIN_NULL_DATA if null_data else 0) | (BIN_NUL_ONLY if nul_only else 0) | \
        (BIN_INIT_WINDOW if init_window else 0)
    r = ctypes.c_int()
    check(lib.ugpu_is_binary(ctypes.c_void_p(dptr), length, flags, ctypes.byref(r), ctypes.c_void_p(stream)))
    return bool(r.value)


def gen(kind, seed, off, dptr, length, stream=0):
    """Generate corpus bytes [off, off+length) on the device (ugpu_gen)."""
    check(lib.ugpu_gen(kind, seed, off, ctypes.c_void_p(dptr), length, ctypes.c_void_p(stream)))
