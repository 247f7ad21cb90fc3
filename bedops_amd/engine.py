"""ctypes binding of libbedgpu (include/bedgpu.h) — the Python side of the C ABI.

Mirrors the reference front-ends' operations (applications/bed/bedops/src/Input.hpp
modes, applications/bed/bedmap/src/Input.hpp visitors). Errors raise BedgpuError with
the library's message; nothing here computes intervals on the CPU.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

BED3, BED3_REST, BED5, BED3_SET, BED5_REST = 0, 1, 2, 3, 4
# operations that read only each input's merged set (or, for element-of, only the
# non-reference inputs' sets): their inputs may be loaded as BED3_SET
SET_MODES = {"-m", "--merge", "-i", "--intersect", "-d", "--difference", "-e", "--element-of",
             "-n", "--not-element-of", "-c", "--complement", "-w", "--chop", "-s", "--symmdiff"}
MAP_COUNT, MAP_MEAN = 1, 2
# bedmap operations and overlap criteria (include/bedgpu.h BG_MAP_* / BG_OVR_*)
MAP_OPS = {"count": 1, "mean": 2, "sum": 3, "min": 4, "max": 5, "indicator": 6, "bases": 7,
           "bases-uniq": 8, "bases-uniq-f": 9, "echo": 10, "echo-ref-size": 11,
           "echo-ref-name": 12, "echo-map": 13, "echo-map-id": 14, "echo-map-score": 15,
           "echo-map-size": 16, "echo-overlap-size": 17, "echo-map-range": 18, "median": 19,
           "kth": 20, "variance": 21, "stdev": 22, "cv": 23, "echo-map-id-uniq": 25, "mad": 24,
           "echo-ref-row-id": 26, "min-element": 27, "max-element": 28, "min-element-rand": 29,
           "max-element-rand": 30, "tmean": 31, "wmean": 32}
SCORE_OPS = ("mean", "sum", "min", "max", "echo-map-score", "median", "kth", "variance", "stdev",
             "cv", "mad", "min-element", "max-element", "min-element-rand", "max-element-rand",
             "tmean", "wmean")
# the map rows' remainders are printed, or order equal rows for the running-double
# operations (CoordRestAddressCompare: id + remainder)
MAP_REST_OPS = ("echo-map", "echo-map-id", "echo-map-id-uniq", "mean", "sum", "variance", "stdev",
                "cv", "min-element", "max-element", "min-element-rand", "max-element-rand", "tmean")
# operations that can see the reference's heap-address order of equal rows (bedmap.c addr_ops)
ADDR_OPS = ("wmean", "tmean", "echo-map", "echo-map-id", "echo-map-score", "echo-map-size",
            "echo-overlap-size", "min-element", "max-element", "min-element-rand", "max-element-rand")
OVR_CRITERIA = {"bp-ovr": 0, "range": 1, "fraction-ref": 2, "fraction-map": 3,
                "fraction-either": 4, "fraction-both": 5, "exact": 6}

ERRORS = {-11: "INTERNAL", -1: "HIP", -2: "PARSE", -3: "UNSORTED", -4: "RANGE", -5: "BLANK", -6: "ARG",
          -7: "NOMEM", -8: "UNSUPPORTED", -9: "CHROM", -10: "IO", -12: "VISITOR"}
BG_E_VISITOR = -12

# exported symbols of include/bedgpu.h (checked by tests/test_abi.py)
SYMBOLS = ["bg_open", "bg_close", "bg_last_error", "bg_sync", "bg_stream", "bg_build_hash", "bg_load",
           "bg_set_rows", "bg_set_restrict_chrom", "bg_set_free", "bg_merge", "bg_intersect",
           "bg_difference", "bg_element_of", "bg_map", "bg_result_rows", "bg_result_format",
           "bg_result_text_device", "bg_result_copy_text", "bg_result_write", "bg_result_free",
           "bg_stats", "bg_host_alloc", "bg_host_free", "bg_prof_enable", "bg_prof_read",
           "bg_result_copy_text_device", "bg_result_chrom_spans", "bg_set_chroms",
           "bg_set_chrom_name", "bg_closest", "bg_complement", "bg_chop", "bg_partition",
           "bg_symmdiff", "bg_everything", "bg_set_pad", "bg_check", "bg_check_message",
           "bg_write_device", "bg_writer_open", "bg_writer_push", "bg_writer_done", "bg_writer_close", "bg_bind", "bg_group_uid", "bg_group_open", "bg_group_open_rank",
           "bg_group_size", "bg_group_ctx", "bg_group_close", "bg_group_gather", "bg_device_free",
           "bg_device_gather_host", "bg_read_file_device", "bg_sortbed", "bg_starch_is",
           "bg_starch_decode", "bg_file_image_open", "bg_file_image_register", "bg_file_image_to_device",
           "bg_file_image_close", "bg_pwrite_device", "bg_device_release", "bg_set_output_skip", "bg_output_skip_left",
           "bg_device_alloc", "bg_file_image_copy", "bg_copy_order", "bg_copy_fence"]
UID_BYTES = 128


class _CheckResult(ctypes.Structure):
    _fields_ = [("row", ctypes.c_uint64), ("code", ctypes.c_int), ("line_off", ctypes.c_uint64),
                ("line_len", ctypes.c_uint64), ("prev_off", ctypes.c_uint64),
                ("prev_len", ctypes.c_uint64)]


def lib_path():
    # BEDGPU_LIB: an alternative build of the same library (A/B experiments)
    return os.environ.get("BEDGPU_LIB") or os.path.join(HERE, "lib", "libbedgpu.so")


class BedgpuError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"bedgpu {ERRORS.get(code, code)}: {msg}")
        self.code = code
        self.msg = msg


class BedgpuStop(BedgpuError):
    """BG_E_VISITOR: the reference throws mid-output; `text` is what it printed before."""

    def __init__(self, code, msg, text):
        super().__init__(code, msg)
        self.text = text


class _Input(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("nbytes", ctypes.c_uint64),
                ("on_device", ctypes.c_int), ("kind", ctypes.c_int)]


class _MapOpts(ctypes.Structure):
    _fields_ = [("overlap_bp", ctypes.c_uint64), ("n_ops", ctypes.c_int),
                ("ops", ctypes.c_int * 16), ("precision", ctypes.c_int),
                ("scientific", ctypes.c_int), ("skip_unmapped", ctypes.c_int),
                ("delim", ctypes.c_char * 16), ("criterion", ctypes.c_int),
                ("range_bp", ctypes.c_uint64), ("fraction", ctypes.c_double),
                ("multidelim", ctypes.c_char * 16), ("op_arg", ctypes.c_double * 16),
                ("op_arg2", ctypes.c_double * 16), ("shard", ctypes.c_int),
                ("faster", ctypes.c_int)]


class _ClosestOpts(ctypes.Structure):
    _fields_ = [("shortest", ctypes.c_int), ("print_dist", ctypes.c_int),
                ("no_ref", ctypes.c_int), ("no_overlaps", ctypes.c_int),
                ("delim", ctypes.c_char * 16)]


_LIB = None


def load_library():
    """Load libbedgpu.so (fails loudly: there is no fallback path)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    p = lib_path()
    if not os.path.exists(p):
        raise BedgpuError(-6, f"{p} not built (run `make lib` or __graft_entry__.build())")
    L = ctypes.CDLL(p)
    vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
    L.bg_starch_is.argtypes = [vp, u64]
    L.bg_starch_decode.argtypes = [vp, u64, ctypes.c_char_p, ctypes.POINTER(vp), ctypes.POINTER(u64),
                                   ctypes.c_char_p, u64]
    L.bg_open.argtypes = [ctypes.POINTER(vp), i32]
    L.bg_close.argtypes = [vp]
    L.bg_close.restype = None
    L.bg_last_error.argtypes = [vp]
    L.bg_last_error.restype = ctypes.c_char_p
    L.bg_sync.argtypes = [vp]
    L.bg_stream.argtypes = [vp]
    L.bg_stream.restype = vp
    L.bg_load.argtypes = [vp, i32, ctypes.POINTER(_Input), ctypes.POINTER(vp)]
    L.bg_set_rows.argtypes = [vp, i32, ctypes.POINTER(u64)]
    L.bg_set_restrict_chrom.argtypes = [vp, vp, ctypes.c_char_p]
    L.bg_set_free.argtypes = [vp]
    L.bg_set_free.restype = None
    L.bg_merge.argtypes = [vp, vp, ctypes.POINTER(i32), i32, ctypes.POINTER(vp)]
    L.bg_intersect.argtypes = [vp, vp, ctypes.POINTER(i32), i32, ctypes.POINTER(vp)]
    L.bg_difference.argtypes = [vp, vp, i32, ctypes.POINTER(i32), i32, ctypes.POINTER(vp)]
    L.bg_element_of.argtypes = [vp, vp, i32, ctypes.POINTER(i32), i32, ctypes.c_double, i32,
                                i32, ctypes.POINTER(vp)]
    L.bg_complement.argtypes = [vp, vp, ctypes.POINTER(i32), i32, i32, ctypes.POINTER(vp)]
    L.bg_chop.argtypes = [vp, vp, ctypes.POINTER(i32), i32, u64, u64, i32, ctypes.POINTER(vp)]
    for fn in (L.bg_partition, L.bg_symmdiff, L.bg_everything):
        fn.argtypes = [vp, vp, ctypes.POINTER(i32), i32, ctypes.POINTER(vp)]
    L.bg_set_pad.argtypes = [vp, vp, i32, i32, i32]
    L.bg_check.argtypes = [vp, vp, i32, i32, vp]
    L.bg_check_message.argtypes = [ctypes.c_char_p, u64, i32, i32, i32, ctypes.c_char_p, u64]
    L.bg_map.argtypes = [vp, vp, i32, i32, ctypes.POINTER(_MapOpts), ctypes.POINTER(vp)]
    L.bg_closest.argtypes = [vp, vp, i32, i32, ctypes.POINTER(_ClosestOpts), ctypes.POINTER(vp)]
    L.bg_result_rows.argtypes = [vp, ctypes.POINTER(u64)]
    L.bg_result_format.argtypes = [vp, vp, ctypes.POINTER(u64)]
    L.bg_result_text_device.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(u64)]
    L.bg_result_copy_text.argtypes = [vp, vp, ctypes.c_char_p, u64]
    L.bg_result_write.argtypes = [vp, vp, i32]
    L.bg_result_free.argtypes = [vp]
    L.bg_result_free.restype = None
    L.bg_stats.argtypes = [vp, ctypes.c_char_p, u64]
    L.bg_host_alloc.argtypes = [u64]
    L.bg_host_alloc.restype = vp
    L.bg_host_free.argtypes = [vp]
    L.bg_host_free.restype = None
    L.bg_prof_enable.argtypes = [vp, ctypes.c_char_p]
    L.bg_prof_read.argtypes = [vp, ctypes.c_char_p, u64]
    L.bg_result_copy_text_device.argtypes = [vp, vp, vp, u64]
    L.bg_result_chrom_spans.argtypes = [vp, vp, ctypes.POINTER(u64), ctypes.c_uint32]
    L.bg_set_chroms.argtypes = [vp, ctypes.POINTER(ctypes.c_uint32)]
    L.bg_set_chrom_name.argtypes = [vp, ctypes.c_uint32]
    L.bg_set_chrom_name.restype = ctypes.c_char_p
    L.bg_write_device.argtypes = [vp, vp, u64, i32]
    L.bg_bind.argtypes = [vp]
    L.bg_group_uid.argtypes = [vp]
    L.bg_group_open.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(i32), i32]
    L.bg_group_open_rank.argtypes = [ctypes.POINTER(vp), i32, vp, i32, i32]
    L.bg_group_size.argtypes = [vp, ctypes.POINTER(i32), ctypes.POINTER(i32), ctypes.POINTER(i32)]
    L.bg_group_ctx.argtypes = [vp, i32]
    L.bg_group_ctx.restype = vp
    L.bg_group_close.argtypes = [vp]
    L.bg_group_close.restype = None
    L.bg_group_gather.argtypes = [vp, i32, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp),
                                  ctypes.POINTER(vp), ctypes.POINTER(u64)]
    L.bg_device_free.argtypes = [vp, vp]
    L.bg_device_free.restype = None
    L.bg_device_gather_host.argtypes = [vp, i32, ctypes.POINTER(vp), ctypes.POINTER(u64),
                                        ctypes.POINTER(vp), ctypes.POINTER(u64)]
    _LIB = L
    return L


def parse_overlap_spec(spec):
    """-e/-n argument -> (threshold, use_percent) (Input.hpp:344-382)."""
    if spec is None:
        return 1.0, 1
    s = str(spec)
    if s.endswith("%"):
        v = s[:-1].lstrip("-")
        d = float(v) / 100.0
        if d > 1:
            raise BedgpuError(-6, "Expect percentage less than or equal to 100%")
        return (1.0, 0) if d == 0 else (d, 1)
    return float(int(s.lstrip("-"))), 0


def starch_to_bed(data, chrom=None):
    """A Starch archive's bytes -> the BED text the reference's reader yields (host decode,
    bg_starch_decode); bytes that are not a Starch archive are returned unchanged."""
    L = load_library()
    data = bytes(data)
    if not L.bg_starch_is(data, len(data)):
        return data
    out, n, err = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.create_string_buffer(512)
    rc = L.bg_starch_decode(data, len(data), chrom.encode() if chrom else None, ctypes.byref(out),
                            ctypes.byref(n), err, 512)
    if rc:
        raise BedgpuError(rc, err.value.decode(errors="replace"))
    try:
        return ctypes.string_at(out, n.value)
    finally:
        ctypes.CDLL(None).free(out)


class Result:
    def __init__(self, eng, handle):
        self.eng, self.h = eng, handle

    def rows(self):
        n = ctypes.c_uint64()
        self.eng._check(self.eng.L.bg_result_rows(self.h, ctypes.byref(n)))
        return n.value

    def format(self):
        n = ctypes.c_uint64()
        self.eng._check(self.eng.L.bg_result_format(self.eng.ctx, self.h, ctypes.byref(n)))
        return n.value

    def device_text(self):
        """(device pointer, nbytes) of the rendered text (formats first)."""
        self.format()
        p, n = ctypes.c_void_p(), ctypes.c_uint64()
        self.eng._check(self.eng.L.bg_result_text_device(self.h, ctypes.byref(p), ctypes.byref(n)))
        return p.value, n.value

    def copy_to_device(self, dst_ptr, cap):
        self.eng._check(self.eng.L.bg_result_copy_text_device(self.eng.ctx, self.h, dst_ptr, cap))

    def chrom_spans(self, nchroms):
        """byte offset of each chromosome's first line (+ total) in the rendered text"""
        arr = (ctypes.c_uint64 * (nchroms + 1))()
        self.eng._check(self.eng.L.bg_result_chrom_spans(self.eng.ctx, self.h, arr, nchroms + 1))
        return list(arr)

    def text(self):
        """the rendered text; raises BedgpuStop (carrying the text before the stop) where the
        reference throws mid-output"""
        n = ctypes.c_uint64()
        rc = self.eng.L.bg_result_format(self.eng.ctx, self.h, ctypes.byref(n))
        if rc and rc != BG_E_VISITOR:
            self.eng._check(rc)
        n = n.value
        buf = ctypes.create_string_buffer(max(n, 1))
        rc2 = self.eng.L.bg_result_copy_text(self.eng.ctx, self.h, buf, n)
        if rc2 and rc2 != BG_E_VISITOR:
            self.eng._check(rc2)
        if rc == BG_E_VISITOR:
            raise BedgpuStop(rc, self.eng.L.bg_last_error(self.eng.ctx).decode(errors="replace"),
                             buf.raw[:n])
        return buf.raw[:n]

    def free(self):
        if self.h:
            self.eng.L.bg_result_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class InputSet:
    def __init__(self, eng, handle, keep):
        self.eng, self.h, self._keep = eng, handle, keep

    def rows(self, i):
        n = ctypes.c_uint64()
        self.eng._check(self.eng.L.bg_set_rows(self.h, i, ctypes.byref(n)))
        return n.value

    def chroms(self):
        n = ctypes.c_uint32()
        self.eng._check(self.eng.L.bg_set_chroms(self.h, ctypes.byref(n)))
        return [self.eng.L.bg_set_chrom_name(self.h, g).decode() for g in range(n.value)]

    def restrict_chrom(self, chrom):
        self.eng._check(self.eng.L.bg_set_restrict_chrom(self.eng.ctx, self.h, chrom.encode()))

    def pad(self, i, lpad, rpad):
        """--range lpad:rpad applied to file i (BedPadReader.hpp:71-284)"""
        self.eng._check(self.eng.L.bg_set_pad(self.eng.ctx, self.h, i, int(lpad), int(rpad)))

    def free(self):
        if self.h:
            self.eng.L.bg_set_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Engine:
    """One libbedgpu context (one device, one HIP stream)."""

    def __init__(self, device=0, ctx=None):
        self.L = load_library()
        self._owns = ctx is None
        if ctx is not None:  # a member of a Group (the group owns the context)
            self.ctx = ctypes.c_void_p(ctx)
            return
        self.ctx = ctypes.c_void_p()
        rc = self.L.bg_open(ctypes.byref(self.ctx), int(device))
        if rc:
            raise BedgpuError(rc, "bg_open failed (no usable GPU?)")

    def _check(self, rc):
        if rc:
            raise BedgpuError(rc, self.L.bg_last_error(self.ctx).decode(errors="replace"))

    def close(self):
        if self.ctx and self._owns:
            self.L.bg_close(self.ctx)
        self.ctx = None

    def write_device(self, dptr, nbytes, fd):
        self._check(self.L.bg_write_device(self.ctx, ctypes.c_void_p(dptr), nbytes, fd))

    def device_free(self, dptr):
        self.L.bg_device_free(self.ctx, ctypes.c_void_p(dptr))

    def stream(self):
        return self.L.bg_stream(self.ctx)

    def sync(self):
        self._check(self.L.bg_sync(self.ctx))

    # -------------------------------------------------------------- loading
    def load(self, inputs):
        """inputs: list of (data, kind) where data is bytes (host), (devptr, nbytes), or
        (hostptr, nbytes, False): host memory the caller keeps alive until load returns."""
        n = len(inputs)
        arr = (_Input * n)()
        keep = []
        for i, (data, kind) in enumerate(inputs):
            if isinstance(data, tuple):
                dev = 1 if len(data) < 3 or data[2] else 0
                arr[i].data, arr[i].nbytes, arr[i].on_device = data[0], data[1], dev
            else:
                b = ctypes.create_string_buffer(bytes(data), len(data) + 1)
                keep.append(b)
                arr[i].data = ctypes.cast(b, ctypes.c_void_p)
                arr[i].nbytes, arr[i].on_device = len(data), 0
            arr[i].kind = kind
        h = ctypes.c_void_p()
        self._check(self.L.bg_load(self.ctx, n, arr, ctypes.byref(h)))
        return InputSet(self, h, keep)

    # -------------------------------------------------------------- bedops
    def op(self, mode, s, files, spec=None, full_left=False, chop=(1, 0, False)):
        """Run one bedops operation on loaded set `s` over file indices `files`.
        spec: -e/-n overlap; full_left: --complement -L; chop: (bp, stagger, -x)."""
        h = ctypes.c_void_p()
        idx = (ctypes.c_int * len(files))(*files)
        L = self.L
        if mode in ("-m", "--merge"):
            self._check(L.bg_merge(self.ctx, s.h, idx, len(files), ctypes.byref(h)))
        elif mode in ("-i", "--intersect"):
            self._check(L.bg_intersect(self.ctx, s.h, idx, len(files), ctypes.byref(h)))
        elif mode in ("-d", "--difference"):
            rest = (ctypes.c_int * (len(files) - 1))(*files[1:])
            self._check(L.bg_difference(self.ctx, s.h, files[0], rest, len(files) - 1,
                                        ctypes.byref(h)))
        elif mode in ("-e", "--element-of", "-n", "--not-element-of"):
            thr, pct = parse_overlap_spec(spec)
            inv = 1 if mode in ("-n", "--not-element-of") else 0
            rest = (ctypes.c_int * (len(files) - 1))(*files[1:])
            self._check(L.bg_element_of(self.ctx, s.h, files[0], rest, len(files) - 1, thr, pct,
                                        inv, ctypes.byref(h)))
        elif mode in ("-c", "--complement"):
            self._check(L.bg_complement(self.ctx, s.h, idx, len(files), int(bool(full_left)),
                                        ctypes.byref(h)))
        elif mode in ("-w", "--chop"):
            bp, stagger, x = chop
            self._check(L.bg_chop(self.ctx, s.h, idx, len(files), int(bp), int(stagger),
                                  int(bool(x)), ctypes.byref(h)))
        elif mode in ("-p", "--partition"):
            self._check(L.bg_partition(self.ctx, s.h, idx, len(files), ctypes.byref(h)))
        elif mode in ("-s", "--symmdiff"):
            self._check(L.bg_symmdiff(self.ctx, s.h, idx, len(files), ctypes.byref(h)))
        elif mode in ("-u", "--everything"):
            self._check(L.bg_everything(self.ctx, s.h, idx, len(files), ctypes.byref(h)))
        else:
            raise BedgpuError(-6, f"unknown operation {mode}")
        return Result(self, h)

    def bedops(self, mode, texts, spec=None, chrom=None, pad=None, full_left=False,
               chop=(1, 0, False), set_load=True):
        """bedops [--chrom C] [--range L:R] <mode> [spec] file1 file2 ... on in-memory BED
        texts -> output bytes. pad = (lpad, rpad). set_load: inputs whose rows the
        operation never reads are parsed straight to their merged set (BED3_SET), as the
        bedops front-end does; False keeps the row columns (BED3)."""
        eo = mode in ("-e", "--element-of", "-n", "--not-element-of")
        every = mode in ("-u", "--everything")
        plain = BED3_SET if (set_load and mode in SET_MODES and not chrom and pad is None) else BED3
        s = self.load([(t, BED3_REST if (every or (eo and i == 0)) else plain)
                       for i, t in enumerate(texts)])
        try:
            if chrom:
                s.restrict_chrom(chrom)
            if pad is not None:
                for i in range(len(texts)):
                    if not (eo and i == 0):
                        s.pad(i, pad[0], pad[1])
            r = self.op(mode, s, list(range(len(texts))), spec, full_left, chop)
            try:
                return r.text()
            finally:
                r.free()
        finally:
            s.free()

    # -------------------------------------------------------------- --ec
    def check(self, text, nfields=3, has_rest=False, name="-"):
        """--ec validation of one input on the GPU (bg_check): None if it passes, else the
        reference's exception text "in <name>\n<message>\nSee row: <n>"."""
        buf = ctypes.create_string_buffer(bytes(text), len(text) or 1)
        i = _Input(ctypes.cast(buf, ctypes.c_void_p), len(text), 0, BED3)
        r = _CheckResult()
        self._check(self.L.bg_check(self.ctx, ctypes.byref(i), nfields, 1 if has_rest else 0,
                                    ctypes.byref(r)))
        if not r.row:
            return None
        line = bytes(text[r.line_off:r.line_off + r.line_len])
        msg = ctypes.create_string_buffer(4096)
        self._check(self.L.bg_check_message(line, len(line), r.code, nfields, 1 if has_rest else 0,
                                            msg, 4096))
        return f"in {name}\n".encode() + msg.value + f"\nSee row: {r.row}".encode()

    # -------------------------------------------------------------- bedmap
    def map_op(self, s, ops, ref=0, map_=1, overlap_bp=1, precision=6, delim="|",
               skip_unmapped=False, criterion="bp-ovr", value=None, multidelim=";", sci=False,
               faster=False):
        """bedmap <ops> on loaded set `s` (ref/map file indices) -> Result.
        criterion: "bp-ovr" (value = overlap_bp), "range" (value = bp), "fraction-ref",
        "fraction-map", "fraction-either", "fraction-both" (value = fraction), "exact"."""
        o = _MapOpts()
        o.overlap_bp = overlap_bp
        o.n_ops = len(ops)
        for k, op in enumerate(ops):  # a name, (name, arg) for kth/mad, (name, lo, hi) for tmean
            t = op if isinstance(op, tuple) else (op,)
            o.ops[k] = MAP_OPS[t[0]]
            o.op_arg[k] = float(t[1]) if len(t) > 1 else 0.0
            o.op_arg2[k] = float(t[2]) if len(t) > 2 else 0.0
        o.precision = precision
        o.scientific = 1 if sci else 0
        o.skip_unmapped = 1 if skip_unmapped else 0
        o.delim = delim.encode()
        o.multidelim = multidelim.encode()
        o.criterion = OVR_CRITERIA[criterion]
        if criterion == "range":
            o.range_bp = int(value)
        elif criterion.startswith("fraction"):
            o.fraction = float(value)
        o.faster = 1 if faster else 0
        h = ctypes.c_void_p()
        self._check(self.L.bg_map(self.ctx, s.h, ref, map_, ctypes.byref(o), ctypes.byref(h)))
        return Result(self, h)

    def bedmap(self, ops, ref_text, map_text=None, overlap_bp=1, precision=6, delim="|",
               skip_unmapped=False, chrom=None, criterion="bp-ovr", value=None, multidelim=";",
               sci=False, faster=False):
        names = [op[0] if isinstance(op, tuple) else op for op in ops]
        need5 = any(op in SCORE_OPS for op in names)
        mrest = any(op in MAP_REST_OPS for op in names)
        single = map_text is None  # single-file mode: rows are their own map rows
        if single:
            mrest = mrest or "echo" in names or "echo-map-id" in names or "echo-map-id-uniq" in names
        mkind = (BED5_REST if mrest else BED5) if need5 else (BED3_REST if mrest else BED3)
        if single:
            s = self.load([(ref_text, mkind)])
        else:
            # the reference rows' remainders size their strings in the heap replay (bg_heap.hip)
            rrest = "echo" in names or any(op in ADDR_OPS for op in names)
            s = self.load([(ref_text, BED3_REST if rrest else BED3), (map_text, mkind)])
        try:
            if chrom:
                s.restrict_chrom(chrom)
            r = self.map_op(s, ops, 0, 0 if single else 1, overlap_bp, precision, delim,
                            skip_unmapped, criterion, value, multidelim, sci, faster)
            try:
                return r.text()
            finally:
                r.free()
        finally:
            s.free()

    # -------------------------------------------------------------- closest-features
    def closest_op(self, s, ref=0, query=1, shortest=False, dist=False, no_ref=False,
                   no_overlaps=False, delim="|"):
        """closest-features on loaded set `s` (both tables BED3_REST) -> Result"""
        o = _ClosestOpts()
        o.shortest, o.print_dist = int(bool(shortest)), int(bool(dist))
        o.no_ref, o.no_overlaps = int(bool(no_ref)), int(bool(no_overlaps))
        o.delim = delim.encode()
        h = ctypes.c_void_p()
        self._check(self.L.bg_closest(self.ctx, s.h, ref, query, ctypes.byref(o), ctypes.byref(h)))
        return Result(self, h)

    def closest(self, input_text, query_text, shortest=False, dist=False, no_ref=False,
                no_overlaps=False, delim="|", chrom=None):
        """closest-features [flags] <input-file> <query-file> on in-memory texts -> bytes"""
        s = self.load([(input_text, BED3_REST), (query_text, BED3_REST)])
        try:
            if chrom:
                s.restrict_chrom(chrom)
            r = self.closest_op(s, 0, 1, shortest, dist, no_ref, no_overlaps, delim)
            try:
                return r.text()
            finally:
                r.free()
        finally:
            s.free()

    def prof_enable(self, filt):
        self._check(self.L.bg_prof_enable(self.ctx, filt.encode() if filt else None))

    def prof_read(self):
        """{kernel: (launches, total_ms)} measured with HIP events on the engine stream"""
        buf = ctypes.create_string_buffer(1 << 16)
        self._check(self.L.bg_prof_read(self.ctx, buf, 1 << 16))
        out = {}
        for ln in buf.value.decode().splitlines():
            name, calls, ms = ln.split()
            out[name] = (int(calls), float(ms))
        return out

    def stats(self):
        buf = ctypes.create_string_buffer(8192)
        self._check(self.L.bg_stats(self.ctx, buf, 8192))
        return buf.value.decode()


def group_uid():
    """ncclGetUniqueId on this process (rank 0 of a multi-process group): 128 bytes."""
    L = load_library()
    buf = ctypes.create_string_buffer(UID_BYTES)
    rc = L.bg_group_uid(buf)
    if rc:
        raise BedgpuError(rc, "bg_group_uid failed (RCCL)")
    return buf.raw


class Group:
    """Several devices working on chromosome shards (include/bedgpu.h bg_group_*):
    Group(devices=[0, 1, ...]) in one process, or Group(device=d, uid=..., nranks=N,
    rank=r) as one rank of a multi-process group. gather() reassembles every member's
    per-chromosome text on rank 0 over RCCL."""

    def __init__(self, devices=None, device=None, uid=None, nranks=1, rank=0):
        self.L = load_library()
        self.h = ctypes.c_void_p()
        if devices is not None:
            arr = (ctypes.c_int * len(devices))(*devices)
            rc = self.L.bg_group_open(ctypes.byref(self.h), arr, len(devices))
        else:
            rc = self.L.bg_group_open_rank(ctypes.byref(self.h), int(device), uid, int(nranks), int(rank))
        if rc:
            raise BedgpuError(rc, "bg_group_open failed")
        nl, nr, r0 = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self.L.bg_group_size(self.h, ctypes.byref(nl), ctypes.byref(nr), ctypes.byref(r0))
        self.nlocal, self.nranks, self.rank0 = nl.value, nr.value, r0.value
        self.engines = [Engine(ctx=self.L.bg_group_ctx(self.h, k)) for k in range(self.nlocal)]

    def gather(self, nchrom, parts):
        """parts: per local member (text_devptr, offsets[nchrom], lengths[nchrom]) over the
        GLOBAL chromosome list. Returns (devptr, nbytes) on rank 0, (None, 0) elsewhere."""
        n = len(parts)
        texts = (ctypes.c_void_p * n)(*[p[0] for p in parts])
        keep = []
        offs, lens = (ctypes.c_void_p * n)(), (ctypes.c_void_p * n)()
        for k, (_, o, ln) in enumerate(parts):
            ao = (ctypes.c_uint64 * max(nchrom, 1))(*o)
            al = (ctypes.c_uint64 * max(nchrom, 1))(*ln)
            keep += [ao, al]
            offs[k] = ctypes.cast(ao, ctypes.c_void_p)
            lens[k] = ctypes.cast(al, ctypes.c_void_p)
        out, nb = ctypes.c_void_p(), ctypes.c_uint64()
        rc = self.L.bg_group_gather(self.h, int(nchrom), texts, offs, lens, ctypes.byref(out),
                                    ctypes.byref(nb))
        if rc:
            raise BedgpuError(rc, self.L.bg_last_error(self.engines[0].ctx).decode(errors="replace"))
        return (out.value, nb.value) if out.value else (None, 0)

    def close(self):
        if self.h:
            for e in self.engines:
                e.ctx = None
            self.L.bg_group_close(self.h)
            self.h = None
