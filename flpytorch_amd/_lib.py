"""ctypes binding of libflcodec.so (the C ABI in include/flcodec.h).

The library is the product: there is no CPU fallback.  If the shared object is missing, or no
MI355X is visible when a compute entry point is called, the call raises — it never reroutes to
anything else.
"""
import collections
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# A/B variant builds (tools/ab_build.sh) live in <repo>/abvar/libflcodec_<tag>.so, outside the
# package: FLC_LIB_VARIANT=<tag> loads one instead of the product library (tuning runs only).
VARIANT_DIR = os.path.join(os.path.dirname(_HERE), "abvar")
LIB_PATH = (os.path.join(VARIANT_DIR, "libflcodec_%s.so" % os.environ["FLC_LIB_VARIANT"])
            if os.environ.get("FLC_LIB_VARIANT") else os.path.join(_HERE, "libflcodec.so"))

FLC_OK, FLC_ERR_ARG, FLC_ERR_DTYPE, FLC_ERR_HIP, FLC_ERR_WORKSPACE, FLC_ERR_UNSUPPORTED = range(6)
FLC_IDENT, FLC_LAZY, FLC_RANDK, FLC_NATURAL, FLC_STD_DITHERING, FLC_NAT_DITHERING, FLC_TOPK, FLC_RANK_K = range(1, 9)
FLC_NORM_LINF, FLC_NORM_L1, FLC_NORM_L2 = 0, 1, 2
FLC_REDUCE_PLAIN, FLC_REDUCE_REL_X = 0, 1
# execution hints (flc_codec_params.flags): how, never what — every choice gives the same bits
FLC_PATH_AUTO, FLC_PATH_SPARSE, FLC_PATH_DENSE = 0, 1, 2
FLC_TIE_LOWEST, FLC_TIE_HIGHEST = 0, 1
ABI_VERSION = 104


def FLC_ROW_GROUPS(g):
    return (int(g) & 0xFF) << 8

# every symbol include/flcodec.h declares (tests/test_host.py checks the .so exports all of them)
EXPORTS = [
    "flc_version", "flc_build_id", "flc_last_error_string",
    "flc_reduce_rows", "flc_reduce_matrix",
    "flc_encode_workspace_size", "flc_encode",
    "flc_encode_reduce_workspace_size", "flc_encode_reduce",
    "flc_encode_shift_workspace_size", "flc_encode_shift",
    "flc_payload_bytes", "flc_payload_format", "flc_payload_validate", "flc_pack_workspace_size", "flc_pack", "flc_unpack",
    "flc_unpack_reduce_workspace_size", "flc_unpack_reduce",
    "flc_combine_workspace_size", "flc_combine_partials",
    "flc_combine_blocks_workspace_size", "flc_combine_blocks",
    "flc_mt_choice", "flc_mt_rand", "flc_mt_randint31",
    "flc_device_uniform", "flc_device_randk_indices",
    "flc_device_randk_counts_workspace_size", "flc_device_randk_counts",
    "flc_profile_enable", "flc_profile_collect", "flc_select_row_flags",
    "flc_selftest_division", "flc_norm2_torch_cpu", "flc_debug_resident",
    "flc_norm2_torch_cpu_workspace_size", "flc_norm2_torch_cpu_ws", "flc_rows_alloc", "flc_rows_free",
]


class FlcCodecParams(ctypes.Structure):
    _fields_ = [
        ("codec", ctypes.c_int32),
        ("s", ctypes.c_int32),
        ("norm", ctypes.c_int32),
        ("flags", ctypes.c_int32),
        ("k", ctypes.c_int64),
        ("lazy_p", ctypes.c_float),
        ("randk_scale", ctypes.c_float),
        ("d_levels", ctypes.c_void_p),
        ("seed", ctypes.c_uint64),
        ("tie", ctypes.c_int32),
    ]


class FlcPattern(ctypes.Structure):
    _fields_ = [
        ("d_randk_idx", ctypes.c_void_p),
        ("d_uniforms", ctypes.c_void_p),
        ("d_lazy_u", ctypes.c_void_p),
        ("client0", ctypes.c_int64),
        ("uniforms_ld", ctypes.c_int64),
        ("idx_ld", ctypes.c_int64),
        ("d_randk_counts", ctypes.c_void_p),
    ]


class FlcError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()


def load():
    """Load libflcodec.so (raises if it was not built — no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"flpytorch_amd: {LIB_PATH} is missing — build it with "
                "`make -C flpytorch_amd/csrc` (or __graft_entry__.build()); there is no CPU fallback")
        _lib = _bind(ctypes.CDLL(LIB_PATH))
        return _lib


def open_variant(tag):
    """Another build of the library for an in-process A/B (tools/ab_inproc.py): tag "" or "prod" is
    the product libflcodec.so, else abvar/libflcodec_<tag>.so.  Not cached; make it the one
    every wrapper calls with ``use(lib)``."""
    path = (os.path.join(_HERE, "libflcodec.so") if tag in ("", "prod")
            else os.path.join(VARIANT_DIR, f"libflcodec_{tag}.so"))
    if not os.path.exists(path):
        raise ImportError(f"flpytorch_amd: {path} is missing")
    return _bind(ctypes.CDLL(path))


class use:
    """Context manager: the wrappers call ``lib`` (an open_variant() handle) inside the block."""

    def __init__(self, lib):
        self.lib, self.prev = lib, None

    def __enter__(self):
        global _lib
        load()
        self.prev, _lib = _lib, self.lib
        return self.lib

    def __exit__(self, *exc):
        global _lib
        _lib = self.prev
        return False


def _bind(lib):
    """Declare the C ABI's argument and result types on a loaded library."""
    vp, i64, f32, i32, sz = ctypes.c_void_p, ctypes.c_int64, ctypes.c_float, ctypes.c_int, ctypes.c_size_t
    P = ctypes.POINTER
    lib.flc_version.restype = i32
    lib.flc_last_error_string.restype = ctypes.c_char_p
    lib.flc_build_id.restype = ctypes.c_char_p
    lib.flc_reduce_rows.argtypes = [vp, i64, i64, vp, vp, f32, i32, vp, vp]
    lib.flc_reduce_matrix.argtypes = [vp, i64, i64, i64, vp, vp, f32, i32, vp, vp]
    lib.flc_encode_workspace_size.argtypes = [P(FlcCodecParams), i64]
    lib.flc_encode_workspace_size.restype = sz
    lib.flc_encode.argtypes = [P(FlcCodecParams), P(FlcPattern), vp, i64, vp, vp, vp, vp, sz, vp]
    lib.flc_encode_reduce_workspace_size.argtypes = [P(FlcCodecParams), i64, i64]
    lib.flc_encode_reduce_workspace_size.restype = sz
    lib.flc_encode_reduce.argtypes = [P(FlcCodecParams), P(FlcPattern), vp, i64, vp, i64, i64, vp, f32, vp, vp,
                                      vp, sz, vp]
    lib.flc_encode_shift_workspace_size.argtypes = [P(FlcCodecParams), i64]
    lib.flc_encode_shift_workspace_size.restype = sz
    lib.flc_encode_shift.argtypes = [P(FlcCodecParams), P(FlcPattern), vp, vp, i64, f32, vp, vp, f32, vp, vp, vp,
                                     vp, sz, vp]
    lib.flc_payload_bytes.argtypes = [P(FlcCodecParams), i64]
    lib.flc_payload_bytes.restype = i64
    lib.flc_payload_format.argtypes = [P(FlcCodecParams)]
    lib.flc_payload_validate.argtypes = [P(FlcCodecParams), vp, i64, i64]
    lib.flc_pack_workspace_size.argtypes = [P(FlcCodecParams), i64]
    lib.flc_pack_workspace_size.restype = sz
    lib.flc_pack.argtypes = [P(FlcCodecParams), P(FlcPattern), vp, i64, vp, vp, sz, vp]
    lib.flc_unpack.argtypes = [P(FlcCodecParams), vp, i64, vp, vp]
    lib.flc_unpack_reduce_workspace_size.argtypes = [P(FlcCodecParams), i64, i64]
    lib.flc_unpack_reduce_workspace_size.restype = sz
    lib.flc_unpack_reduce.argtypes = [P(FlcCodecParams), vp, i64, vp, i64, i64, vp, f32, vp, vp, sz, vp]
    lib.flc_combine_workspace_size.argtypes = [vp, i64, i32]
    lib.flc_combine_workspace_size.restype = sz
    lib.flc_combine_partials.argtypes = [vp, vp, i64, f32, i32, vp, sz, vp]
    lib.flc_combine_blocks_workspace_size.argtypes = [vp, i64, i64]
    lib.flc_combine_blocks_workspace_size.restype = sz
    lib.flc_combine_blocks.argtypes = [vp, vp, i64, i64, i64, f32, vp, vp, sz, vp]
    lib.flc_mt_choice.argtypes = [vp, vp, i64, i64, vp, vp]
    lib.flc_mt_rand.argtypes = [vp, vp, i64, vp]
    lib.flc_mt_randint31.argtypes = [vp, vp, i64, vp]
    lib.flc_device_uniform.argtypes = [ctypes.c_uint64, i64, i64]
    lib.flc_device_uniform.restype = ctypes.c_double
    lib.flc_device_randk_indices.argtypes = [ctypes.c_uint64, i64, i64, i64, vp]
    lib.flc_device_randk_counts_workspace_size.argtypes = [i64, i64]
    lib.flc_device_randk_counts_workspace_size.restype = sz
    lib.flc_device_randk_counts.argtypes = [ctypes.c_uint64, i64, i64, i64, i64, vp, vp, sz, vp]
    lib.flc_profile_enable.argtypes = [i32]
    lib.flc_profile_collect.argtypes = [ctypes.c_char_p, vp, vp]
    lib.flc_selftest_division.argtypes = [vp, i32, vp, vp]
    if hasattr(lib, "flc_norm2_torch_cpu"):         # (absent from A/B builds of older revisions)
        lib.flc_norm2_torch_cpu.argtypes = [vp, i64, i64, i64, vp, vp]
    if hasattr(lib, "flc_norm2_torch_cpu_ws"):      # (absent from A/B builds of older revisions)
        lib.flc_norm2_torch_cpu_workspace_size.argtypes = [i64, i64]
        lib.flc_norm2_torch_cpu_workspace_size.restype = sz
        lib.flc_norm2_torch_cpu_ws.argtypes = [vp, i64, i64, i64, vp, vp, sz, vp]
    if hasattr(lib, "flc_rows_alloc"):              # (absent from A/B builds of older revisions)
        lib.flc_rows_alloc.argtypes = [sz, i32, vp]
        lib.flc_rows_free.argtypes = [vp]
    if hasattr(lib, "flc_debug_resident"):          # (absent from A/B builds of older revisions)
        lib.flc_debug_resident.argtypes = [i32, i64]
    if hasattr(lib, "flc_select_row_flags"):        # (absent from A/B builds of older revisions)
        lib.flc_select_row_flags.argtypes = [P(FlcCodecParams), i64, i64, vp, sz, vp, vp]
    for name in EXPORTS:
        if not hasattr(lib, name):
            continue
        if name not in ("flc_version", "flc_build_id", "flc_last_error_string", "flc_device_uniform",
                        "flc_encode_workspace_size", "flc_encode_reduce_workspace_size",
                        "flc_encode_shift_workspace_size", "flc_payload_bytes", "flc_pack_workspace_size",
                        "flc_unpack_reduce_workspace_size", "flc_combine_workspace_size",
                        "flc_combine_blocks_workspace_size", "flc_device_randk_counts_workspace_size",
                        "flc_norm2_torch_cpu_workspace_size"):
            getattr(lib, name).restype = i32
    return lib


def source_hash(root=None):
    """The digest flc_build_id() reports for a library built from the tree at ``root`` (default:
    this package's tree): sha256 over csrc/*.hip, *.hpp, *.cpp in name order, csrc/Makefile, then
    include/flcodec.h; first 16 hex digits."""
    import glob
    import hashlib
    root = root or os.path.dirname(_HERE)
    csrc = os.path.join(root, "flpytorch_amd", "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.hpp")) +
                   glob.glob(os.path.join(csrc, "*.cpp")))
    files += [os.path.join(csrc, "Makefile"), os.path.join(root, "include", "flcodec.h")]
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_id():
    return load().flc_build_id().decode()


def check_provenance():
    """Raise unless the loaded library was built from this tree's sources (a stale or foreign
    .so would otherwise be measured and tested under this tree's name).  A FLC_LIB_VARIANT
    library (A/B builds) is reported, not checked."""
    bid, want = build_id(), source_hash()
    if os.environ.get("FLC_LIB_VARIANT"):
        return bid
    if bid != want:
        raise RuntimeError(f"flpytorch_amd: {LIB_PATH} was built from sources {bid}, the tree is {want} — "
                           "rebuild with `make -C flpytorch_amd/csrc`")
    return bid


def check(rc, what):
    if rc == FLC_OK:
        return
    msg = f"{what}: {load().flc_last_error_string().decode(errors='replace')} (status {rc})"
    if rc == FLC_ERR_ARG:
        raise ValueError(msg)
    if rc == FLC_ERR_DTYPE:
        raise TypeError(msg)
    if rc == FLC_ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    raise FlcError(msg)


def profile_enable(on=True):
    load().flc_profile_enable(1 if on else 0)


def profile_collect(kernel):
    """(total_ms, launches) of one kernel name since the last collect (waits for its events)."""
    ms, n = ctypes.c_double(0.0), ctypes.c_int64(0)
    check(load().flc_profile_collect(kernel.encode(), ctypes.byref(ms), ctypes.byref(n)), "flc_profile_collect")
    return ms.value, n.value


def require_gpu():
    """Raise unless an MI355X (HIP device) is visible — the product has no CPU path."""
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("flpytorch_amd: no HIP device visible — the codec/reduce path runs only on "
                           "MI355X (gfx950); there is no CPU fallback")


def stream_ptr(device=None):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class Workspace:
    """Per-(device, stream) scratch for the library (grown on demand, reused across calls).

    Keyed by the CURRENT stream, not the thread: calls queued on one stream run in
    stream order, so they may share one buffer; two streams never do, so concurrent calls on two
    streams (of one thread or of several) cannot race on the scratch.  A buffer is allocated while
    its stream is current, so when it grows the caching allocator hands the old block out again
    only to work queued after it on that same stream (torch's stream-ordered reuse): a kernel
    still reading the old scratch is never overwritten."""

    # streams whose scratch is kept (least recently used dropped beyond it: a thread pool that
    # makes streams per worker does not hold one buffer per stream ever seen — VERDICT r05); a
    # dropped buffer goes back to torch's caching allocator in its stream's order, so work still
    # queued on that stream keeps it until done
    MAX_STREAMS = 16

    def __init__(self):
        self._bufs = collections.OrderedDict()
        self._lock = threading.Lock()

    def get(self, device, nbytes):
        import torch
        dev = torch.device(device)
        st = torch.cuda.current_stream(dev)
        key = (str(dev), st.cuda_stream)
        with self._lock:
            buf = self._bufs.get(key)
            if buf is None or buf.numel() < nbytes:
                buf = None
                self._bufs.pop(key, None)
                if nbytes >= WS_CONTIG_MIN and os.environ.get("FLC_WS_CONTIG", "0") == "1":
                    # (A/B: large scratch in physically contiguous HBM, flc_rows_alloc)
                    from .resident import resident_rows
                    buf, _ = resident_rows(1, int(nbytes), dtype=torch.uint8, device=dev)
                    buf = buf.view(-1)
                else:
                    with torch.cuda.stream(st):
                        buf = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=dev)
                self._bufs[key] = buf
            self._bufs.move_to_end(key)
            while len(self._bufs) > self.MAX_STREAMS:
                self._bufs.popitem(last=False)
            return buf

    def release(self):
        """Drop every cached buffer (tests; a long-lived process after a large call)."""
        with self._lock:
            self._bufs.clear()


WS_CONTIG_MIN = 1 << 30
WORKSPACE = Workspace()
