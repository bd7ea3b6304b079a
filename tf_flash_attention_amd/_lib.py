"""ctypes binding to the C ABI in ``include/fa_api.h`` (libfa_hip.so).

This is the only way the Python layer reaches the device: there is no eager /
CPU fallback.  If the HIP library is missing the first call raises
:class:`LibraryNotBuiltError` — loudly, by design.
"""

from __future__ import annotations

import contextlib
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FA_HIP_LIB", os.path.join(_HERE, "libfa_hip.so"))

F16, F32, F64 = 0, 1, 2
FULL, CAUSAL, LOCAL = 0, 1, 2
NONE_FRONT, SCALE_FRONT, SCALE_END = 0, 1, 2

FA_OK = 0
FA_ERR_INVALID_ARGUMENT = -1
FA_ERR_UNSUPPORTED = -2
FA_ERR_WORKSPACE_TOO_SMALL = -3

# every symbol include/fa_api.h declares (checked by tests/test_boundary.py)
EXPORTED_SYMBOLS = (
    "fa_sync_mode_from_string",
    "fa_validate",
    "fa_forward",
    "fa_backward_workspace_bytes",
    "fa_backward",
    "fa_estimate_forward_flops",
    "fa_allowed_pairs",
    "fa_error_string",
    "fa_last_error",
    "fa_build_info",
    "fa_rule_mask",
    "fa_rule_probe",
)


class LibraryNotBuiltError(RuntimeError):
    pass


class FaProblem(ctypes.Structure):
    _fields_ = [
        ("dtype", ctypes.c_int32),
        ("policy", ctypes.c_int32),
        ("seq_dims", ctypes.c_int32),
        ("sync_mode", ctypes.c_int32),
        ("b", ctypes.c_int64),
        ("q_seq", ctypes.c_int32 * 2),
        ("k_seq", ctypes.c_int32 * 2),
        ("d", ctypes.c_int32),
        ("v_d", ctypes.c_int32),
        ("window_size", ctypes.c_int32),
        ("log2_stride_size", ctypes.c_int32),
        ("is_causal", ctypes.c_int32),
    ]


_lock = threading.Lock()
_lib = None
_tls = threading.local()  # .override: a library routed in by using() on THIS thread (tests: the diag build)
# the library routed in by using() for the whole process: autograd runs a CUDA tensor's backward on
# its own device thread, which does not see the thread-local override of the thread that called
# .backward() (the diag-variant backward tests otherwise ran the product library)
_process_override = None
_process_owner = None   # thread ident of the using() block that set _process_override
_process_depth = 0
_loaded = {}
DIAG_LIB_PATH = os.path.join(_HERE, "libfa_hip_diag.so")


def _declare(lib):
    P = ctypes.POINTER(FaProblem)
    vp = ctypes.c_void_p
    lib.fa_sync_mode_from_string.argtypes = [ctypes.c_char_p]
    lib.fa_sync_mode_from_string.restype = ctypes.c_int
    lib.fa_validate.argtypes = [P]
    lib.fa_validate.restype = ctypes.c_int
    lib.fa_forward.argtypes = [vp, P, vp, vp, vp, vp, vp, vp]
    lib.fa_forward.restype = ctypes.c_int
    lib.fa_backward_workspace_bytes.argtypes = [P]
    lib.fa_backward_workspace_bytes.restype = ctypes.c_size_t
    lib.fa_backward.argtypes = [vp, P, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, ctypes.c_size_t]
    lib.fa_backward.restype = ctypes.c_int
    lib.fa_estimate_forward_flops.argtypes = [P]
    lib.fa_estimate_forward_flops.restype = ctypes.c_double
    lib.fa_allowed_pairs.argtypes = [P]
    lib.fa_allowed_pairs.restype = ctypes.c_int64
    lib.fa_error_string.argtypes = [ctypes.c_int]
    lib.fa_error_string.restype = ctypes.c_char_p
    lib.fa_last_error.argtypes = []
    lib.fa_last_error.restype = ctypes.c_char_p
    lib.fa_rule_mask.argtypes = [P, vp]
    lib.fa_rule_mask.restype = ctypes.c_int
    lib.fa_rule_probe.argtypes = [P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                  ctypes.POINTER(ctypes.c_int32)]
    lib.fa_rule_probe.restype = ctypes.c_int
    lib.fa_build_info.argtypes = []
    lib.fa_build_info.restype = ctypes.c_char_p
    return lib


def lib():
    """Load (once) and return the HIP library, or raise LibraryNotBuiltError."""
    global _lib
    ov = getattr(_tls, "override", None)
    if ov is not None:
        return ov
    if _process_override is not None:
        return _process_override
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise LibraryNotBuiltError(
                    f"HIP library not found at {LIB_PATH}; build it with "
                    "`python -c 'import __graft_entry__ as g; g.build()'` or `make -C tf_flash_attention_amd`")
            try:
                _lib = _declare(ctypes.CDLL(LIB_PATH))
            except OSError as e:  # pragma: no cover - environment problem
                raise LibraryNotBuiltError(f"failed to load {LIB_PATH}: {e}") from e
    return _lib


@contextlib.contextmanager
def using(path):
    """Route every call made inside the block through the library at ``path``.

    The GPU tests use it to run the diagnostic build (libfa_hip_diag.so, ``make -C
    tf_flash_attention_amd diag``): its FA_FWD_VARIANT / FA_BWD_VARIANT structures are not in
    the product library.  ctypes loads each library RTLD_LOCAL, so both can live in one process.
    The routing covers this thread and, while the block runs, every other thread of the process
    (autograd's device thread runs the backward of a CUDA tensor); blocks do not nest across
    threads: a second thread entering ``using()`` while another thread's block is open raises."""
    global _process_override, _process_owner, _process_depth
    me = threading.get_ident()
    with _lock:
        if _process_owner is not None and _process_owner != me:
            raise RuntimeError("_lib.using(): another thread's library override is active; "
                               "blocks may not overlap across threads")
        h = _loaded.get(path)
        if h is None:
            if not os.path.exists(path):
                raise LibraryNotBuiltError(f"library not found at {path}")
            h = _loaded[path] = _declare(ctypes.CDLL(path))
        prev = getattr(_tls, "override", None)
        prev_proc = _process_override
        _tls.override = h
        _process_override = h
        _process_owner = me
        _process_depth += 1
    try:
        yield h
    finally:
        with _lock:
            _tls.override = prev
            _process_override = prev_proc
            _process_depth -= 1
            if _process_depth == 0:
                _process_owner = None


def make_problem(dtype, policy, seq_dims, sync_mode, b, q_seq, k_seq, d, v_d,
                 window_size=1, log2_stride_size=0, is_causal=False) -> FaProblem:
    p = FaProblem()
    p.dtype, p.policy, p.seq_dims, p.sync_mode = dtype, policy, seq_dims, sync_mode
    p.b = int(b)
    for i in range(2):
        p.q_seq[i] = int(q_seq[i]) if i < len(q_seq) else 1
        p.k_seq[i] = int(k_seq[i]) if i < len(k_seq) else 1
    p.d, p.v_d = int(d), int(v_d)
    p.window_size, p.log2_stride_size, p.is_causal = int(window_size), int(log2_stride_size), int(bool(is_causal))
    return p


def source_hash(diag: bool = False) -> str:
    """sha256 (first 16 hex digits) of the product sources, computed exactly as the Makefile's
    SRC_HASH (csrc/*.hip, csrc/*.h, ../include/fa_api.h in make's byte-wise sort order); with
    ``diag`` the diagnostic library's DIAG_HASH, which also covers csrc/diag/*.hip."""
    import glob
    import hashlib
    files = glob.glob(os.path.join(_HERE, "csrc", "*.hip")) + glob.glob(os.path.join(_HERE, "csrc", "*.h"))
    if diag:
        files += glob.glob(os.path.join(_HERE, "csrc", "diag", "*.hip"))
    rel = [os.path.relpath(p, _HERE) for p in files] + ["../include/fa_api.h"]
    h = hashlib.sha256()
    for r in sorted(rel, key=lambda x: x.encode()):
        with open(os.path.join(_HERE, r), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def build_info() -> str:
    return lib().fa_build_info().decode()


def last_error() -> str:
    return lib().fa_last_error().decode()
