"""ctypes binding of libcelestia_eds.so (include/celestia_eds.h).

The shared library holds the HIP kernels and the C++ host layer; this module only
declares signatures and turns status codes into exceptions. It fails loudly when
the library or a device is missing: there is no CPU fallback anywhere in the
product path.
"""
import ctypes
import os
import threading

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_PKG_DIR)
LIB_PATH = os.environ.get("CEL_EDS_LIB", os.path.join(_ROOT, "libcelestia_eds.so"))

OK, EINVAL, ENOTPOW2, ECHUNK, ETOOBIG, EORDER, ETOOFEW, EBYZANTINE, EUNREPAIRABLE, EDEVICE, ENOMEM, \
    ESHORT, EPUSHPAST, EBADROOT, ENODATA = range(15)
FLAG_ORDER_CHECK = 0x1
FLAG_PARITY_ONLY = 0x2
FLAG_CALLER_STREAM = 0x4
FLAG_SHARD_EXCHANGE = 0x8
FLAG_SHARD_PEERCOPY = 0x10
SHARE_SIZE = 512
NAMESPACE_SIZE = 29
NMT_NODE_SIZE = 90

# Exported symbols (must match include/celestia_eds.h; tests check both ways).
EXPORTS = [
    "cel_ctx_create", "cel_ctx_destroy", "cel_strerror", "cel_last_error", "cel_device_name",
    "cel_extend_shares", "cel_extend_batch", "cel_dev_workspace_size", "cel_dev_extend_batch",
    "cel_dev_extend_only", "cel_dev_commit_only", "cel_dev_place_ods", "cel_dev_decode", "cel_host_alloc", "cel_host_free", "cel_codec_encode", "cel_codec_decode",
    "cel_codec_max_chunks", "cel_codec_name", "cel_codec_validate_chunk_size", "cel_axis_root",
    "cel_nmt_root", "cel_dah_hash", "cel_merkle_hash_slices", "cel_repair", "cel_dev_repair", "cel_debug_schedule_fuzz", "cel_debug_repair_plan", "cel_dev_shard_workspace_size", "cel_dev_shard_rows",
    "cel_dev_shard_cols", "cel_dev_shard_finish", "cel_square_construct", "cel_square_last_error", "cel_square_tx_range",
    "cel_axis_trees", "cel_axis_tree", "cel_dah_tree", "cel_nmt_prove_range", "cel_merkle_aunts", "cel_commitment_paths",
    "cel_get_commitment", "cel_subtree_root_coordinates",
    "cel_extend_sharded", "cel_shard_plan_create", "cel_shard_plan_destroy", "cel_shard_plan_transport",
    "cel_shard_plan_last_error", "cel_shard_plan_note", "cel_shard_plan_time_exchange", "cel_shard_plan_upload", "cel_shard_plan_run", "cel_shard_plan_wait",
    "cel_extend_batch_multi", "cel_probe_sha256", "cel_probe_hbm_copy", "cel_probe_hbm_stream",
    "cel_probe_rs_transform",
]

_lib = None
_lock = threading.Lock()


class CelError(Exception):
    def __init__(self, status, message):
        super().__init__(message)
        self.status = status


def load():
    """Load the library (no device needed) and declare every signature."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise CelError(EDEVICE, f"{LIB_PATH} is missing: build it with `make -C celestia-app_amd`")
        l = ctypes.CDLL(LIB_PATH)
        P, u32, i32, u64, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint64, ctypes.c_size_t
        PP = ctypes.POINTER(ctypes.c_void_p)
        sigs = {
            "cel_ctx_create": (i32, [ctypes.c_int, PP]),
            "cel_ctx_destroy": (None, [P]),
            "cel_strerror": (ctypes.c_char_p, [i32]),
            "cel_last_error": (ctypes.c_char_p, [P]),
            "cel_device_name": (i32, [P, ctypes.c_char_p, sz]),
            "cel_extend_shares": (i32, [P, P, u32, u32, P, P, P, P, u32]),
            "cel_extend_batch": (i32, [P, P, u32, u32, u32, P, P, P, P, P, u32]),
            "cel_dev_workspace_size": (sz, [u32, u32]),
            "cel_dev_extend_batch": (i32, [P, P, u32, u32, P, P, P, P, P, P, P, u32]),
            "cel_dev_extend_only": (i32, [P, P, u32, u32, P, P]),
            "cel_dev_place_ods": (i32, [P, P, u32, u32, P, P]),
            "cel_host_alloc": (P, [ctypes.c_size_t]),
            "cel_host_free": (None, [P]),
            "cel_dev_commit_only": (i32, [P, P, u32, u32, P, P, P, P, P, P, u32]),
            "cel_codec_encode": (i32, [P, P, u32, u32, P]),
            "cel_codec_decode": (i32, [P, P, P, u32, u32]),
            "cel_dev_decode": (i32, [P, P, P, u32, u32, u32, P]),
            "cel_codec_max_chunks": (u64, []),
            "cel_codec_name": (ctypes.c_char_p, []),
            "cel_codec_validate_chunk_size": (i32, [u32]),
            "cel_axis_root": (i32, [P, P, u32, u32, u32, P, u32]),
            "cel_nmt_root": (i32, [P, P, u32, u32, P, u32]),
            "cel_dah_hash": (i32, [P, P, P, u32, P]),
            "cel_merkle_hash_slices": (i32, [P, P, P, u32, P]),
            "cel_repair": (i32, [P, P, P, u32, u32, P, P, P, P, P, P]),
            "cel_dev_repair": (i32, [P, P, P, u32, P, P, P, P, P, P]),
            "cel_debug_schedule_fuzz": (i32, [P, u64, u32]),
            "cel_debug_repair_plan": (i32, [P, u32, P, P, P, P, P]),
            "cel_dev_shard_workspace_size": (sz, [u32, u32]),
            "cel_dev_shard_rows": (i32, [P, P, u32, u32, P, P]),
            "cel_dev_shard_cols": (i32, [P, P, u32, u32, u32, P, P, P, P, P, u32]),
            "cel_dev_shard_finish": (i32, [P, P, u32, u32, P, P, P, P, P, P, u32]),
            "cel_square_construct": (i32, [P, P, u32, u32, u32, u32, P, u32, P, P]),
            "cel_square_last_error": (ctypes.c_char_p, []),
            "cel_square_tx_range": (i32, [P, P, u32, u32, u32, u32, P, P]),
            "cel_axis_trees": (i32, [P, P, u32, u32, u32, u32, u32, P]),
            "cel_axis_tree": (i32, [P, P, u32, u32, u32, P]),
            "cel_dah_tree": (i32, [P, P, P, u32, P]),
            "cel_nmt_prove_range": (i32, [P, u32, u32, u32, P, P]),
            "cel_merkle_aunts": (i32, [P, u32, u32, P, P]),
            "cel_commitment_paths": (i32, [u32, u32, u32, u32, P, P, P, u32, P]),
            "cel_get_commitment": (i32, [P, P, u32, u32, u32, u32, u32, P]),
            "cel_subtree_root_coordinates": (i32, [u32, u32, u32, u32, P, P, u32, P]),
            "cel_extend_sharded": (i32, [P, u32, P, u32, u32, P, P, P, P, u32]),
            "cel_shard_plan_create": (i32, [P, u32, u32, u32, PP]),
            "cel_shard_plan_destroy": (None, [P]),
            "cel_shard_plan_transport": (ctypes.c_char_p, [P]),
            "cel_shard_plan_last_error": (ctypes.c_char_p, [P]),
            "cel_shard_plan_note": (ctypes.c_char_p, [P]),
            "cel_shard_plan_time_exchange": (i32, [P, u32, ctypes.POINTER(ctypes.c_double)]),
            "cel_shard_plan_upload": (i32, [P, P]),
            "cel_shard_plan_run": (i32, [P]),
            "cel_shard_plan_wait": (i32, [P, P, P, P, P]),
            "cel_extend_batch_multi": (i32, [P, u32, P, u32, u32, u32, P, P, P, P, P, u32]),
            "cel_probe_sha256": (i32, [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
            "cel_probe_hbm_copy": (i32, [P, u64, ctypes.POINTER(ctypes.c_double)]),
            "cel_probe_hbm_stream": (i32, [P, u64] + [ctypes.POINTER(ctypes.c_double)] * 3),
            "cel_probe_rs_transform": (i32, [P, u32, ctypes.POINTER(ctypes.c_double)]),
        }
        for name, (res, args) in sigs.items():
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        _lib = l
        return l


class Context:
    """One HIP device + stream (cel_ctx)."""

    def __init__(self, device=0):
        l = load()
        h = ctypes.c_void_p()
        st = l.cel_ctx_create(int(device), ctypes.byref(h))
        if st != OK:
            raise CelError(st, f"cel_ctx_create(device={device}) failed: {l.cel_strerror(st).decode()}")
        self.handle = h
        self.device = device
        self.lib = l

    def check(self, st):
        if st != OK:
            msg = self.lib.cel_last_error(self.handle).decode() or self.lib.cel_strerror(st).decode()
            raise CelError(st, msg)

    def device_name(self):
        buf = ctypes.create_string_buffer(256)
        self.check(self.lib.cel_device_name(self.handle, buf, 256))
        return buf.value.decode()

    def close(self):
        if self.handle:
            self.lib.cel_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default = {}


def default_context(device=None):
    if device is None:
        device = int(os.environ.get("CEL_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    with _lock:
        ctx = _default.get(device)
    if ctx is None:
        ctx = Context(device)
        with _lock:
            _default[device] = ctx
    return ctx
