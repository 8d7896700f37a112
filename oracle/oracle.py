"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes binding of the plain-C CPU restatement in this directory (see oracle.h for
what is restated and where it is pinned). Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module; the product package never does.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

NS = 29
NODE = 90
OK, EINVAL, ENOTPOW2, ECHUNK, EORDER, ETOOFEW, EBYZANTINE, EUNREPAIRABLE, EBADROOT = 0, 1, 2, 3, 5, 6, 7, 8, 13


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        l = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        u32, sz, i32 = ctypes.c_uint32, ctypes.c_size_t, ctypes.c_int
        l.orc_init.restype = None
        l.orc_set_simd.argtypes = [i32]
        l.orc_set_threads.argtypes = [i32]
        l.orc_gf_exp.argtypes = [i32, i32]
        l.orc_gf_log.argtypes = [i32, i32]
        l.orc_gf_skew.argtypes = [i32, i32]
        l.orc_gf_mul.argtypes = [i32, i32, i32]
        l.orc_sha256.argtypes = [P, sz, P]
        l.orc_rs_encode.argtypes = [u32, sz, P, P]
        l.orc_rs_decode.argtypes = [u32, sz, P, P]
        l.orc_extend.argtypes = [P, u32, sz, P]
        l.orc_roots.argtypes = [P, u32, sz, P, P, i32, P]
        l.orc_nmt_root.argtypes = [P, u32, sz, P, i32]
        l.orc_axis_root.argtypes = [P, sz, u32, u32, sz, P, i32]
        l.orc_merkle_root.argtypes = [P, u32, sz, P]
        l.orc_dah_hash.argtypes = [P, P, u32, P]
        l.orc_extend_and_commit.argtypes = [P, u32, sz, P, P, P, P]
        l.orc_repair.argtypes = [P, P, u32, sz, P, P, P, P, P, P]
        l.orc_repair_order.argtypes = [P, P, u32, sz, P, P, P, P, P, P, i32]
        l.orc_extend_commit_many.argtypes = [P, u32, u32, sz, P]
        l.orc_repair_many.argtypes = [P, P, u32, sz, P, P, u32, P]
        l.orc_init()
        _lib = l
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def set_simd(on):
    lib().orc_set_simd(1 if on else 0)


def set_threads(n):
    lib().orc_set_threads(int(n))


def sha256(msg: bytes) -> bytes:
    a = np.frombuffer(bytes(msg), dtype=np.uint8).copy() if msg else np.zeros(1, np.uint8)
    out = np.zeros(32, np.uint8)
    lib().orc_sha256(_p(a), len(msg), _p(out))
    return out.tobytes()


def rs_encode(data: np.ndarray) -> np.ndarray:
    """data: (n, len) uint8 -> parity (n, len)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    n, ln = data.shape
    par = np.zeros_like(data)
    rc = lib().orc_rs_encode(n, ln, _p(data), _p(par))
    if rc:
        raise ValueError(f"orc_rs_encode rc={rc}")
    return par


def rs_decode(shards: np.ndarray, present: np.ndarray) -> np.ndarray:
    shards = np.ascontiguousarray(shards, dtype=np.uint8).copy()
    present = np.ascontiguousarray(present, dtype=np.uint8)
    n2, ln = shards.shape
    rc = lib().orc_rs_decode(n2 // 2, ln, _p(shards), _p(present))
    if rc:
        raise ValueError(f"orc_rs_decode rc={rc}")
    return shards


def extend(ods: np.ndarray) -> np.ndarray:
    """ods: (k, k, share) -> eds (2k, 2k, share) in rsmt2d order."""
    ods = np.ascontiguousarray(ods, dtype=np.uint8)
    k, _, share = ods.shape
    eds = np.zeros((2 * k, 2 * k, share), np.uint8)
    rc = lib().orc_extend(_p(ods), k, share, _p(eds))
    if rc:
        raise ValueError(f"orc_extend rc={rc}")
    return eds


def roots(eds: np.ndarray, check_order=True):
    eds = np.ascontiguousarray(eds, dtype=np.uint8)
    w, _, share = eds.shape
    rr = np.zeros((w, NODE), np.uint8)
    cr = np.zeros((w, NODE), np.uint8)
    bad = ctypes.c_int32(-1)
    rc = lib().orc_roots(_p(eds), w // 2, share, _p(rr), _p(cr), 1 if check_order else 0,
                         ctypes.byref(bad))
    return rc, rr, cr


def dah_hash(row_roots: np.ndarray, col_roots: np.ndarray) -> bytes:
    rr = np.ascontiguousarray(row_roots, dtype=np.uint8)
    cr = np.ascontiguousarray(col_roots, dtype=np.uint8)
    out = np.zeros(32, np.uint8)
    lib().orc_dah_hash(_p(rr) if rr.size else None, _p(cr) if cr.size else None, rr.shape[0], _p(out))
    return out.tobytes()


def merkle_root(items: np.ndarray) -> bytes:
    items = np.ascontiguousarray(items, dtype=np.uint8)
    out = np.zeros(32, np.uint8)
    n = items.shape[0] if items.ndim == 2 else 0
    il = items.shape[1] if items.ndim == 2 else 0
    lib().orc_merkle_root(_p(items) if items.size else None, n, il, _p(out))
    return out.tobytes()


def nmt_root(leaves, check_order=True):
    """leaves: list of equal-length namespaced byte strings. Returns (rc, 90-byte root)."""
    n = len(leaves)
    ln = len(leaves[0]) if n else NS
    buf = np.frombuffer(b"".join(leaves), np.uint8).copy() if n else np.zeros(1, np.uint8)
    out = np.zeros(NODE, np.uint8)
    rc = lib().orc_nmt_root(_p(buf), n, ln, _p(out), 1 if check_order else 0)
    return rc, out.tobytes()


def axis_root(cells: np.ndarray, k: int, axis: int, check_order=True):
    cells = np.ascontiguousarray(cells, dtype=np.uint8)
    out = np.zeros(NODE, np.uint8)
    share = cells.shape[1]
    rc = lib().orc_axis_root(_p(cells), share, k, axis, share, _p(out), 1 if check_order else 0)
    return rc, out.tobytes()


def extend_and_commit(ods: np.ndarray, want_eds=True):
    ods = np.ascontiguousarray(ods, dtype=np.uint8)
    k, _, share = ods.shape
    eds = np.zeros((2 * k, 2 * k, share), np.uint8) if want_eds else None
    rr = np.zeros((2 * k, NODE), np.uint8)
    cr = np.zeros((2 * k, NODE), np.uint8)
    dah = np.zeros(32, np.uint8)
    rc = lib().orc_extend_and_commit(_p(ods), k, share, _p(eds) if want_eds else None, _p(rr), _p(cr),
                                     _p(dah))
    if rc:
        raise ValueError(f"orc_extend_and_commit rc={rc}")
    return eds, rr, cr, dah.tobytes()


def repair(eds: np.ndarray, present: np.ndarray, row_roots, col_roots, want_shares=False, order=0):
    """rsmt2d Repair restatement (eds.c). Returns (rc, eds, present, (axis, index)), plus
    (byz_shares (W, share), byz_present (W,)) when want_shares. order 0 = rsmt2d's sweep
    (row i, then column i); 1 = all rows, then all columns (tests only)."""
    eds = np.ascontiguousarray(eds, dtype=np.uint8).copy()
    present = np.ascontiguousarray(present, dtype=np.uint8).copy()
    w, _, share = eds.shape
    ba, bi = ctypes.c_int32(-1), ctypes.c_int32(-1)
    bs = np.zeros((w, share), np.uint8)
    bp = np.zeros(w, np.uint8)
    rc = lib().orc_repair_order(_p(eds), _p(present), w // 2, share, _p(np.ascontiguousarray(row_roots)),
                                _p(np.ascontiguousarray(col_roots)), ctypes.byref(ba), ctypes.byref(bi), _p(bs),
                                _p(bp), int(order))
    if want_shares:
        return rc, eds, present, (ba.value, bi.value), (bs, bp)
    return rc, eds, present, (ba.value, bi.value)


def gf(field):
    l = lib()
    n = 1 << field
    exp = np.array([l.orc_gf_exp(field, i) for i in range(min(n, 1 << 16))])
    return exp


def extend_commit_many(ods_batch: np.ndarray) -> np.ndarray:
    """CPU baseline: (n, k, k, share) ODSs on parallel threads -> (n, 32) DAHs."""
    ods_batch = np.ascontiguousarray(ods_batch, dtype=np.uint8)
    n, k, _, share = ods_batch.shape
    out = np.zeros((n, 32), np.uint8)
    rc = lib().orc_extend_commit_many(_p(ods_batch), n, k, share, _p(out))
    if rc:
        raise ValueError(f"orc_extend_commit_many rc={rc}")
    return out


def repair_many(eds: np.ndarray, present: np.ndarray, row_roots, col_roots, n: int) -> np.ndarray:
    """CPU baseline: n repairs of copies of one damaged square on parallel threads."""
    eds = np.ascontiguousarray(eds, dtype=np.uint8)
    present = np.ascontiguousarray(present, dtype=np.uint8)
    w, _, share = eds.shape
    st = np.zeros(n, np.int32)
    lib().orc_repair_many(_p(eds), _p(present), w // 2, share, _p(np.ascontiguousarray(row_roots)),
                          _p(np.ascontiguousarray(col_roots)), n, _p(st))
    return st
