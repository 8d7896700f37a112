"""CPU: the C-ABI library loads and exports exactly what include/celestia_eds.h
declares (no compute calls: there is no GPU here)."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "celestia_eds.h")
LIB = os.path.join(ROOT, "celestia-app_amd", "libcelestia_eds.so")


def header_symbols():
    text = open(HEADER).read()
    return set(re.findall(r"^\s*(?:[a-zA-Z_][\w\s\*]*?)\b(cel_\w+)\s*\(", text, re.M))


def test_library_built():
    assert os.path.exists(LIB), "run `make -C celestia-app_amd` (or __graft_entry__.build())"


def test_exports_match_header():
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB], text=True)
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln and ln.split()[-1].startswith("cel_")}
    declared = header_symbols()
    assert declared, "no declarations parsed"
    assert declared == exported, (declared - exported, exported - declared)


def test_binding_declares_every_export():
    import celestia_eds._lib as L
    assert set(L.EXPORTS) == header_symbols()
    lib = L.load()
    for name in L.EXPORTS:
        assert hasattr(lib, name)


def test_device_independent_entry_points():
    import celestia_eds._lib as L
    lib = L.load()
    assert lib.cel_codec_name().decode() == "Leopard"
    assert lib.cel_codec_max_chunks() == 32768 * 32768
    assert lib.cel_codec_validate_chunk_size(512) == L.OK
    assert lib.cel_codec_validate_chunk_size(100) == L.ECHUNK
    assert lib.cel_codec_validate_chunk_size(0) == L.OK  # rsmt2d: chunkSize % 64 != 0 only
    assert lib.cel_strerror(L.ENOTPOW2).decode().startswith("number of shares is not a power of 2")
    assert lib.cel_strerror(L.EBADROOT).decode() == "bad root input"
    assert lib.cel_dev_workspace_size(128, 1) > 0


def test_status_codes_match_header():
    """Every CEL_E* code of the header equals the binding's constant: the Go shim keys its
    fallback to the reference path on CEL_ETOOBIG and its errors on the rest, so the
    numbers are part of the ABI (strerror texts included)."""
    import celestia_eds._lib as L
    codes = dict(re.findall(r"^#define CEL_(OK|E[A-Z]+) (\d+)", open(HEADER).read(), re.M))
    assert {k: int(v) for k, v in codes.items()} == {k: getattr(L, k) for k in codes}
    assert int(codes["ETOOBIG"]) == 4 and int(codes["ENODATA"]) == 14
    lib = L.load()
    assert lib.cel_strerror(L.ENODATA).decode() == "no shard data"
    assert lib.cel_strerror(L.ETOOBIG).decode() == "square too large for the device path"


def test_gfx950_code_object():
    """The library carries a gfx950 code object in its HIP fat binary."""
    data = open(LIB, "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in data


def test_multi_gpu_entry_points_validate_without_a_device():
    """The multi-GPU and probe entry points reject missing contexts and outputs before any
    device or RCCL call (no GPU here): CEL_EINVAL, and a NULL plan handle back."""
    import ctypes
    import celestia_eds._lib as L
    lib = L.load()
    h = ctypes.c_void_p(123)
    assert lib.cel_shard_plan_create(None, 1, 256, 0, ctypes.byref(h)) == L.EINVAL
    assert h.value is None
    assert lib.cel_shard_plan_create(None, 1, 256, 0, None) == L.EINVAL
    null_ctxs = (ctypes.c_void_p * 2)(None, None)
    assert lib.cel_shard_plan_create(null_ctxs, 2, 256, 0, ctypes.byref(h)) == L.EINVAL
    assert lib.cel_extend_sharded(None, 1, None, 256, 512, None, None, None, None, 0) == L.EINVAL
    assert lib.cel_extend_batch_multi(None, 2, None, 1, 64, 512, None, None, None, None, None, 0) == L.EINVAL
    assert lib.cel_extend_batch_multi(null_ctxs, 2, None, 1, 64, 512, None, None, None, None, None, 0) == L.EINVAL
    assert lib.cel_shard_plan_run(None) == L.EINVAL
    assert lib.cel_shard_plan_upload(None, None) == L.EINVAL
    assert lib.cel_shard_plan_wait(None, None, None, None, None) == L.EINVAL
    assert lib.cel_shard_plan_transport(None) == b""
    lib.cel_shard_plan_destroy(None)
    d = ctypes.c_double()
    assert lib.cel_probe_sha256(None, ctypes.byref(d), None) == L.EINVAL
    assert lib.cel_probe_hbm_copy(None, 1 << 20, ctypes.byref(d)) == L.EINVAL
    assert lib.cel_probe_rs_transform(None, 128, ctypes.byref(d)) == L.EINVAL
