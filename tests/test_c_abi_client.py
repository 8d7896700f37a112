"""The C ABI from plain C (tests/c_abi_client.c), as the cgo stub binds it: the header
compiles as C99 with gcc and the client links against libcelestia_eds.so. Here (no GPU)
the client must get CEL_EDEVICE from cel_ctx_create (no CPU fallback); on the MI355X it
checks the k = 2 DAH known answer, the DAH-only call and the power-of-two error string, then
cel_extend_batch_multi (two ctxs) and cel_extend_sharded (k = 256) as the Go Group calls them."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "celestia-app_amd")


def _build(tmp):
    exe = os.path.join(tmp, "c_abi_client")
    subprocess.check_call(["gcc", "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror", "-I",
                           os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "c_abi_client.c"), "-o", exe,
                           "-L", LIBDIR, "-lcelestia_eds", f"-Wl,-rpath,{LIBDIR}"])
    return exe


def test_c_client_without_device(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present: test_gpu_c_client covers it")
    p = subprocess.run([_build(str(tmp_path))], capture_output=True, text=True, timeout=120)
    assert p.returncode == 2, p.stdout + p.stderr


@pytest.mark.gpu
def test_gpu_c_client(tmp_path):
    p = subprocess.run([_build(str(tmp_path))], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
