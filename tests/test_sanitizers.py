"""Host-code sanitizers.

GPU AddressSanitizer / XNACK runs are not available on this pool, so the
sanitizers go where host-side pointer arithmetic lives: the shared-memory
transport (csrc/host/shm_comm.cpp) is built with ``-fsanitize=address,undefined``
together with a driver (tests/native/shm_sanitize.cpp) that forks W ranks and
runs every collective on known data. Any ASan/UBSan report fails the test.
"""
import os
import shutil
import subprocess

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "san")
SRCS = [os.path.join(ROOT, "tests", "native", "shm_sanitize.cpp"), os.path.join(CSRC, "host", "shm_comm.cpp")]
HDRS = [os.path.join(CSRC, "host", "shm_comm.h"), os.path.join(CSRC, "host", "cpu_reduce.h")]


def _build() -> str:
    exe = os.path.join(BUILD, "shm_sanitize")
    if os.path.exists(exe) and os.path.getmtime(exe) > max(os.path.getmtime(p) for p in SRCS + HDRS):
        return exe
    os.makedirs(BUILD, exist_ok=True)
    tdir = os.path.dirname(torch.__file__)
    inc, lib = os.path.join(tdir, "include"), os.path.join(tdir, "lib")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-static-libasan", "-static-libubsan",
           "-Wno-deprecated-declarations", "-Wno-attributes",
           f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}",
           f"-I{CSRC}", f"-I{inc}", f"-I{os.path.join(inc, 'torch', 'csrc', 'api', 'include')}",
           *SRCS, "-o", exe + ".tmp", f"-L{lib}", "-ltorch_cpu", "-lc10", f"-Wl,-rpath,{lib}", "-lpthread", "-lrt"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout + r.stderr[-6000:]
    os.replace(exe + ".tmp", exe)
    return exe


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("world", [2, 3, 4])
def test_shm_transport_under_asan_and_ubsan(world):
    exe = _build()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, str(world)], capture_output=True, text=True, timeout=600, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-6000:]
    assert f"OK: 0 of {world} ranks failed" in r.stdout
