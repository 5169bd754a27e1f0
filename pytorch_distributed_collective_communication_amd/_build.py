"""In-tree native build: gfx950 HIP kernels + C++ backend -> ``_C*.so``.

Explicit ``hipcc``/``g++`` command lines (no hipify, no JIT cache): the kernels
in ``csrc/kernels/*.hip`` are compiled for ``--offload-arch=gfx950`` only, the
host C++ (c10d backend, shm transport, RCCL/IPC communicators, bindings) with
``g++`` against the torch headers, and everything is linked against torch's own
bundled HIP/RCCL (``torch/lib``) so the extension binds to the same runtime
torch already loaded (SURVEY.md §7.1 "runtime duality").

Usage: ``python -m pytorch_distributed_collective_communication_amd._build [-j N] [--force]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
CSRC = os.path.join(ROOT, "csrc")
# PDCC_OFFLOAD_COMPRESS=1 (default): the gfx950 code objects go into the fat binary compressed
# (clang --offload-compress; the runtime inflates them when the library loads): the .so shrinks ~6x
COMPRESS = os.environ.get("PDCC_OFFLOAD_COMPRESS", "1") not in ("0", "")
BUILD = os.path.join(ROOT, "build", "objz" if COMPRESS else "obj")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PDCC_ARCH", "gfx950")


SAN_DIR = os.path.join(ROOT, "build", "san_ext")
SAN_FLAGS = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize=vptr",
             "-fno-sanitize-recover=undefined"]


def ext_path(sanitize: bool = False) -> str:
    name = "_C" + sysconfig.get_config_var("EXT_SUFFIX")
    return os.path.join(SAN_DIR, name) if sanitize else os.path.join(PKG_DIR, name)


def asan_runtime() -> str:
    """The ASan runtime the sanitized extension links against (LD_PRELOAD it into Python)."""
    return subprocess.run(["g++", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()


def _torch_dirs():
    import torch

    tdir = os.path.dirname(torch.__file__)
    return tdir, os.path.join(tdir, "include"), os.path.join(tdir, "lib")


def _hipcc() -> str:
    p = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    if not os.path.exists(p):
        raise RuntimeError("hipcc not found (ROCm toolchain required to build the gfx950 kernels)")
    return p


def _sources():
    hip = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    cpp = sorted(
        glob.glob(os.path.join(CSRC, "host", "*.cpp"))
        + glob.glob(os.path.join(CSRC, "device", "*.cpp"))
        + glob.glob(os.path.join(CSRC, "backend", "*.cpp"))
        + [os.path.join(CSRC, "bindings.cpp")]
    )
    return hip, cpp


def _headers_mtime(sub: str) -> float:
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    if sub == "kernels":
        hs = [h for h in hs if os.sep + "kernels" + os.sep in h]
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _obj(src: str, sanitize: bool = False) -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
    # (the sanitized variant instruments the host C++ only: the gfx950 kernels are shared)
    return os.path.join(BUILD + ("_san" if sanitize and not src.endswith(".hip") else ""), rel + ".o")


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build step failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def build(jobs: int | None = None, force: bool = False, verbose: bool = False, sanitize: bool = False) -> str:
    """Compile (incrementally) and link the extension; returns the .so path. `sanitize`: the host C++
    with ASan + UBSan into build/san_ext/ (load it with PDCC_NATIVE_SO and the ASan runtime preloaded)."""
    tdir, tinc, tlib = _torch_dirs()
    import torch

    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(BUILD + "_san", exist_ok=True)
    os.makedirs(SAN_DIR, exist_ok=True)
    hip_srcs, cpp_srcs = _sources()
    py_inc = sysconfig.get_paths()["include"]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    common_defs = [
        "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DTORCH_EXTENSION_NAME=_C",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
    ]
    incs = [
        f"-I{CSRC}",
        f"-I{tinc}",
        f"-I{os.path.join(tinc, 'torch', 'csrc', 'api', 'include')}",
        f"-I{py_inc}",
        f"-I{os.path.join(ROCM, 'include')}",
    ]
    hipcc = _hipcc()
    jobs = jobs or min(8, os.cpu_count() or 4)
    kern_hdr = _headers_mtime("kernels")
    all_hdr = _headers_mtime("all")

    def stale(src, obj, hdr):
        if force or not os.path.exists(obj):
            return True
        t = os.path.getmtime(obj)
        return t < os.path.getmtime(src) or t < hdr

    tasks = []
    for s in hip_srcs:
        o = _obj(s, sanitize)
        if stale(s, o, kern_hdr):
            tasks.append(
                [hipcc, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", f"-I{CSRC}"]
                + (["--offload-compress"] if COMPRESS else []) + ["-c", s, "-o", o]
            )
    for s in cpp_srcs:
        o = _obj(s, sanitize)
        if stale(s, o, all_hdr):
            tasks.append(
                ["g++"] + (SAN_FLAGS if sanitize else ["-O2", "-g0"])
                + ["-fPIC", "-std=c++17", "-Wno-deprecated-declarations", "-Wno-attributes"]
                + common_defs
                + incs
                + ["-c", s, "-o", o]
            )
    if tasks:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = [ex.submit(_run, t, verbose) for t in tasks]
            for f in futs:
                f.result()

    objs = [_obj(s, sanitize) for s in hip_srcs + cpp_srcs]
    out = ext_path(sanitize)
    if force or tasks or not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(o) for o in objs):
        link = (
            ["g++", "-shared"] + (["-fsanitize=address,undefined"] if sanitize else []) + ["-o", out + ".tmp"]
            + objs
            + [
                f"-L{tlib}",
                f"-L{os.path.join(ROCM, 'lib')}",
                "-lc10",
                "-lc10_hip",
                "-ltorch",
                "-ltorch_cpu",
                "-ltorch_hip",
                "-ltorch_python",
                f"-Wl,-rpath,{tlib}",
                # torch's bundled runtime first: the extension must bind to the HIP/RCCL torch loaded
                os.path.join(tlib, "libamdhip64.so"),
                os.path.join(tlib, "librccl.so"),
                "-lrt",
                "-lpthread",
                "-ldl",
            ]
        )
        _run(link, verbose)
        os.replace(out + ".tmp", out)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--sanitize", action="store_true", help="ASan + UBSan host build into build/san_ext/")
    a = ap.parse_args(argv)
    p = build(a.jobs, a.force, a.verbose, a.sanitize)
    print(p)


if __name__ == "__main__":
    main(sys.argv[1:])
