"""The cross-GPU memory model of the IPC kernels, checked in the machine code
that ships (verdict r1 weak #3). The gfx950 code objects embedded in the built
extension are disassembled; the protocol (dev_common.h, K4 "write-through
hand-off") requires, in every IPC kernel:

  1. every byte a peer reads is stored system-coherent: staging stores are
     ``global_store_dwordx4 ... sc0 sc1`` (written through to memory);
  2. every peer read is system-coherent: every LDS-DMA load of staging is
     ``global_load_lds_dwordx4 ... sc0 sc1`` (misses every cache, so no
     invalidate is needed on the reading GPU);
  3. before each flag store (``global_store_dword ... sc0 sc1``) the data stores
     are drained (``s_waitcnt vmcnt(0)``) and the workgroup has met (``s_barrier``)
     -- the MI355X compiler hazard (MI355X_MICROARCH.md) drops waits it thinks
     redundant, which is why the drain is inline asm;
  4. the peers' flags are polled with system-scope loads (``global_load_dword ... sc0 sc1``).

Runs on the CPU box (llvm-objcopy + llvm-objdump from ROCm, no GPU)."""
import os
import re
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _so():
    from pytorch_distributed_collective_communication_amd._build import ext_path

    p = ext_path()
    if not os.path.exists(p):
        pytest.skip("extension not built (python -m pytorch_distributed_collective_communication_amd._build)")
    if not os.path.exists(os.path.join(LLVM, "llvm-objdump")):
        pytest.skip("ROCm llvm-objdump not available")
    return p


def _code_objects(so, tmp):
    fat = os.path.join(tmp, "fatbin.bin")
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "-O", "binary", "--only-section=.hip_fatbin", so, fat],
                   check=True)
    b = open(fat, "rb").read()
    out, pos = [], 0
    while True:
        i = b.find(MAGIC, pos)
        if i < 0:
            return out
        (num,) = struct.unpack_from("<Q", b, i + 24)
        p = i + 32
        for _ in range(num):
            off, size, tl = struct.unpack_from("<QQQ", b, p)
            p += 24
            triple = b[p:p + tl].decode()
            p += tl
            if "gfx950" in triple and size:
                out.append(b[i + off:i + off + size])
        pos = i + len(MAGIC)


@pytest.fixture(scope="module")
def kernels(tmp_path_factory):
    so = _so()
    tmp = str(tmp_path_factory.mktemp("isa"))
    funcs = {}
    for k, co in enumerate(_code_objects(so, tmp)):
        path = os.path.join(tmp, f"co{k}.elf")
        open(path, "wb").write(co)
        txt = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", path], check=True,
                             capture_output=True, text=True).stdout
        name = None
        for line in txt.splitlines():
            m = re.match(r"^[0-9a-f]+ <(\S+)>:$", line)
            if m:
                name = m.group(1)
                funcs[name] = []
            elif name and line.startswith("\t"):
                funcs[name].append(line.split("//")[0].strip())
    assert funcs, "no gfx950 code object found in the extension"
    return funcs


def _ipc_kernels(funcs):
    ks = {n: body for n, body in funcs.items() if "k_ipc_reduce" in n or "k_ipc_copy" in n}
    assert len(ks) >= 7 * 2, sorted(funcs)[:20]  # at least copy + one reduce family for W = 2..8
    return ks


def _is_data_store(ins):
    return ins.startswith("global_store_dwordx") or ins.startswith("global_store_b") or \
        ins.startswith("global_store_short") or ins.startswith("buffer_store")


def _check_barriers(name, body):
    stores16 = [s for s in body if s.startswith("global_store_dwordx4")]
    assert any(s.endswith("sc0 sc1") for s in stores16), f"{name}: no system-coherent staging store"
    ldma = [s for s in body if s.startswith("global_load_lds_dwordx4")]
    assert ldma and all(s.endswith("sc0 sc1") for s in ldma), \
        f"{name}: LDS-DMA loads of peer staging must be sc0 sc1: {[s for s in ldma if not s.endswith('sc0 sc1')][:3]}"
    flags = [i for i, s in enumerate(body) if s.startswith("global_store_dword ") and s.endswith("sc0 sc1")]
    assert flags, f"{name}: no system-scope flag store"
    polls = [i for i, s in enumerate(body) if s.startswith("global_load_dword ") and s.endswith("sc0 sc1")]
    assert polls, f"{name}: no system-scope flag poll"
    checked = 0
    for f in flags:
        # back to the previous data store (or the kernel start): a drain and a barrier must lie between
        j = f - 1
        while j >= 0 and not _is_data_store(body[j]):
            j -= 1
        seg = body[j + 1:f]
        if j < 0 or not body[j].startswith("global_store_dwordx4"):
            continue  # error-word stores after a timeout, or flags before any payload (BARRIER)
        checked += 1
        assert any(x.startswith("s_waitcnt") and "vmcnt(0)" in x for x in seg), \
            f"{name}: flag store at {f} not behind a vmcnt(0) drain of the payload stores"
        assert any(x == "s_barrier" for x in seg), f"{name}: flag store at {f} not behind the workgroup barrier"
    assert checked, f"{name}: no flag store follows a payload store (checker found nothing to check)"


def test_every_ipc_kernel_orders_cross_gpu_handoffs(kernels):
    for name, body in _ipc_kernels(kernels).items():
        _check_barriers(name, body)


def test_lds_dma_engine_in_the_shipped_kernels(kernels):
    # K1/K2 and the IPC kernels stream through LDS with global_load_lds
    names = [n for n in kernels if "k1_reduce_lds" in n or "k2_multi_copy" in n or "k_ipc_" in n]
    assert names
    for n in names:
        assert any(s.startswith("global_load_lds_dwordx4") for s in kernels[n]), n
