"""The cross-GPU memory model of the IPC kernels, checked in the machine code
that ships (verdict r1 weak #3): the gfx950 code objects embedded in the built
extension are disassembled and every cross-GPU barrier (dev_common.h
block_barrier, K4) must

  1. write back the L2 at system scope (``buffer_wbl2 sc0 sc1``) and WAIT for it
     (``s_waitcnt vmcnt(0)``) before the flag store -- the MI355X compiler hazard
     (MI355X_MICROARCH.md "Compiler hazard") drops that wait unless it is inline asm;
  2. store the flag and poll the peers' flags with system-scope accesses
     (``global_store_dword / global_load_dword ... sc0 sc1``: uncached, past L2);
  3. invalidate at system scope (``buffer_inv sc0 sc1``) after the poll, and wait
     for the invalidate, before any peer data is read.

The kernels read their arguments from LDS (a gated zero-copy launch swaps peer buffers in
there), typed as global pointers (dev_common.h ``gp``), so no access may be a flat one.

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


def _compressed_code_objects(b, tmp):
    """The gfx950 code objects of compressed bundles ("CCOB", clang --offload-compress, the default build):
    each bundle's header holds its total size; clang-offload-bundler inflates and unbundles it."""
    out, pos, k = [], 0, 0
    while True:
        i = b.find(b"CCOB", pos)
        if i < 0:
            return out
        ver = struct.unpack_from("<H", b, i + 4)[0]
        total = struct.unpack_from("<Q" if ver >= 3 else "<I", b, i + 8)[0]
        src, dst = os.path.join(tmp, f"bundle{k}.ccob"), os.path.join(tmp, f"bundle{k}.co")
        open(src, "wb").write(b[i:i + total])
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={src}", f"--output={dst}"], check=True)
        out.append(open(dst, "rb").read())
        pos, k = i + max(total, 4), k + 1


def _code_objects(so, tmp):
    fat = os.path.join(tmp, "fatbin.bin")
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "-O", "binary", "--only-section=.hip_fatbin", so, fat],
                   check=True)
    b = open(fat, "rb").read()
    if b.find(MAGIC) < 0 and b.find(b"CCOB") >= 0:
        return _compressed_code_objects(b, tmp)
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


def _check_barriers(name, body):
    wbl = [i for i, s in enumerate(body) if s == "buffer_wbl2 sc0 sc1"]
    inv = [i for i, s in enumerate(body) if s == "buffer_inv sc0 sc1"]
    # the zero-copy gate (dev_common.h gate_wait): an acquire right after the 8-byte system-scope
    # poll of the host-published slot's seq -- nothing is released before it (the host wrote it)
    gate = [i for i in inv if any(body[j].startswith("global_load_dwordx2 ") and body[j].endswith("sc0 sc1")
                                  for j in range(max(0, i - 3), i))]
    assert gate, f"{name}: no system-scope acquire after the gate poll"
    inv = [i for i in inv if i not in gate]
    assert wbl, f"{name}: no system-scope L2 write-back"
    assert len(wbl) == len(inv), f"{name}: {len(wbl)} releases vs {len(inv)} acquires"
    for w in wbl:
        # the flag store: first system-scope store after the release
        f = next(i for i in range(w + 1, len(body))
                 if body[i].startswith("global_store_dword ") and body[i].endswith("sc0 sc1"))
        assert any(body[i].startswith("s_waitcnt") and "vmcnt(0)" in body[i] for i in range(w + 1, f)), \
            f"{name}: flag store at +{f - w} not behind a vmcnt(0) wait after buffer_wbl2"
        # the poll: system-scope load after the flag store, and the acquire after it
        p = next(i for i in range(f + 1, len(body))
                 if body[i].startswith("global_load_dword ") and body[i].endswith("sc0 sc1"))
        a = next((i for i in inv if i > p), None)
        assert a is not None, f"{name}: no buffer_inv sc0 sc1 after the poll at {p}"
        nxt = body[a + 1:a + 4]
        assert any(s.startswith("s_waitcnt") and "vmcnt(0)" in s for s in nxt), \
            f"{name}: the system-scope invalidate is not waited for: {nxt}"


def test_every_ipc_kernel_orders_cross_gpu_handoffs(kernels):
    for name, body in _ipc_kernels(kernels).items():
        _check_barriers(name, body)


def test_lds_dma_engine_in_the_shipped_kernels(kernels):
    # K1/K2 and the IPC kernels stream through LDS with global_load_lds
    names = [n for n in kernels if "k1_reduce_lds" in n or "k2_multi_copy" in n or "k_ipc_" in n]
    assert names
    for n in names:
        assert any(s.startswith("global_load_lds_dwordx4") for s in kernels[n]), n


def test_no_scratch_in_the_hot_kernels(kernels):
    # a register spill, a private copy of the kernel-argument view (e.g. a reference to it kept in a
    # struct) or an out-of-line device call puts state in scratch and turns peer pointers into flat
    # ones -- check it never ships
    names = [n for n in kernels if "k1_reduce" in n or "k2_multi_copy" in n or "k_ipc_" in n]
    assert names
    for n in names:
        bad = [s for s in kernels[n] if s.startswith(("scratch_", "flat_", "s_swappc"))]  # spills, flat, calls
        assert not bad, (n, bad[:4])


def test_ll_allreduce_words_are_single_stores_and_uncached_polls(kernels):
    # LL (csrc/kernels/reduce_impl.h k_ll_allreduce / k_ll_allgather): each {data, epoch} word must reach the
    # peer as ONE 8-byte system-scope store (single-copy atomic: a poller never sees new
    # data with an old epoch or the reverse), and the poll must read 8 bytes at system
    # scope (uncached, past L2); no scratch, flat accesses or calls
    # (and the rooted k_ll_reduce / k_ll_rooted: data one way, token lines on the other pairs)
    # (and k_ll_reduce_scatter / k_ll_alltoall: chunk q pushed to rank q)
    ks = {n: b for n, b in kernels.items() if any(k in n for k in ("k_ll_allreduce", "k_ll_allgather", "k_ll_reduce",
                                                                 "k_ll_rooted", "k_ll_alltoall"))}
    assert sum("k_ll_allgather" in n for n in ks) == 7, sorted(ks)  # all-gather: one per W = 2..8
    assert sum("k_ll_rooted" in n for n in ks) == 7, sorted(ks)  # broadcast / gather / scatter: one per W
    assert sum("11k_ll_reduceI" in n for n in ks) >= 7, sorted(ks)  # (mangled: not k_ll_reduce_scatter)
    assert sum("k_ll_reduce_scatter" in n for n in ks) >= 7, sorted(ks)
    assert sum("k_ll_alltoall" in n for n in ks) == 7, sorted(ks)
    assert len(ks) >= 28, sorted(kernels)[:20]
    for name, body in ks.items():
        stores = [s for s in body if s.startswith("global_store_dwordx2") and s.endswith("sc0 sc1")]
        polls = [s for s in body if s.startswith("global_load_dwordx2") and s.endswith("sc0 sc1")]
        assert stores and polls, (name, [s for s in body if "sc0 sc1" in s][:8])
        bad = [s for s in body if s.startswith(("scratch_", "flat_", "s_swappc"))]
        assert not bad, (name, bad[:4])
        # the data words never go out as wider stores that could tear across the epoch
        wide = [s for s in body if s.startswith(("global_store_dwordx4", "global_store_dwordx3")) and "sc0 sc1" in s]
        assert not wide, (name, wide[:4])
