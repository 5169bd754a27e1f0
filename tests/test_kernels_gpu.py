"""Numerics of the gfx950 kernels vs plain-PyTorch references (1 GPU).

K1 reduce_nway: every op x dtype x source count, ragged sizes (tails that are
not a multiple of the 16-B vector or the 4-KiB tile), the LDS-DMA engine, the
register-staged variant and the streaming kernel (normal and non-temporal). Bitwise for MAX/MIN/integers; SUM/PROD/AVG in
low precision compared against an fp32-accumulated reference.
K2 multi_copy / pack / unpack: ragged lists, mixed dtypes.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

SIZES = [1, 3, 1023, 4096, 4099, 65536 + 17, (1 << 20) + 5]
FLOAT_OPS = ["sum", "avg", "prod", "min", "max"]
INT_OPS = FLOAT_OPS + ["band", "bor", "bxor"]


def _ops():
    from pytorch_distributed_collective_communication_amd import ops

    return ops


def _rand(n, dt, dev, k):
    g = torch.Generator(device="cpu").manual_seed(1234 + k)
    if dt.is_floating_point:
        x = torch.rand(n, generator=g) * 2 - 1
        if k % 2:
            x = x * 3
        return x.to(dt).to(dev)
    if dt == torch.bool:
        return (torch.rand(n, generator=g) > 0.5).to(dev)
    lo, hi = (-50, 50) if dt in (torch.int8, torch.int32, torch.int64) else (0, 100)
    return torch.randint(lo, hi, (n,), generator=g, dtype=torch.int64).to(dt).to(dev)


@pytest.mark.parametrize("impl", ["lds", "regs", "lds_ntl", "stream", "stream_ntl"])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16, torch.float64])
@pytest.mark.parametrize("nsrc", [1, 2, 3, 5, 8])
def test_reduce_nway_float(dt, nsrc, impl):
    ops = _ops()
    dev = torch.device("cuda", 0)
    for n in SIZES:
        srcs = [_rand(n, dt, dev, k) for k in range(nsrc)]
        for op in FLOAT_OPS:
            if op == "prod" and dt in (torch.bfloat16, torch.float16):
                srcs_p = [s.clamp(-1.5, 1.5) for s in srcs]
            else:
                srcs_p = srcs
            got = ops.reduce_nway(srcs_p, op=op, impl=impl)
            ref = ops.reduce_nway_reference(srcs_p, op)
            if op in ("min", "max"):
                assert torch.equal(got, ref), (op, n)
            else:
                tol = {torch.float32: 1e-5, torch.float64: 1e-12, torch.bfloat16: 1e-2, torch.float16: 2e-3}[dt]
                torch.testing.assert_close(got, ref, rtol=tol, atol=tol, msg=lambda m: f"{op} n={n}: {m}")


@pytest.mark.parametrize("dt", [torch.int32, torch.int64, torch.int8, torch.uint8])
@pytest.mark.parametrize("nsrc", [2, 4, 7])
def test_reduce_nway_int(dt, nsrc):
    ops = _ops()
    dev = torch.device("cuda", 0)
    for n in SIZES[:6]:
        srcs = [_rand(n, dt, dev, k) for k in range(nsrc)]
        for op in INT_OPS:
            got = ops.reduce_nway(srcs, op=op)
            ref = ops.reduce_nway_reference(srcs, op)
            assert torch.equal(got, ref), (op, n, dt)


def test_reduce_nway_bool_and_nan():
    ops = _ops()
    dev = torch.device("cuda", 0)
    a = _rand(5000, torch.bool, dev, 0)
    b = _rand(5000, torch.bool, dev, 1)
    assert torch.equal(ops.reduce_nway([a, b], op="sum"), a | b)
    assert torch.equal(ops.reduce_nway([a, b], op="prod"), a & b)
    x = torch.tensor([1.0, float("nan"), 3.0, -1.0] * 1024, device=dev)
    y = torch.tensor([2.0, 0.0, float("nan"), -2.0] * 1024, device=dev)
    m = ops.reduce_nway([x, y], op="max")
    assert torch.isnan(m[1::4]).all() and torch.isnan(m[2::4]).all()
    assert torch.equal(m[0::4], torch.full_like(m[0::4], 2.0))
    xb = x.to(torch.bfloat16)
    assert torch.isnan(ops.reduce_nway([xb, xb], op="sum")[1::4]).all()


def test_reduce_nway_in_place_aliasing():
    ops = _ops()
    dev = torch.device("cuda", 0)
    a = torch.randn(300000, device=dev)
    b = torch.randn(300000, device=dev)
    ref = a + b
    ops.reduce_nway([a, b], out=a)
    torch.testing.assert_close(a, ref)


@pytest.mark.parametrize("max_blocks", [1, 7, 0])
def test_reduce_nway_grid_sizes(max_blocks):
    ops = _ops()
    dev = torch.device("cuda", 0)
    srcs = [torch.randn(1 << 18, device=dev) for _ in range(3)]
    torch.testing.assert_close(ops.reduce_nway(srcs, max_blocks=max_blocks), srcs[0] + srcs[1] + srcs[2])


def test_multi_copy_pack_unpack():
    ops = _ops()
    dev = torch.device("cuda", 0)
    sizes = [1, 4, 1000, 4096, 4097, 123457, 0, 65536]
    parts = [torch.randn(max(n, 1), device=dev)[:n] if n else torch.empty(0, device=dev) for n in sizes]
    parts = [p.contiguous() for p in parts]
    flat = ops.pack(parts)
    assert flat.numel() == sum(p.numel() * 4 for p in parts)
    assert torch.equal(flat.view(torch.float32), torch.cat(parts))
    back = [torch.empty_like(p) for p in parts]
    ops.unpack(flat, back)
    for a, b in zip(parts, back):
        assert torch.equal(a, b)
    # mixed dtypes
    mixed = [torch.arange(33, dtype=torch.int64, device=dev), torch.randn(77, device=dev).half(),
             torch.randint(0, 255, (4099,), dtype=torch.uint8, device=dev)]
    f2 = ops.pack([m for m in mixed])
    back2 = [torch.empty_like(m) for m in mixed]
    ops.unpack(f2, back2)
    for a, b in zip(mixed, back2):
        assert torch.equal(a, b)


def test_multi_copy_many_descriptors():
    ops = _ops()
    dev = torch.device("cuda", 0)
    srcs = [torch.full((513 + i,), float(i), device=dev) for i in range(150)]  # > 64 per launch
    dsts = [torch.empty_like(s) for s in srcs]
    ops.multi_copy(srcs, dsts)
    for s, d in zip(srcs, dsts):
        assert torch.equal(s, d)


def test_kernel_errors_are_loud():
    ops = _ops()
    dev = torch.device("cuda", 0)
    a = torch.randn(100, device=dev)
    with pytest.raises(RuntimeError):
        ops.reduce_nway([a, a[1:]], op="sum")
    with pytest.raises(RuntimeError):
        ops.reduce_nway([a.float(), a.float()], op="band")
    with pytest.raises(ValueError):
        ops.reduce_nway([a], op="nope")


def test_issue_order_across_streams():
    # two streams, one communicator's issue order: the op on stream B must see stream A's
    # earlier op even though A is held back by a long sleep kernel
    import pytorch_distributed_collective_communication_amd as pdcc

    C = pdcc._load_native()
    for shared in (False, True):
        o = C.IssueOrder(dry=False)
        if shared:
            o.add_user()
        a, b = torch.cuda.Stream(), torch.cuda.Stream()
        x = torch.zeros(1 << 20, device="cuda")
        torch.cuda.synchronize()
        with torch.cuda.stream(a):
            o.enter(a.cuda_stream)
            torch.cuda._sleep(50_000_000)
            x.fill_(1.0)
            o.leave(a.cuda_stream)
        with torch.cuda.stream(b):
            o.enter(b.cuda_stream)
            y = x.clone()
            o.leave(b.cuda_stream)
        torch.cuda.synchronize()
        assert bool(torch.all(y == 1.0)), shared
        assert o.waits() == 1
