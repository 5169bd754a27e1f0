#!/usr/bin/env python3
"""Probe the HIP runtime facts the zero-copy IPC path relies on (torch's bundled
libamdhip64, the runtime our extension binds to):

* HIP_POINTER_ATTRIBUTE_BUFFER_ID names an allocation uniquely: a caching-allocator
  segment freed and re-allocated at the SAME base gets a different id;
* hipIpcGetMemHandle on a segment base: host cost per call and whether repeated
  exports leak file descriptors (dmabuf IPC mode);
* hipPointerGetAttribute / hipMemGetAddressRange host cost.

Prints one JSON line.
"""
import ctypes
import json
import os
import time

import torch

HIP_POINTER_ATTRIBUTE_BUFFER_ID = 7


def main():
    torch.cuda.init()
    lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    out = {}

    def rng(p):
        base = ctypes.c_void_p()
        size = ctypes.c_size_t()
        e = lib.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(size), ctypes.c_void_p(p))
        return e, base.value, size.value

    def bid(p):
        v = ctypes.c_uint64(0)
        e = lib.hipPointerGetAttribute(ctypes.byref(v), HIP_POINTER_ATTRIBUTE_BUFFER_ID, ctypes.c_void_p(p))
        return e, v.value

    def handle(p):
        h = (ctypes.c_char * 64)()
        e = lib.hipIpcGetMemHandle(h, ctypes.c_void_p(p))
        return e, bytes(h)

    def nfd():
        return len(os.listdir("/proc/self/fd"))

    x = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
    e, base1, size1 = rng(x.data_ptr() + 4096)
    out["range"] = [e, base1 == x.data_ptr(), size1]
    out["id_base"] = bid(base1)
    out["id_inner"] = bid(x.data_ptr() + 12345)
    eh, h1 = handle(base1)
    out["handle_err"] = eh
    del x
    torch.cuda.empty_cache()
    y = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
    e, base2, size2 = rng(y.data_ptr())
    out["realloc_same_base"] = base2 == base1
    out["id_realloc"] = bid(base2)
    out["id_differs_after_realloc"] = out["id_realloc"][1] != out["id_base"][1]
    eh2, h2 = handle(base2)
    out["handle_differs_after_realloc"] = h1 != h2
    # costs
    fd0 = nfd()
    t0 = time.perf_counter()
    for _ in range(200):
        handle(base2)
    out["ipc_get_handle_us"] = round((time.perf_counter() - t0) / 200 * 1e6, 2)
    out["fd_growth_per_200_exports"] = nfd() - fd0
    t0 = time.perf_counter()
    for _ in range(2000):
        bid(y.data_ptr())
    out["buffer_id_us"] = round((time.perf_counter() - t0) / 2000 * 1e6, 2)
    t0 = time.perf_counter()
    for _ in range(2000):
        rng(y.data_ptr())
    out["address_range_us"] = round((time.perf_counter() - t0) / 2000 * 1e6, 2)
    # two tensors carved out of one caching-allocator segment share an id
    a = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
    b = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
    out["small_pair_same_segment"] = rng(a.data_ptr())[1] == rng(b.data_ptr())[1]
    out["small_pair_same_id"] = bid(a.data_ptr())[1] == bid(b.data_ptr())[1]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
