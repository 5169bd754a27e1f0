#!/usr/bin/env python3
"""Does a hipGraph capture change the launch cost of later eager kernels on this
runtime? One process, no collectives: 16 tiny torch kernels per step, eager
before a capture, replayed, and eager after. Prints one JSON line."""
import json
import time

import torch


def main():
    dev = torch.device("cuda", 0)
    xs = [torch.zeros(1024, device=dev) for _ in range(16)]

    def step():
        for x in xs:
            x.add_(1.0)

    def timed(fn, iters=200):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        return round((time.perf_counter() - t0) / iters / 16 * 1e6, 2)

    out = {"eager_us_per_op": timed(step)}
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        step()
    out["replay_us_per_op"] = timed(g.replay)
    out["eager_after_us_per_op"] = timed(step)
    del g
    torch.cuda.synchronize()
    out["eager_after_graph_deleted_us_per_op"] = timed(step)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
