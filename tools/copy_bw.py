#!/usr/bin/env python3
"""Reference HBM rates on this box for the byte mix of the pre-process launches (diagnostic).

Times torch's elementwise copy / fill / sum over buffers of a given size, cycling a pool of sets larger
than the 256 MiB Infinity Cache (as bench.py does) or re-using one set (resident), with HIP events.
Prints one JSON line per measurement. Usage: python tools/copy_bw.py [--mb 100] [--sets 5]
"""
import argparse
import json

import torch


def timed(fn, steps, sets):
    for k in range(2 * sets):
        fn(k % sets)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for t in range(steps):
        fn(t % sets)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, default=100.0)
    ap.add_argument("--sets", type=int, default=5)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    n = int(a.mb * 1e6) // 4
    for sets in (a.sets, 1):
        src = [torch.randn(n, device="cuda") for _ in range(sets)]
        dst = [torch.empty(n, device="cuda") for _ in range(sets)]
        acc = torch.empty((), device="cuda")
        for name, fn, nbytes in (
                ("copy", lambda k: dst[k].copy_(src[k]), 8 * n),
                ("fill", lambda k: dst[k].fill_(1.0), 4 * n),
                ("sum", lambda k: torch.sum(src[k], dim=0, out=acc), 4 * n)):
            s = timed(fn, a.steps, sets)
            print(json.dumps({"op": name, "sets": sets, "MB": round(nbytes / 1e6, 1), "us": round(s * 1e6, 2),
                              "TBps": round(nbytes / s / 1e12, 3)}), flush=True)
        del src, dst


if __name__ == "__main__":
    main()
