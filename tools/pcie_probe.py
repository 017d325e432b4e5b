"""PCIe ceiling for the end-to-end (pinned host) path: H2D alone, D2H alone, both at once on
two streams, and the same split into many small copies.  Prints one JSON line (GB/s)."""
import json
import time

import torch


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    dev = torch.device("cuda", 0)
    nin, nout = 276 << 20, 129 << 20
    h_in = torch.empty(nin, dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(nout, dtype=torch.uint8, pin_memory=True)
    d_in = torch.empty(nin, dtype=torch.uint8, device=dev)
    d_out = torch.empty(nout, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def h2d():
        with torch.cuda.stream(s1):
            d_in.copy_(h_in, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            h_out.copy_(d_out, non_blocking=True)

    def both():
        h2d()
        d2h()

    def many(k):
        def f():
            with torch.cuda.stream(s1):
                for c in range(k):
                    a, b = nin * c // k, nin * (c + 1) // k
                    d_in[a:b].copy_(h_in[a:b], non_blocking=True)
            with torch.cuda.stream(s2):
                for c in range(k):
                    a, b = nout * c // k, nout * (c + 1) // k
                    h_out[a:b].copy_(d_out[a:b], non_blocking=True)
        return f

    r = {}
    t = timed(h2d)
    r["h2d_gb_s"] = round(nin / t / 1e9, 1)
    t = timed(d2h)
    r["d2h_gb_s"] = round(nout / t / 1e9, 1)
    t = timed(both)
    r["both_ms"] = round(t * 1e3, 3)
    r["both_gb_s"] = round((nin + nout) / t / 1e9, 1)
    for k in (8, 64, 136):
        t = timed(many(k))
        r[f"both_{k}copies_ms"] = round(t * 1e3, 3)
    print(json.dumps(r))


if __name__ == "__main__":
    main()
