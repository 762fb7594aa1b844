"""Device-to-device copy rates of a few torch kernels (HIP events, best of 5),
to pick the stream-copy reference bench.py's roofline quotes beside 8 TB/s.

    python tools/copy_peak.py
"""
import json

import torch


def rate(fn, nbytes, reps=5):
    fn()
    torch.cuda.synchronize()
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    return round(2.0 * nbytes / (best * 1e-3) / 1e9, 1)


def main():
    dev = torch.device("cuda:0")
    out = {}
    for nbytes in (1 << 30, 4 << 30):
        a = torch.ones(nbytes // 4, dtype=torch.float32, device=dev)
        b = torch.empty_like(a)
        out[f"copy_{nbytes >> 30}G"] = rate(lambda: b.copy_(a), nbytes)
        out[f"mul1_{nbytes >> 30}G"] = rate(lambda: torch.mul(a, 1.0, out=b), nbytes)
        out[f"add0_{nbytes >> 30}G"] = rate(lambda: torch.add(a, 0.0, out=b), nbytes)
        a4 = a.view(-1, 4)
        b4 = b.view(-1, 4)
        out[f"copy4_{nbytes >> 30}G"] = rate(lambda: b4.copy_(a4), nbytes)
        del a, b, a4, b4
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
