"""Practical HBM rates on the box for the complex-output kernel's traffic mix (context for the
roofline fraction): pure write (fill), 1:1 copy, and a 1:2 read:write pattern
(read a buffer once, write it twice) at the bench's sizes (11.5 GB in, 23 GB out)."""
import json

import torch


def rate(fn, nbytes, iters=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / iters
    return {"ms": ms, "GBps": nbytes / ms / 1e6}


n_in = 11_520_000_000 // 4
x = torch.ones(n_in, device="cuda", dtype=torch.float32)
y = torch.empty(2 * n_in, device="cuda", dtype=torch.float32)
y2 = y.view(n_in, 2)
res = {
    "fill_23GB": rate(lambda: y.fill_(1.0), y.numel() * 4),
    "copy_11.5GB": rate(lambda: y[:n_in].copy_(x), 2 * x.numel() * 4),
    "read1_write2_34.6GB": rate(lambda: y2.copy_(x.view(n_in, 1).expand(n_in, 2)), 3 * x.numel() * 4),
}
print(json.dumps(res))
