#!/usr/bin/env python
"""HBM write-only and copy rates on one MI355X (torch fill_ / copy_), the
ceilings a write-heavy launch such as the config-5 rollout (1.1 GB written, 20 MB
read per launch) runs against."""
import json
import torch

dev = torch.device("cuda", 0)
for mb in (1024, 4096):
    n = mb * 2**20 // 4
    a = torch.empty(n, device=dev)
    b = torch.empty(n, device=dev)
    for name, fn, bytes_ in (("fill", lambda: a.fill_(1.0), n * 4), ("copy", lambda: b.copy_(a), n * 8)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print(json.dumps({"op": name, "mb": mb, "ms": round(ms, 4), "tb_s": round(bytes_ / ms / 1e9, 3)}), flush=True)
    del a, b
