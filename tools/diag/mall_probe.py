"""Diagnostic: does a 64 MB re-read right after a read hit the 256 MiB Infinity Cache?
Times torch copies (plain loads / stores) of one 64 MB source, cold (after a 1 GiB flush) and
again right after, with and without other 64 MB streams in between."""
import json
import torch

dev = torch.device("cuda", 0)
n = 16_777_216
a = torch.randn(n, device=dev)
b = torch.empty_like(a)
c = torch.empty_like(a)
d = torch.randn(n, device=dev)
flush = torch.empty(256 * 2 ** 20, device=dev)  # 1 GiB


def t(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3


res = {k: [] for k in ("cold", "warm", "warm_after_64MB_read", "warm_after_128MB_rw",
                       "sum_cold", "sum_warm")}
for _ in range(20):
    flush.fill_(1.0)
    res["cold"].append(t(lambda: b.copy_(a)))
    res["warm"].append(t(lambda: c.copy_(a)))
    flush.fill_(1.0)
    b.copy_(a)
    s = d.sum()
    res["warm_after_64MB_read"].append(t(lambda: c.copy_(a)))
    flush.fill_(1.0)
    b.copy_(a)
    torch.add(d, 1.0, out=b)
    res["warm_after_128MB_rw"].append(t(lambda: c.copy_(a)))
    flush.fill_(1.0)
    res["sum_cold"].append(t(lambda: a.sum()))
    res["sum_warm"].append(t(lambda: a.sum()))
print(json.dumps({k: round(sorted(v)[len(v) // 2], 2) for k, v in res.items()}))
