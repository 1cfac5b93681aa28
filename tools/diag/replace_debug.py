"""Diagnostic: positions where the replace decode differs from the oracle, relative to chunks."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from decentralizepy_amd import codec  # noqa: E402
from oracle import fold as ofold  # noqa: E402

dev = torch.device("cuda", 0)
for n, k in ((100_003, 1000), (1_000_003, 10_000)):
    g = torch.Generator().manual_seed(3)
    loc = torch.randn(n, generator=g)
    idx = torch.sort(torch.randperm(n, generator=g)[:k])[0].to(torch.int32)
    val = torch.randn(k, generator=g)
    out = codec.replace(loc.to(dev), idx.to(dev), val.to(dev)).cpu().numpy()
    ref = ofold.replace(loc.numpy(), idx.numpy(), val.numpy())
    bad = np.nonzero(out.view(np.uint32) != ref.view(np.uint32))[0]
    print(n, k, "mismatches", len(bad))
    pos = {int(i): j for j, i in enumerate(idx.numpy())}
    for b in bad[:20]:
        j = pos.get(int(b))
        print(f"  elem {b} (mod4 {b % 4}) entry {j} chunk {None if j is None else j // 64} "
              f"lane {None if j is None else j % 64} out {out[b]} ref {ref[b]} local {loc[b].item()}")
