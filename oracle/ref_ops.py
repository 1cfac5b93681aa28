"""The reference's own CPU op sequence for the top-k path — TEST/BASELINE INFRASTRUCTURE ONLY.

This is what ``bench.py`` times as ``cpu_baseline`` (kind "port"): the exact ATen-CPU calls the
reference issues per encode and per decode, on torch CPU tensors, without any of this build's
code.  It exists because the reference itself cannot travel to the GPU box.

* encode = ``PartialModel._pre_step`` (flatten, change; ``sharing/PartialModel.py:312-331``) +
  ``extract_top_gradients`` (``:177-185``: abs, std_mean, topk(sorted=True), sort) +
  ``serialized_model`` bookkeeping (``:207-246``: counter[idx] += 1, values x[idx], int32 cast).
* decode = ``PartialModel.deserialized_model`` (``:283-295``: cat of the local state,
  ``T[idx] = params``).
"""
import numpy as np
import torch


def encode(x, x0, alpha, counter):
    change = x - x0                                                    # PartialModel.py:320
    g = torch.abs(change)                                              # :177
    std, mean = torch.std_mean(g, unbiased=False)                      # :178
    _, index = torch.topk(g, round(alpha * g.shape[0]), dim=0, sorted=True)  # :181-183
    index, _ = torch.sort(index)                                       # :185
    counter[index] += 1                                                # :207
    vals = x[index]                                                    # :231
    return index.numpy().astype(np.int32), vals.numpy()                # :242-244


def decode(local, indices, params):
    t = torch.cat([local])                                             # :292 (one-tensor model)
    t[torch.tensor(indices, dtype=torch.long)] = torch.tensor(params)  # :293-295
    return t
