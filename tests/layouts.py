"""Adversarial input layouts for the sampled top-k path (decentralizepy_amd/csrc/dpz_topk_sampled.hip):
positions that its sample kernel never reads, mirrored from its constants."""
import numpy as np

SMP_CHUNK = 64     # contiguous elements per sample chunk
SMP_NCHUNK = 1024  # chunks, spread evenly over [0, n)


def sample_starts(n):
    return [(c * (n - SMP_CHUNK)) // (SMP_NCHUNK - 1) for c in range(SMP_NCHUNK)]


def miss_layout(n, k, seed=11):
    """x (x0 = 0): tiny changes everywhere, and more than k large ones placed only in the gaps
    between sample chunks, so the sample sees none of them and the window misses the k-th key."""
    rng = np.random.default_rng(seed)
    starts = sample_starts(n)
    per_gap = -(-int(1.15 * k) // (len(starts) - 1))
    big = []
    for s, e in zip(starts[:-1], starts[1:]):
        lo = s + SMP_CHUNK + 100
        assert e - 100 - lo > per_gap, "gap too small for the layout"
        big.extend(range(lo, lo + per_gap))
    big = np.array(big)
    x = (1e-6 * rng.standard_normal(n)).astype(np.float32)
    x[big] = rng.uniform(1.0, 2.0, big.shape[0]).astype(np.float32)
    return x, np.zeros(n, dtype=np.float32)
