"""Secondary workloads of bench.py: C3 (JWINS wavelet + top-k, 16-payload
batched decode + weighted average), C5 (256 MiB, 0.1 % top-k, fp16 value packing) and the
PCIe-inclusive end-to-end rate (the reference path starts and ends in host memory: pyzmq socket
buffers / CPU model parameters).

Every function times whole steps with the device already holding what a node keeps resident
across rounds (init_model, accumulated changes, counters); inputs are synthetic (device PRNG).
Node states rotate so each step streams its inputs from HBM, not the 256 MiB Infinity Cache.
"""
import math
import os
import time

import numpy as np
import torch

L3_BYTES = 256 * 2 ** 20


def _cpu_leg(make_step, units_per_step, unit_bytes, sample, seconds=12.0, scale=1.0,
             full_affinity=True):
    """cpu_baseline of a workload: the reference's op sequence (oracle/ref_round.py,
    oracle/ref_ops.py — test infrastructure, imported by the callers' CPU legs only) timed on this
    box's host cores.  ``make_step()`` builds the inputs once and returns a step function; steps
    repeat until ``seconds`` (at least one), at torch's intra-op threads (the job's CPU share) and,
    when the step is short enough, at every CPU of the affinity mask.  ``scale``: the step is a
    bounded sample of the workload's unit (e.g. 1 of 16 nodes): time x scale = one unit.
    value = unit_bytes / (median time x scale) in GiB/s."""
    import os

    step = make_step()

    def run(threads, budget):
        prev = torch.get_num_threads()
        torch.set_num_threads(threads)
        try:
            times = []
            t_start = time.perf_counter()
            while True:
                t0 = time.perf_counter()
                step()
                times.append(time.perf_counter() - t0)
                if time.perf_counter() - t_start > budget:
                    break
        finally:
            torch.set_num_threads(prev)
        return sorted(times)[len(times) // 2], len(times)

    cores = torch.get_num_threads()
    step()  # warm: first-touch of the inputs, the thread pool
    t, nsteps = run(cores, seconds)
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    res = {"value": round(unit_bytes / (t * scale) / 2 ** 30, 5), "unit": "GiB/s",
           "cores": cores, "kind": "port", "host_cpu_count": os.cpu_count(),
           "affinity_cpus": affinity, "seconds_per_unit": round(t * scale, 4),
           "units_per_step": units_per_step,
           "sample": f"{sample}; median of {nsteps} step(s) at {cores} torch threads (the job's "
                     f"CPU share)" + (f", x{scale:g} to one unit" if scale != 1 else "")}
    if full_affinity and affinity and affinity > cores and t < 0.6:
        tf, nf = run(affinity, seconds / 3)
        res["full_affinity"] = {"threads": affinity, "steps": nf,
                                "value": round(unit_bytes / (tf * scale) / 2 ** 30, 5),
                                "unit": "GiB/s",
                                "note": "every CPU of the affinity mask (shared host)"}
    elif full_affinity and affinity and affinity <= cores:
        res["full_affinity"] = {"threads": affinity, "value": res["value"],
                                "note": "the job's threads are every CPU of the affinity mask"}
    elif full_affinity:
        res["full_affinity"] = {"threads": affinity, "value": None,
                                "note": f"not timed: one step takes {t:.2f} s at {cores} threads "
                                        "(the 64 MiB headline's full-affinity leg measured 20x "
                                        "slower than its 16-thread leg on a shared host)"}
    return res


def _host_payloads(m, k, npay, seed, dtype=np.float32):
    """npay sorted, duplicate-free random index sets of about k entries over [0, m) with values
    (host numpy, for the CPU legs)."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(npay):
        idx = np.unique(rng.integers(0, m, size=int(k * 1.12) + 8))[:k].astype(np.int32)
        out.append((idx, rng.standard_normal(idx.shape[0]).astype(dtype)))
    return out


def cpu_wavelet_round(n, alpha, npay, seed, level=4, wavelet="sym2", scale=1.0, seconds=10.0,
                      what="one JWINS node round"):
    """cpu_baseline of the wavelet rounds: oracle/ref_round.py wavelet_node (the reference's ATen
    ops, pywt's sym2 / haar as the NumPy restatement) on one node's N-parameter model."""
    def make():
        from oracle import ref_round
        from oracle import wavelet as owav
        g = torch.Generator().manual_seed(seed)
        x = torch.randn(n, generator=g)
        x0 = x - 0.01 * torch.randn(n, generator=g)
        m = owav.coeff_len(n, level, wavelet)
        acc = 0.01 * torch.randn(m, generator=g)
        cnt = torch.zeros(m, dtype=torch.int32)
        pays = _host_payloads(m, round(alpha * m), npay, seed)
        w = [1 / (npay + 1)] * npay
        return lambda: ref_round.wavelet_node(x, x0, acc, alpha, cnt, pays, w, level, wavelet)
    return _cpu_leg(make, 1, 4 * n, f"{what}: oracle/ref_round.py wavelet_node, N={n}, "
                                    f"{wavelet} level {level}, alpha={alpha}, {npay} payloads "
                                    f"(ATen ops + the NumPy pywt restatement)",
                    seconds=seconds, scale=scale)


def cpu_partial_round(n, alpha, npay, seed, fp16=False, scale=1.0, seconds=10.0,
                      what="one PartialModel node round"):
    """cpu_baseline of the PartialModel rounds: oracle/ref_round.py partial_node (encode + the MH
    fold of npay payloads; npay = 0: encode + the replace decode of one payload, C5 / C2 shape)."""
    def make():
        from oracle import ref_ops, ref_round
        g = torch.Generator().manual_seed(seed)
        x = torch.randn(n, generator=g)
        x0 = x - 0.01 * torch.randn(n, generator=g)
        cnt = torch.zeros(n, dtype=torch.int32)
        if npay == 0:
            def step():
                idx, vals = ref_ops.encode(x, x0, alpha, cnt)
                if fp16:
                    vals = torch.from_numpy(vals).half().float().numpy()
                ref_ops.decode(x0, idx, vals)
            return step
        pays = _host_payloads(n, round(alpha * n), npay, seed,
                              dtype=np.float16 if fp16 else np.float32)
        w = [1 / (npay + 1)] * npay
        return lambda: ref_round.partial_node(x, x0, alpha, cnt, pays, w, fp16=fp16)
    shape = (f"{npay} payloads MH-folded" if npay else "encode + replace decode")
    return _cpu_leg(make, 1, 4 * n, f"{what}: oracle/ref_round.py, N={n}, alpha={alpha}, "
                                    f"{shape}{', fp16 values' if fp16 else ''}",
                    seconds=seconds, scale=scale)


def _sync_time(fn, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        fn(i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def c3_case(dev, n=25_000_000, alpha=0.01, npay=16, steps=40, warmup=5, seed=3, wavelet="sym2",
            cpu=True):
    """C3: one JWINS node round on an N-parameter model (reference Wavelet.py:142-329 with the
    tutorial/JWINS/config.ini settings change_based_selection, accumulation and
    accumulate_averaging_changes on): encode = W(x), W(x - x0) in one DWT launch, top-k of
    |W(x - x0) + acc| (PartialModel.py:322-327: change += acc), counter += 1 and acc rewind at
    the selected coefficients, values from W(x); decode = 16 neighbour payloads replaced +
    Metro-Hastings-folded in the wavelet domain in one batched launch (w = 1/17 each, self
    1 - 16/17), one IDWT launch back to N parameters; post-step = acc += W(x_new - prev)
    (PartialModel.py:346-349, one accumulating DWT launch).
    The product path (the Wavelet plugin and gossip_jwins with accumulate_averaging_changes)
    keeps the bookkeeping coalesced: dpz_topk_encode_sliced adds the selection to a bit-sliced
    counter and writes a selection mask, and the post-step's DWT applies the rewind
    (dpz_dwt_sym2_rewind); ``scattered_ms_per_step`` times the same round with the reference's
    scattered counter[idx] += 1 / acc[idx] = 0 inside the encode (dpz_topk_encode).
    Algorithmic bytes: B_enc = 8N + 8M + 12k (+ acc 8M read), B_dec = 4M + 4N +
    8 n k (+ 8M fold write / IDWT read), B_post = 8N + 8M."""
    from decentralizepy_amd import codec
    level = 4
    m = codec.wavedec_len(n, level, wavelet)
    k = round(alpha * m)
    nw = codec.mask_words(m)
    per_set = 4 * (3 * n + 4 * m) + 8 * k + 4 * 33 * nw
    R = max(2, math.ceil(2 * L3_BYTES / per_set) + 1)
    g = torch.Generator(device=dev).manual_seed(seed)
    sets = []
    for _ in range(R):
        x = torch.randn(n, device=dev, generator=g)
        sets.append(dict(x=x, x0=x - 0.01 * torch.randn(n, device=dev, generator=g),
                         acc=0.01 * torch.randn(m, device=dev, generator=g),
                         cnt=torch.zeros(m, dtype=torch.int32, device=dev),
                         planes=torch.zeros(32 * nw, dtype=torch.int32, device=dev),
                         mask=torch.zeros(nw, dtype=torch.int32, device=dev),
                         wx=torch.empty(m, device=dev), wc=torch.empty(m, device=dev),
                         idx=torch.empty(k, dtype=torch.int32, device=dev),
                         val=torch.empty(k, device=dev), tot=torch.empty(m, device=dev),
                         out=torch.empty(n, device=dev)))
    # 16 received payloads (fixed, distinct index sets)
    pays = []
    for j in range(npay):
        idx = torch.sort(torch.randperm(m, device=dev, generator=g)[:k])[0].to(torch.int32)
        pays.append((idx, torch.randn(k, device=dev, generator=g)))
    w = [1 / (npay + 1)] * npay
    wt = 0.0
    for v in w:
        wt += v
    w_self = 1 - wt
    ws = codec.Workspace(dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    mode = {"sliced": True}
    # BENCH_HINT=1: the key window from the previous encode's exact threshold (DPZ_TOPK_HINT, no
    # sample launch).  Off by default: this synthetic round's post-step adds W(fold - x0) to the
    # accumulator every step (the fold mixes in unit-scale random payloads), so the k-th key moves
    # by more than the window's +-1/16 from step to step and every hinted encode misses (measured
    # on MI355X: fell_back on every line, filter 92-95 us with the window's extra candidates)
    hint = {"on": os.environ.get("BENCH_HINT", "0") == "1"}

    def encode(d):
        codec.wavedec(d["x"], level, x0=d["x0"], coeffs_x=d["wx"], coeffs_diff=d["wc"],
                      wavelet=wavelet)
        if mode["sliced"]:
            codec.topk_encode_sliced(d["wc"], k, d["mask"], d["planes"], acc=d["acc"],
                                     acc_mode=codec.DPZ_ACC_ADD, vals_src=d["wx"],
                                     idx_out=d["idx"], val_out=d["val"], workspace=ws,
                                     status_out=st, hint=hint["on"])
        else:
            codec.topk_encode(d["wc"], k, acc=d["acc"], acc_mode=codec.DPZ_ACC_ADD,
                              vals_src=d["wx"], counter=d["cnt"], idx_out=d["idx"],
                              val_out=d["val"], workspace=ws, asynchronous=True,
                              hint=hint["on"])

    def decode(d):
        codec.decode_average(d["wx"], pays, w, w_self, out=d["tot"], workspace=ws)
        codec.waverec(d["tot"], n, level, out=d["out"], wavelet=wavelet)

    def post(d):
        # acc += W(x_new - prev) (prev = init_model = x0; the synthetic states keep their x0)
        codec.wavedec(d["out"], level, x0=d["x0"], want_x=False, coeffs_diff=d["acc"],
                      accumulate=True, wavelet=wavelet,
                      rewind_mask=d["mask"] if mode["sliced"] else None)

    def step(i):
        d = sets[i % R]
        encode(d)
        decode(d)
        post(d)

    for i in range(max(warmup, R)):
        step(i)
    t_step = _sync_time(step, steps)
    t_enc = _sync_time(lambda i: encode(sets[i % R]), steps)
    t_dec = _sync_time(lambda i: decode(sets[i % R]), steps)
    t_post = _sync_time(lambda i: post(sets[i % R]), steps)
    torch.cuda.synchronize()
    # any missed encode of the timed steps (the sticky word ORs every call's status)
    fb = int(st.item()) != 0 or codec.topk_sticky_status(ws) != 0
    with codec.KernelTimer() as kt:
        torch.cuda._sleep(int(100e6))
        for i in range(R * 2):
            step(i)
        torch.cuda.synchronize()
    kern = {nm: round(ms / c * 1e3, 2) for nm, (ms, c) in kt.result.items()}
    mode["sliced"] = False
    for i in range(R):
        step(i)
    t_scat = _sync_time(step, steps)
    t_scat_enc = _sync_time(lambda i: encode(sets[i % R]), steps)
    with codec.KernelTimer() as kt2:
        torch.cuda._sleep(int(100e6))
        for i in range(R * 2):
            step(i)
        torch.cuda.synchronize()
    kern_scat = {nm: round(ms / c * 1e3, 2) for nm, (ms, c) in kt2.result.items()}
    fb = fb or codec.topk_status(ws) != 0
    b_enc = 8 * n + 8 * m + 8 * m + 12 * k  # x, x0 -> W(x), W(dx); read W(dx), acc; k triples
    b_dec = 4 * m + 4 * n + 8 * npay * k + 8 * m
    b_post = 8 * n + 8 * m  # read x_new, prev; acc read + write
    b = b_enc + b_dec + b_post
    res = dict(workload=f"C3: JWINS {wavelet} level-4 node round of an N={n} model (M={m} "
                         f"coefficients): DWT pair + top-k (accumulation), {npay}-payload batched "
                         f"decode + MH average + IDWT, accumulating post-step DWT",
                n=n, m=m, k=k, alpha=alpha, rotated_states=R,
                value=4 * n / t_step / 2 ** 30, ms_per_step=t_step * 1e3,
                encode_us=t_enc * 1e6, decode_us=t_dec * 1e6, post_us=t_post * 1e6,
                alg_bytes_enc=b_enc, alg_bytes_dec=b_dec, alg_bytes_post=b_post,
                step_frac_of_hbm_peak=b / t_step / 8e12, fell_back=fb,
                side_effects="coalesced (bit-sliced counter, rewind in the post-step DWT)",
                kernels_avg_us=kern,
                scattered_ms_per_step=t_scat * 1e3, scattered_encode_us=t_scat_enc * 1e6,
                scattered_step_frac_of_hbm_peak=b / t_scat / 8e12,
                scattered_kernels_avg_us=kern_scat)
    if cpu:
        res["cpu_baseline"] = cpu_wavelet_round(n, alpha, npay, seed, level, wavelet,
                                                seconds=8.0)
    return res


def c3_round_case(dev, rank, world, dist, n=25_000_000, rounds=10, warmup=2, seed=21,
                  wavelet="sym2", cpu=True):
    """C3 shape (b): the topology-faithful JWINS round of tutorial/JWINS/regular_16.txt (16 nodes
    of degree 3, copied under tests/golden/) with the tutorial config (sym2 level 4, alpha_list
    [0.1, 0.15, 0.2, 0.25, 0.3, 0.4, 1.0] drawn per node from random.seed(uid), metadata_cap
    0.5, accumulation + accumulate_averaging_changes): every node encodes (DWT pair, top-k with
    ADD accumulation, or a full share), payloads all-gathered over RCCL when world > 1, every
    node folds its 3 neighbours in the wavelet domain, IDWT, accumulating post-step
    (decentralizepy_amd/gossip_jwins.py).  The alpha draws are deterministic, so the timed rounds
    are the same sequence on every run.  Algorithmic bytes per node: DWT pair 8N + 8M; encode
    read W(dx), acc 8M + 20k (idx, val, counter r+w, acc rewind), or a 4M acc zeroing; fold 4M +
    payloads + 4M; IDWT 4M + 4N; post-step 8N + 8M; init_model copy 8N."""
    import os

    from decentralizepy_amd.gossip import read_edges, shard
    from decentralizepy_amd.gossip_jwins import JwinsRound
    here = os.path.dirname(os.path.abspath(__file__))
    adj = read_edges(os.path.join(here, "tests", "golden", "regular_16.edges"))
    lo, hi, _ = shard(len(adj), world, rank)
    g = torch.Generator(device=dev).manual_seed(seed + rank)
    x = torch.randn(hi - lo, n, device=dev, generator=g)
    eng = JwinsRound(adj, x, "[0.1,0.15,0.2,0.25,0.3,0.4,1.0]", rank=rank, world=world,
                     wavelet=wavelet, metadata_cap=0.5, device=dev)
    del x
    noise = 0.01 * torch.randn(hi - lo, n, device=dev, generator=g)
    m = eng.M
    times, alg = [], []
    for r in range(warmup + rounds):
        eng.x += noise
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        eng.step()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        dt = time.perf_counter() - t0
        if dist is not None:
            tt = torch.tensor([dt], device=dev, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            dt = float(tt.item())
        if r >= warmup:
            times.append(dt)
            b = 0
            for i in range(len(adj)):
                a = eng.alphas[i]
                k = round(a * m) if a < 0.5 else 0
                b += 8 * n + 8 * m + (8 * m + 20 * k if k else 4 * m)
                b += 8 * m + sum((8 * round(eng.alphas[q] * m) if eng.alphas[q] < 0.5 else 4 * m)
                                 for q in adj[i])
                b += 4 * m + 4 * n + 8 * n + 8 * m + 8 * n
            alg.append(b)
    t = sum(times) / len(times)
    b = sum(alg) / len(alg)
    res = dict(workload=f"C3 shape (b): JWINS round of regular_16 (16 nodes x degree 3), "
                         f"N={n} per node, {wavelet} level 4, tutorial alpha_list",
                n=n, m=m, nodes=len(adj), world=world, rounds=rounds,
                ms_per_round=t * 1e3, ms_per_round_min=min(times) * 1e3,
                value=len(adj) * 4 * n / t / 2 ** 30,
                alg_bytes_per_round=b, round_frac_of_hbm_peak=b / t / 8e12 / world,
                scaling="strong (16 nodes fixed)")
    if cpu and rank == 0:  # one node's round at the alpha list's median draw, x16 nodes
        res["cpu_baseline"] = cpu_wavelet_round(
            n, 0.2, 3, seed, 4, wavelet, scale=len(adj), seconds=8.0,
            what="one of the 16 nodes (alpha 0.2, the tutorial list's median draw; degree 3)")
        res["cpu_baseline"]["value"] = round(len(adj) * 4 * n / (
            res["cpu_baseline"]["seconds_per_unit"]) / 2 ** 30, 5)
        res["cpu_baseline"]["unit_note"] = "seconds_per_unit = one round of all 16 nodes"
    return res


def c5_case(dev, n=67_108_864, alpha=0.001, steps=40, warmup=5, seed=5, streams=3, cpu=True):
    """C5: 256 MiB fp32 tensor, 0.1 % top-k, payload values packed to fp16 (RNE, torch.half
    semantics) by the encode itself (DPZ_TOPK_VAL_FP16: compact writes the fp16 words, no
    packing launch); decode = fp16 unpack + replace.  B = 16N + 12k."""
    from decentralizepy_amd import codec
    k = round(alpha * n)
    per_set = 4 * n * 4 + 10 * k
    R = max(streams, math.ceil(2 * L3_BYTES / per_set) + 1)
    R = -(-R // streams) * streams
    g = torch.Generator(device=dev).manual_seed(seed)
    sets = []
    for _ in range(R):
        x = torch.randn(n, device=dev, generator=g)
        sets.append(dict(x=x, x0=x - 0.01 * torch.randn(n, device=dev, generator=g),
                         cnt=torch.zeros(n, dtype=torch.int32, device=dev),
                         idx=torch.empty(k, dtype=torch.int32, device=dev),
                         h=torch.empty(k, dtype=torch.float16, device=dev),
                         v32=torch.empty(k, device=dev), out=torch.empty(n, device=dev)))
    S = [torch.cuda.Stream(dev) for _ in range(streams)]
    W = [codec.Workspace(dev) for _ in range(streams)]

    def step_on(d, ws):
        codec.topk_encode(d["x"], k, x0=d["x0"], counter=d["cnt"], idx_out=d["idx"],
                          val_out=d["h"], workspace=ws, asynchronous=True, val_fp16=True)
        codec.unpack_fp16(d["h"], out=d["v32"])
        codec.replace(d["x0"], d["idx"], d["v32"], out=d["out"], workspace=ws)

    def step(i):
        step_on(sets[i % R], W[0])

    def step_multi(i):
        q = i % streams
        with torch.cuda.stream(S[q]):
            step_on(sets[i % R], W[q])

    for i in range(max(warmup, R)):
        step_multi(i)
    t_multi = _sync_time(step_multi, steps)
    t_one = _sync_time(step, steps)
    fb = codec.topk_status(W[0]) != 0
    b = 16 * n + 12 * k
    res = dict(workload=f"C5: N={n} (256 MiB) fp32, alpha={alpha} top-k, fp16 value packing",
               n=n, k=k, rotated_states=R, streams=streams,
               value=4 * n / t_multi / 2 ** 30, ms_per_step=t_multi * 1e3,
               one_node_ms_per_step=t_one * 1e3, alg_bytes=b,
               step_frac_of_hbm_peak=b / t_multi / 8e12, fell_back=fb)
    del sets
    torch.cuda.empty_cache()
    if cpu:
        res["cpu_baseline"] = cpu_partial_round(n, alpha, 0, seed, fp16=True,
                                                what="the C5 step (encode, fp16 values, decode)")
    return res


def e2e_case(dev, n, alpha, fp16=False, steps=20, warmup=3, seed=7, streams=3, cpu=True):
    """PCIe-inclusive rate: the node's flat model arrives from host memory (pinned, H2D 4N), the
    payload leaves for the socket (D2H 8k, or 6k with fp16 values); a received payload arrives
    (H2D) and the averaged model returns to host memory (D2H 4N) — the reference's Sharing path
    starts and ends in numpy buffers.  init_model / counters stay resident on the device.
    Reported for one node (one stream: every copy serialised with the kernels) and for
    `streams` concurrent nodes (H2D and D2H of different nodes overlap on the full-duplex link)."""
    from decentralizepy_amd import codec
    k = round(alpha * n)
    R = streams * 2
    g = torch.Generator(device=dev).manual_seed(seed)
    vdt = torch.float16 if fp16 else torch.float32
    sets = []
    for _ in range(R):
        x = torch.randn(n, device=dev, generator=g)
        d = dict(x=torch.empty(n, device=dev), x0=x - 0.01 * torch.randn(n, device=dev, generator=g),
                 cnt=torch.zeros(n, dtype=torch.int32, device=dev),
                 idx=torch.empty(k, dtype=torch.int32, device=dev),
                 val=torch.empty(k, device=dev), h=torch.empty(k, dtype=torch.float16, device=dev),
                 ridx=torch.empty(k, dtype=torch.int32, device=dev),
                 rval=torch.empty(k, dtype=vdt, device=dev), v32=torch.empty(k, device=dev),
                 out=torch.empty(n, device=dev),
                 hx=x.cpu().pin_memory(), hidx=torch.empty(k, dtype=torch.int32).pin_memory(),
                 hval=torch.empty(k, dtype=vdt).pin_memory(),
                 hout=torch.empty(n).pin_memory())
        sets.append(d)
    S = [torch.cuda.Stream(dev) for _ in range(streams)]
    W = [codec.Workspace(dev) for _ in range(streams)]

    def step_on(d, ws):
        d["x"].copy_(d["hx"], non_blocking=True)                       # model params in
        codec.topk_encode(d["x"], k, x0=d["x0"], counter=d["cnt"], idx_out=d["idx"],
                          val_out=d["val"], workspace=ws, asynchronous=True)
        v = codec.pack_fp16(d["val"], out=d["h"]) if fp16 else d["val"]
        d["hidx"].copy_(d["idx"], non_blocking=True)                   # payload out
        d["hval"].copy_(v, non_blocking=True)
        d["ridx"].copy_(d["hidx"], non_blocking=True)                  # a payload in
        d["rval"].copy_(d["hval"], non_blocking=True)
        rv = codec.unpack_fp16(d["rval"], out=d["v32"]) if fp16 else d["rval"]
        codec.replace(d["x0"], d["ridx"], rv, out=d["out"], workspace=ws)
        d["hout"].copy_(d["out"], non_blocking=True)                   # averaged model out

    def step(i):
        step_on(sets[i % R], W[0])

    def step_multi(i):
        q = i % streams
        with torch.cuda.stream(S[q]):
            step_on(sets[i % R], W[q])

    for i in range(max(warmup, R)):
        step_multi(i)
    t_one = _sync_time(step, steps)
    t_multi = _sync_time(step_multi, steps)
    pcie = 8 * n + (2 * (4 + (2 if fp16 else 4)) * k)
    res = dict(n=n, k=k, fp16_values=fp16, pcie_bytes_per_step=pcie,
               one_node_GiBps=4 * n / t_one / 2 ** 30, one_node_ms_per_step=t_one * 1e3,
               concurrent_GiBps=4 * n / t_multi / 2 ** 30, concurrent_ms_per_step=t_multi * 1e3,
               concurrent_pcie_GBps=pcie / t_multi / 1e9, streams=streams)
    del sets
    torch.cuda.empty_cache()
    if cpu:  # the reference's path is host-resident: no PCIe legs at all
        res["cpu_baseline"] = cpu_partial_round(n, alpha, 0, seed, fp16=fp16, seconds=6.0,
                                                what="the host-resident reference step")
    return res


def shard_case(dev, rank, world, dist, n=67_108_864, alpha=0.001, steps=20, warmup=3, seed=9,
               fp16=True, cpu=False, ops=None, unpack=None):
    """One tensor of N parameters sharded over the ranks (BASELINE config 5: 256 MiB
    on 8 GPUs, 0.1 % top-k, fp16 value packing): the global top-k with one all-gather of every
    rank's k candidates (decentralizepy_amd/shard.py; with ``fp16`` the local encodes write fp16
    values themselves and the candidates travel as 10 bytes), then each rank decodes the global
    payload into its own slice (fp16 unpack + replace; indices outside the slice fall outside
    [0, n_r) and are skipped).  Strong scaling: N fixed, value = N params / time."""
    from decentralizepy_amd import codec
    from decentralizepy_amd.shard import HipShardOps, sharded_replace, sharded_topk_encode
    k = round(alpha * n)
    lo = n * rank // world
    hi = n * (rank + 1) // world
    nl = hi - lo
    R = 3
    g = torch.Generator(device=dev).manual_seed(seed + rank)
    sets = []
    for _ in range(R):
        x = torch.randn(nl, device=dev, generator=g)
        sets.append(dict(x=x, x0=x - 0.01 * torch.randn(nl, device=dev, generator=g),
                         cnt=torch.zeros(nl, dtype=torch.int32, device=dev),
                         out=torch.empty(nl, device=dev)))
    # ops / unpack: injectable device steps (tests/test_cpu_bench_collectives.py runs this
    # function on gloo ranks with the oracle in place of the HIP codec)
    ops = ops or HipShardOps(dev)
    unpack = unpack or codec.unpack_fp16

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    def step(i):
        d = sets[i % R]
        idx, val = sharded_topk_encode(d["x"], d["x0"], k, lo, counter=d["cnt"], ops=ops,
                                       val_fp16=fp16)
        if fp16:
            val = unpack(val)
        sharded_replace(d["x0"], lo, idx, val, out=d["out"], ops=ops)

    for i in range(warmup):
        step(i)
    sync()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    sync()
    if dist is not None:
        dist.barrier()
    t = (time.perf_counter() - t0) / steps
    if dist is not None:
        tt = torch.tensor([t], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
    res = dict(workload=f"one N={n} tensor sharded over {world} GPU(s), alpha={alpha}"
                        f"{', fp16 values written by the encode' if fp16 else ''}: sharded "
                        f"top-k (one all-gather of {world} x {k} candidates) + slice decode",
               n=n, k=k, world=world, value=4 * n / t / 2 ** 30, ms_per_step=t * 1e3,
               scaling="strong")
    if cpu and rank == 0:  # the whole tensor on the host (the reference has no sharding)
        del sets
        res["cpu_baseline"] = cpu_partial_round(n, alpha, 0, seed, fp16=fp16,
                                                what="the whole tensor's step on the host")
    return res


def _lib_native(n):
    from decentralizepy_amd import _lib
    return _lib.lib().dpz_fft_native(int(n))


def fft_case(dev, n=11_000_000, alpha=0.01, npay=3, steps=30, warmup=5, seed=9, cpu=True):
    """The FFT sharing plugin's device round (reference sharing/JWINS/FFT.py:132-302) on an
    N-parameter model: encode = x - x0, rfft(x) and rfft(x - x0) (native kernels), |change|
    (complex), top-k on it with the counter, complex values gathered from rfft(x); decode = npay
    complex payloads folded (Metro-Hastings) over the (re, im) pairs, irfft (1/n in its last
    pass).  The step rate is reported on the GiB/s metric (4N bytes of model per step) with the
    kernels' average durations, and the transforms alone against the HBM roofline."""
    from decentralizepy_amd import codec
    m = n // 2 + 1
    k = round(alpha * m)
    g = torch.Generator(device=dev).manual_seed(seed)
    R = 3
    sets = []
    for _ in range(R):
        x = torch.randn(n, device=dev, generator=g)
        sets.append(dict(x=x, x0=x - 0.01 * torch.randn(n, device=dev, generator=g),
                         d=torch.empty(n, device=dev),
                         cnt=torch.zeros(m, dtype=torch.int32, device=dev),
                         out=torch.empty(n, device=dev)))
    pays = []
    for j in range(npay):
        idx = torch.sort(torch.randperm(m, device=dev, generator=g)[:k])[0].to(torch.int32)
        vals = torch.randn(2 * k, device=dev, generator=g)
        pays.append((codec.cplx_pair_indices(idx), vals))
    w = [1 / (npay + 1)] * npay
    wt = 0.0
    for v in w:
        wt += v
    ws = codec.Workspace(dev)

    def step(i):
        d = sets[i % R]
        codec.elementwise(codec.DPZ_EW_SUB, d["x"], d["x0"], out=d["d"])
        fx = codec.rfft(d["x"], workspace=ws)
        ch = codec.rfft(d["d"], workspace=ws)
        key = codec.cplx_key(ch)
        idx, _ = codec.topk_encode(key, k, counter=d["cnt"], workspace=ws, asynchronous=True)
        codec.cplx_gather(fx, idx)
        tot = codec.decode_average(fx.view(torch.float32), pays, w, 1 - wt, workspace=ws)
        codec.irfft(tot.view(torch.complex64), n, out=d["out"], workspace=ws)

    for i in range(warmup):
        step(i)
    t = _sync_time(step, steps)
    with codec.KernelTimer() as kt:
        for i in range(R):
            step(i)
        torch.cuda.synchronize()
    kern = {nm: round(ms / c * 1e3, 2) for nm, (ms, c) in kt.result.items()}
    # the transforms alone (event pairs around `reps` back-to-back calls on rotated inputs):
    # algorithmic bytes = the n reals read + the n / 2 + 1 complex written (and back for irfft)
    reps = 20
    spec = [codec.rfft(d["x"], workspace=ws) for d in sets]
    buf = [torch.empty_like(s_) for s_ in spec]

    def t_of(fn):
        fn(0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(reps):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    def inv(i):
        buf[i % R].copy_(spec[i % R])
        codec.irfft(buf[i % R], n, out=sets[i % R]["out"], workspace=ws)

    t_copy = t_of(lambda i: buf[i % R].copy_(spec[i % R]))
    t_r = t_of(lambda i: codec.rfft(sets[i % R]["x"], out=spec[i % R], workspace=ws))
    t_i = t_of(inv) - t_copy
    ab = 4 * n + 8 * m
    native = bool(_lib_native(n))
    res = dict(workload=f"FFT plugin round: rfft top-k encode + {npay}-payload complex fold + "
                        f"irfft of an N={n} model (M={m} coefficients)",
               n=n, m=m, k=k, alpha=alpha, value=4 * n / t / 2 ** 30, ms_per_step=t * 1e3,
               transforms=("native mixed-radix Stockham kernels (csrc/dpz_fft.hip)" if native
                           else "hipFFT fallback (a prime factor above 4096)"),
               kernels_avg_us=kern,
               rfft_us=round(t_r, 2), irfft_us=round(t_i, 2),
               roofline={"bound": "hbm", "kernel": "rfft (all its launches)",
                         "alg_bytes": ab, "achieved_GBps": round(ab / t_r / 1e3, 1),
                         "peak_GBps": 8000.0, "frac": round(ab / t_r / 1e3 / 8000.0, 4),
                         "irfft_frac": round(ab / t_i / 1e3 / 8000.0, 4),
                         "note": "algorithmic bytes 4N read + 8(N/2+1) written; the passes move "
                                 "each complex element once per pass (read + write)"})
    if cpu:
        def make():
            # the reference's FFT round on the host (sharing/JWINS/FFT.py:12-26 rfft transformer,
            # :132-148 apply_fft, :170-172 counter, :245-290 _averaging): torch.fft on CPU
            gq = torch.Generator().manual_seed(seed)
            x = torch.randn(n, generator=gq)
            x0 = x - 0.01 * torch.randn(n, generator=gq)
            cnt = torch.zeros(m, dtype=torch.int32)
            hp = _host_payloads(m, k, npay, seed)
            hp = [(torch.from_numpy(i).long(), torch.complex(torch.from_numpy(v),
                                                             torch.from_numpy(v)))
                  for i, v in hp]

            def step():
                fx = torch.fft.rfft(x)
                ch = torch.fft.rfft(x - x0)
                _, index = torch.topk(ch.abs(), k, dim=0, sorted=False)
                index, _ = torch.sort(index)
                fx[index]
                cnt[index] += 1
                total, wt_ = None, 0
                for (pi, pv), wv in zip(hp, w):
                    tk = fx.clone()
                    tk[pi] = pv
                    wt_ += wv
                    total = wv * tk if total is None else total + wv * tk
                total += (1 - wt_) * fx
                torch.fft.irfft(total, n)
            return step
        res["cpu_baseline"] = _cpu_leg(make, 1, 4 * n, f"the reference's FFT round (torch.fft "
                                                      f"on CPU), N={n}, {npay} payloads",
                                       seconds=8.0)
    return res


def wire_case(dev, n=11_000_000, alpha=0.01, reps=30, seed=13):
    """Device wire codecs on a C2 payload (k = 110,000 indices of an 11M model, fp32 values):
    Elias-gamma (the reference's byte format), LZ4 frames of the int32 gaps (Lz4Wrapper's index
    leg) and of the fp32 values, and the block-floating fp32 codec (EliasFpzip's value leg).
    Encode and decode are timed device-to-device (each call ends with its size read-back) and
    the wire bytes are reported against the raw int32 / fp32 legs.  cpu_baseline: liblz4 1.9.3
    (what python-lz4 wraps) on the same gaps, one host thread."""
    import numpy as np

    from decentralizepy_amd import codec
    k = round(alpha * n)
    g = torch.Generator(device=dev).manual_seed(seed)
    idx = torch.sort(torch.randperm(n, device=dev, generator=g)[:k])[0].to(torch.int32)
    vals = 0.01 * torch.randn(k, device=dev, generator=g)
    ws = codec.Workspace(dev)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            out = fn()
        torch.cuda.synchronize()
        return out, (time.perf_counter() - t0) / reps * 1e6

    res = {"k": k, "raw_idx_bytes": 4 * k, "raw_val_bytes": 4 * k}
    el, t = timed(lambda: codec.elias_encode(idx, workspace=ws))
    res["elias"] = {"bytes": int(el.numel()), "encode_us": round(t, 1)}
    # decode = what the receiving plugin runs: the host stream (from pickle) up to the device and
    # decoded into int32 indices there (compression/Elias.py decompress_device)
    from decentralizepy_amd.compression.Elias import Elias
    el_host = el.cpu().numpy()
    E = Elias()
    E._dev(dev)
    dec, t = timed(lambda: E.decompress_device(el_host, device=dev))
    assert torch.equal(dec, idx)
    res["elias"]["decode_us"] = round(t, 1)
    res["elias"]["decode_note"] = ("host bytes -> device int32 indices, H2D included "
                                   "(Elias.decompress_device)")
    gaps = codec.delta_i32(idx)
    fr, t = timed(lambda: codec.lz4_compress(gaps.view(torch.uint8), workspace=ws))
    frame = fr.cpu().numpy().tobytes()
    # decode = Lz4Wrapper.decompress's work (frame -> gaps -> running sum); decompress = the
    # frame alone
    _, td = timed(lambda: codec.running_sum_i32(
        codec.lz4_decompress(frame, dev, workspace=ws).view(torch.int32), dtype=torch.int32,
        workspace=ws))
    _, tf = timed(lambda: codec.lz4_decompress(frame, dev, workspace=ws))
    res["lz4_idx"] = {"bytes": len(frame), "encode_us": round(t, 1), "decode_us": round(td, 1),
                      "decompress_us": round(tf, 1)}
    fv, t = timed(lambda: codec.lz4_compress(vals.view(torch.uint8), workspace=ws))
    res["lz4_vals"] = {"bytes": int(fv.numel()), "encode_us": round(t, 1)}
    fz, t = timed(lambda: codec.fpz_encode(vals, 0, workspace=ws))
    res["fpz_vals"] = {"bytes": int(fz.numel()), "encode_us": round(t, 1)}
    try:  # cpu_baseline leg (test infrastructure: liblz4 through the oracle's ctypes binding)
        from oracle import lz4 as olz4
        gh = np.diff(idx.cpu().numpy(), prepend=0).astype(np.int32).tobytes()
        t0 = time.perf_counter()
        for _ in range(reps):
            cf = olz4.ref_compress(gh)
        te = (time.perf_counter() - t0) / reps * 1e6
        t0 = time.perf_counter()
        for _ in range(reps):
            olz4.ref_decompress(cf)
        tfc = (time.perf_counter() - t0) / reps * 1e6
        t0 = time.perf_counter()
        for _ in range(reps):  # Lz4Wrapper.decompress: frame, then np.cumsum of the gaps
            np.cumsum(np.frombuffer(olz4.ref_decompress(cf), dtype=np.int32))
        tdc = (time.perf_counter() - t0) / reps * 1e6
        res["cpu_baseline"] = {"kind": "liblz4 1.9.3 (python-lz4 default preferences)",
                               "cores": 1, "bytes": len(cf), "encode_us": round(te, 1),
                               "decode_us": round(tdc, 1), "decompress_us": round(tfc, 1)}
    except OSError:
        pass
    # the reference's own Elias decode (compression/Elias.py:54-97: a pure-Python walk over the
    # codes), restated in oracle/elias.py and timed on one host thread (cpu_baseline leg)
    from oracle import elias as oelias
    t0 = time.perf_counter()
    ref = oelias.decode(el_host)
    res["elias"]["cpu_reference_decode_us"] = round((time.perf_counter() - t0) * 1e6, 1)
    t0 = time.perf_counter()
    oelias.encode(idx.cpu().numpy())
    res["elias"]["cpu_reference_encode_us"] = round((time.perf_counter() - t0) * 1e6, 1)
    assert np.array_equal(ref, idx.cpu().numpy().astype(np.int64))
    return res


# ---- the drop-in plugins' round, host to host ------------------------------------------------------
class _Mapping:
    """The Node's mapping as the plugins use it (get_uid only)."""

    def get_uid(self, rank, machine_id):
        return machine_id * 16 + rank


class _Graph:
    """A degree-3 neighbourhood (the regular topologies of the tutorial / eval configs)."""

    def __init__(self, nbrs):
        self.nbrs = set(nbrs)

    def neighbors(self, uid):
        return self.nbrs


def _net(n, seed):
    """An n-parameter fp32 model on the host (a weight matrix + a bias vector), with the codec
    fields the reference Model carries (models/Model.py:15-25)."""
    cols = 2048
    rows = n // cols

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            g = torch.Generator().manual_seed(seed)
            self.weight = torch.nn.Parameter(torch.randn(rows, cols, generator=g))
            self.bias = torch.nn.Parameter(torch.randn(n - rows * cols, generator=g))
            self.model_change = None
            self.accumulated_changes = None
            self.shared_parameters_counter = None

    return Net()


def _perturb(model, g, scale=0.01):
    """The training step's effect on the parameters (excluded from every timed region)."""
    with torch.no_grad():
        for p in model.parameters():
            p.add_(scale * torch.randn(p.shape, generator=g))


def plugin_case(dev, kind="partial", rounds=6, warmup=2, seed=17, cpu_rounds=1, tmpdir=None,
                on_warm=None):
    """One node's gossip round through the drop-in classes, host memory to host memory, as
    node/DPSGDNode.py:72-115 drives them: ``get_data_to_send(degree=3)`` (state_dict -> pinned H2D
    -> device encode -> device Elias (+ float codec) -> D2H -> the wire dict), the TCP wire
    (``pickle.dumps`` / ``pickle.loads``, communication/TCP.py:110-232), and ``_averaging`` of three
    neighbours' payloads (H2D of the received legs, device decode, Metro-Hastings fold, D2H of the
    averaged model, ``load_state_dict``).  The neighbours' messages are produced by three more
    plugin instances before the timed rounds (other processes in a real run).

    kind "partial": PartialModel, alpha 0.01, Elias (C2: N = 11 M).  kind "jwins": the JWINS
    tutorial [SHARING] (sym2 level 4, alpha list, accumulation, EliasFpzip) at N = 25 M.

    cpu_baseline (partial only): the reference's own op sequence for the same round on the host
    (oracle/ref_ops.py: cat, sub, abs, std_mean, topk, sort, counter, gather; the reference
    Elias encode / decode restated in oracle/elias.py — the decode is the reference's pure-Python
    code walk, compression/Elias.py:54-97; deserialized_model's cat + index_put per payload, the
    MH fold, load_state_dict) on torch's CPU threads."""
    import os
    import pickle
    import tempfile
    from collections import deque

    import numpy as np

    from decentralizepy_amd.sharing.JWINS.JWINS import JWINS
    from decentralizepy_amd.sharing.PartialModel import PartialModel

    tmpdir = tmpdir or tempfile.mkdtemp(prefix="dpz_plugin_")
    if kind == "partial":
        n = 11_000_000
        cls = PartialModel
        kw = dict(alpha=0.01, compress=True, compression_class="Elias",
                  compression_package="decentralizepy_amd.compression.Elias")
    else:
        n = 25_000_000
        cls = JWINS
        kw = dict(change_based_selection=True, alpha_list="[0.1,0.15,0.2,0.25,0.3,0.4,1.0]",
                  wavelet="sym2", level=4, accumulation=True, accumulate_averaging_changes=True,
                  metadata_cap=0.5, compress=True, compression_class="EliasFpzip",
                  compression_package="decentralizepy_amd.compression.EliasFpzip")
    nbr_uids = [1, 2, 3]
    models = [_net(n, seed + i) for i in range(4)]
    plugins = [cls(i, 0, None, _Mapping(), _Graph([u for u in range(4) if u != i]), models[i],
                   None, tmpdir, **kw) for i in range(4)]
    g = torch.Generator().manual_seed(seed + 100)
    node, nmodel = plugins[0], models[0]

    def neighbour_wires():
        wires = []
        for i in nbr_uids:
            _perturb(models[i], g)
            d = plugins[i].get_data_to_send(degree=3)
            d["CHANNEL"] = "DPSGD"
            wires.append(pickle.dumps(d))
        return wires

    t_send, t_recv, out_bytes, in_bytes = [], [], 0, 0
    for r in range(warmup + rounds):
        if r == warmup and on_warm is not None:
            on_warm()  # a diagnostic's counters start with the timed rounds
        wires = neighbour_wires()  # the neighbours' round (not this node's work)
        _perturb(nmodel, g)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        data = node.get_data_to_send(degree=3)
        data["CHANNEL"] = "DPSGD"
        wire = pickle.dumps(data)
        t1 = time.perf_counter()
        peer = {u: deque([pickle.loads(w)]) for u, w in zip(nbr_uids, wires)}
        node._averaging(peer)
        t2 = time.perf_counter()
        if r >= warmup:
            t_send.append(t1 - t0)
            t_recv.append(t2 - t1)
            out_bytes = len(wire)
            in_bytes = sum(len(w) for w in wires)
    send_ms = 1e3 * float(np.median(t_send))
    recv_ms = 1e3 * float(np.median(t_recv))
    # the PCIe legs of the round, timed alone with pinned buffers: the flat model up (4N), the
    # averaged model down (4N), and the payload legs (~ the wire bytes) each way
    a = torch.empty(n, dtype=torch.float32).pin_memory()
    b = torch.empty(n, dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        b.copy_(a, non_blocking=True)
        torch.cuda.synchronize()
        a.copy_(b, non_blocking=True)
        torch.cuda.synchronize()
    pcie_model_ms = (time.perf_counter() - t0) / 5 * 1e3
    del a, b
    res = {"kind": kind, "n": n, "class": cls.__name__,
           "compression": kw["compression_class"], "rounds": rounds,
           "round_ms": round(send_ms + recv_ms, 3), "send_ms": round(send_ms, 3),
           "receive_ms": round(recv_ms, 3), "wire_out_bytes": out_bytes,
           "wire_in_bytes": in_bytes,
           "pcie_model_up_down_ms": round(pcie_model_ms, 3),
           "pcie_model_share": round(pcie_model_ms / (send_ms + recv_ms), 3),
           "GiBps_params": round(4 * n / ((send_ms + recv_ms) * 1e-3) / 2 ** 30, 3)}
    del plugins, node, models, nmodel
    torch.cuda.empty_cache()
    if kind == "partial" and cpu_rounds > 0:
        res["cpu_baseline"] = _plugin_cpu_round(n, 0.01, cpu_rounds, seed)
    elif cpu_rounds > 0:
        # the JWINS round's reference op sequence (Wavelet.py:142-329 + PartialModel.py:305-350)
        # at the alpha list's median draw; the payload compression legs are not in it (fpzip is
        # absent, and the reference Elias walk over ~1-10 M indices takes seconds to minutes:
        # compression/Elias.py, timed per entry by --workload wire)
        res["cpu_baseline"] = cpu_wavelet_round(
            n, 0.2, 3, seed, 4, "sym2", seconds=8.0,
            what="the JWINS node round's reference ops without the compressor legs")
    return res


def _plugin_cpu_round(n, alpha, rounds, seed):
    """The reference's op sequence for the same node round on the host's CPU threads (test
    infrastructure: oracle/ref_ops.py and oracle/elias.py, imported here only as the baseline)."""
    import pickle

    import numpy as np

    from oracle import elias as oelias
    from oracle import ref_ops
    gen = torch.Generator().manual_seed(seed)
    x = torch.randn(n, generator=gen)
    x0 = x - 0.01 * torch.randn(n, generator=gen)
    counter = torch.zeros(n, dtype=torch.int32)
    k = round(alpha * n)
    wires = []
    for j in range(3):
        idx = np.sort(np.random.default_rng(seed + j).choice(n, size=k, replace=False))
        d = {"alpha": alpha, "indices": oelias.encode(idx.astype(np.int32)),
             "params": np.random.default_rng(seed + 10 + j).standard_normal(k).astype(np.float32),
             "send_partial": True, "degree": 3, "iteration": 0, "CHANNEL": "DPSGD"}
        wires.append(pickle.dumps(d))
    times = {"send": [], "receive": [], "elias_decode": []}
    for _ in range(rounds):
        t0 = time.perf_counter()
        idx, vals = ref_ops.encode(x, x0, alpha, counter)          # PartialModel.py:164-246
        msg = {"alpha": alpha, "indices": oelias.encode(idx), "params": vals,
               "send_partial": True, "degree": 3, "iteration": 0}  # Elias.py:20-52
        pickle.dumps(msg)
        t1 = time.perf_counter()
        total = None
        te = 0.0
        for w in wires:                                            # Sharing.py:156-190
            d = pickle.loads(w)
            t2 = time.perf_counter()
            ind = oelias.decode(d["indices"])                      # Elias.py:54-97
            te += time.perf_counter() - t2
            t_ = ref_ops.decode(x, ind, d["params"])               # PartialModel.py:257-303
            term = t_ * (1 / 4)
            total = term if total is None else total + term
        total += (1 - 3 / 4) * x
        x0 = total.clone()                                         # load_state_dict / _post_step
        t3 = time.perf_counter()
        times["send"].append(t1 - t0)
        times["receive"].append(t3 - t1)
        times["elias_decode"].append(te / 3)
    med = {kk: 1e3 * float(np.median(v)) for kk, v in times.items()}
    return {"kind": "port", "cores": torch.get_num_threads(),
            "round_ms": round(med["send"] + med["receive"], 2), "send_ms": round(med["send"], 2),
            "receive_ms": round(med["receive"], 2),
            "elias_decode_ms_per_payload": round(med["elias_decode"], 2),
            "sample": f"{rounds} round(s) of the reference op sequence at N={n}, 3 payloads, "
                      f"{torch.get_num_threads()} torch threads; the Elias decode is the "
                      "reference's pure-Python code walk (oracle/elias.py)"}
