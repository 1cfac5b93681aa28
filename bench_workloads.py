"""Secondary workloads of bench.py: C3 (JWINS wavelet + top-k, 16-payload
batched decode + weighted average), C5 (256 MiB, 0.1 % top-k, fp16 value packing) and the
PCIe-inclusive end-to-end rate (the reference path starts and ends in host memory: pyzmq socket
buffers / CPU model parameters).

Every function times whole steps with the device already holding what a node keeps resident
across rounds (init_model, accumulated changes, counters); inputs are synthetic (device PRNG).
Node states rotate so each step streams its inputs from HBM, not the 256 MiB Infinity Cache.
"""
import math
import time

import torch

L3_BYTES = 256 * 2 ** 20


def _sync_time(fn, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        fn(i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def c3_case(dev, n=25_000_000, alpha=0.01, npay=16, steps=40, warmup=5, seed=3, wavelet="sym2"):
    """C3: one JWINS receiver round on an N-parameter model (reference Wavelet.py:142-329 with
    the tutorial/JWINS/config.ini settings change_based_selection, accumulation and
    accumulate_averaging_changes on): encode = W(x), W(x - x0) in one DWT launch, top-k of
    |W(x - x0) + acc| (PartialModel.py:322-327: change += acc), acc rewind and counter at the
    selected coefficients, values from W(x); decode =
    16 neighbour payloads replaced + Metro-Hastings-folded in the wavelet domain in one batched
    launch (w = 1/17 each, self 1 - 16/17), then one IDWT launch back to N parameters.
    Algorithmic bytes: B_enc = 8N + 8M + 12k (+ acc 8M read/write), B_dec =
    4M + 4N + 8 n k."""
    from decentralizepy_amd import codec
    level = 4
    m = codec.wavedec_len(n, level, wavelet)
    k = round(alpha * m)
    per_set = 4 * (2 * n + 4 * m) + 8 * k
    R = max(2, math.ceil(2 * L3_BYTES / per_set) + 1)
    g = torch.Generator(device=dev).manual_seed(seed)
    sets = []
    for _ in range(R):
        x = torch.randn(n, device=dev, generator=g)
        sets.append(dict(x=x, x0=x - 0.01 * torch.randn(n, device=dev, generator=g),
                         acc=0.01 * torch.randn(m, device=dev, generator=g),
                         cnt=torch.zeros(m, dtype=torch.int32, device=dev),
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

    def encode(d):
        codec.wavedec(d["x"], level, x0=d["x0"], coeffs_x=d["wx"], coeffs_diff=d["wc"],
                      wavelet=wavelet)
        codec.topk_encode(d["wc"], k, acc=d["acc"], acc_mode=codec.DPZ_ACC_ADD,
                          vals_src=d["wx"], counter=d["cnt"], idx_out=d["idx"],
                          val_out=d["val"], workspace=ws, asynchronous=True)

    def decode(d):
        codec.decode_average(d["wx"], pays, w, w_self, out=d["tot"], workspace=ws)
        codec.waverec(d["tot"], n, level, out=d["out"], wavelet=wavelet)

    def step(i):
        d = sets[i % R]
        encode(d)
        decode(d)

    for i in range(max(warmup, R)):
        step(i)
    t_step = _sync_time(step, steps)
    t_enc = _sync_time(lambda i: encode(sets[i % R]), steps)
    t_dec = _sync_time(lambda i: decode(sets[i % R]), steps)
    fb = codec.topk_status(ws) != 0
    with codec.KernelTimer() as kt:
        torch.cuda._sleep(int(100e6))
        for i in range(R * 2):
            step(i)
        torch.cuda.synchronize()
    kern = {nm: round(ms / c * 1e3, 2) for nm, (ms, c) in kt.result.items()}
    b_enc = 8 * n + 8 * m + 8 * m + 12 * k  # x, x0 -> W(x), W(dx); read W(dx), acc; k triples
    b_dec = 4 * m + 4 * n + 8 * npay * k + 8 * m
    return dict(workload=f"C3: JWINS {wavelet} level-4 wavelet + top-k (accumulation) of an "
                         f"N={n} tensor (M={m} coefficients), {npay}-payload batched decode + "
                         f"MH average + IDWT", n=n, m=m, k=k, alpha=alpha, rotated_states=R,
                value=4 * n / t_step / 2 ** 30, ms_per_step=t_step * 1e3,
                encode_us=t_enc * 1e6, decode_us=t_dec * 1e6,
                alg_bytes_enc=b_enc, alg_bytes_dec=b_dec,
                step_frac_of_hbm_peak=(b_enc + b_dec) / t_step / 8e12, fell_back=fb,
                kernels_avg_us=kern)


def c3_round_case(dev, rank, world, dist, n=25_000_000, rounds=10, warmup=2, seed=21,
                  wavelet="sym2"):
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
    return dict(workload=f"C3 shape (b): JWINS round of regular_16 (16 nodes x degree 3), "
                         f"N={n} per node, {wavelet} level 4, tutorial alpha_list",
                n=n, m=m, nodes=len(adj), world=world, rounds=rounds,
                ms_per_round=t * 1e3, ms_per_round_min=min(times) * 1e3,
                value=len(adj) * 4 * n / t / 2 ** 30,
                alg_bytes_per_round=b, round_frac_of_hbm_peak=b / t / 8e12 / world,
                scaling="strong (16 nodes fixed)")


def c5_case(dev, n=67_108_864, alpha=0.001, steps=40, warmup=5, seed=5, streams=3):
    """C5: 256 MiB fp32 tensor, 0.1 % top-k, payload values packed to fp16 (RNE, torch.half
    semantics): encode = top-k + fp16 pack; decode = fp16 unpack + replace.  B = 16N + 12k."""
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
                         val=torch.empty(k, device=dev),
                         h=torch.empty(k, dtype=torch.float16, device=dev),
                         v32=torch.empty(k, device=dev), out=torch.empty(n, device=dev)))
    S = [torch.cuda.Stream(dev) for _ in range(streams)]
    W = [codec.Workspace(dev) for _ in range(streams)]

    def step_on(d, ws):
        codec.topk_encode(d["x"], k, x0=d["x0"], counter=d["cnt"], idx_out=d["idx"],
                          val_out=d["val"], workspace=ws, asynchronous=True)
        codec.pack_fp16(d["val"], out=d["h"])
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
    return dict(workload=f"C5: N={n} (256 MiB) fp32, alpha={alpha} top-k, fp16 value packing",
                n=n, k=k, rotated_states=R, streams=streams,
                value=4 * n / t_multi / 2 ** 30, ms_per_step=t_multi * 1e3,
                one_node_ms_per_step=t_one * 1e3, alg_bytes=b,
                step_frac_of_hbm_peak=b / t_multi / 8e12, fell_back=fb)


def e2e_case(dev, n, alpha, fp16=False, steps=20, warmup=3, seed=7, streams=3):
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
    return dict(n=n, k=k, fp16_values=fp16, pcie_bytes_per_step=pcie,
                one_node_GiBps=4 * n / t_one / 2 ** 30, one_node_ms_per_step=t_one * 1e3,
                concurrent_GiBps=4 * n / t_multi / 2 ** 30, concurrent_ms_per_step=t_multi * 1e3,
                concurrent_pcie_GBps=pcie / t_multi / 1e9, streams=streams)


def shard_case(dev, rank, world, dist, n=67_108_864, alpha=0.001, steps=20, warmup=3, seed=9):
    """One tensor of N parameters sharded over the ranks (SURVEY §8e, C5 on 8 GPUs): the global
    top-k with one all-gather of every rank's k candidates (decentralizepy_amd/shard.py), then
    each rank decodes the global payload into its own slice (replace; indices outside the slice
    fall outside [0, n_r) and are skipped).  Strong scaling: N fixed, value = N params / time."""
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
    ops = HipShardOps(dev)
    ws = codec.Workspace(dev)

    def step(i):
        d = sets[i % R]
        idx, val = sharded_topk_encode(d["x"], d["x0"], k, lo, counter=d["cnt"], ops=ops)
        sharded_replace(d["x0"], lo, idx, val, out=d["out"], ops=ops)

    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t = (time.perf_counter() - t0) / steps
    if dist is not None:
        tt = torch.tensor([t], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
    return dict(workload=f"one N={n} tensor sharded over {world} GPU(s), alpha={alpha}: sharded "
                         f"top-k (one all-gather of {world} x {k} candidates) + slice decode",
                n=n, k=k, world=world, value=4 * n / t / 2 ** 30, ms_per_step=t * 1e3,
                scaling="strong")


def fft_case(dev, n=11_000_000, alpha=0.01, npay=3, steps=30, warmup=5, seed=9):
    """The FFT sharing plugin's device round (reference sharing/JWINS/FFT.py:132-302) on an
    N-parameter model: encode = x - x0, rfft(x) and rfft(x - x0) (hipFFT), |change| (complex, HIP),
    top-k on it with the counter, complex values gathered from rfft(x); decode = npay complex
    payloads folded (Metro-Hastings) over the (re, im) pairs, irfft (hipFFT) + 1/n.  The step
    rate is reported on the GiB/s metric (4N bytes of model per step) with the HIP kernels'
    average durations; the hipFFT kernels are library launches outside the per-kernel table."""
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
    return dict(workload=f"FFT plugin round: rfft top-k encode + {npay}-payload complex fold + "
                         f"irfft of an N={n} model (M={m} coefficients)",
                n=n, m=m, k=k, alpha=alpha, value=4 * n / t / 2 ** 30, ms_per_step=t * 1e3,
                note="hipFFT transforms are not in the per-kernel table (library kernels)",
                kernels_avg_us=kern)


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
    return res
