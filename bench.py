#!/usr/bin/env python3
"""Benchmark: GiB/s of fp32 params encoded+decoded (device-resident), 1 % top-k.

One step = one PartialModel top-k encode (fused |x - x0| -> sampled radix select -> ordered
compaction with counter update) of an N-element fp32 tensor already resident in HBM, plus the
matching decode (replace the k payload values into a copy of the local model), exactly the
reference's PartialModel.serialized_model + deserialized_model pair.

Workload (BASELINE.json north_star): the 64 MiB fp32 tensor, N = 16,777,216, alpha = 0.01 ->
k = 167,772 — the configuration the north-star target (>= 50 % of HBM peak) is quoted on.  The
C2 tensor (configs[1], N = 11,000,000, ResNet-18-sized) runs beside it as the `secondary` object.
Multi-GPU (torchrun): each rank encodes+decodes its own node's tensor (the gossip round is a set
of independent per-node codecs: no data-path collective) -> weak scaling; value = all ranks'
params / max-over-ranks time.  Beside it, every run times one C4 gossip round of the 96-node
topology sharded over the ranks, whose payload exchange is an RCCL all-gather ("gossip_round").

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (GB/s), /opt/skills/guides/MI355X_MICROARCH.md
NORTH_STAR_N = 16_777_216  # 64 MiB of fp32: BASELINE.json north_star's target tensor
C2_N = 11_000_000          # BASELINE.json configs[1] (ResNet-18-sized)


def workload_name(n):
    if n == NORTH_STAR_N:
        return ("north-star: PartialModel top-k encode + decode of one 64 MiB fp32 tensor "
                "(N=16,777,216), 1% top-k")
    if n == C2_N:
        return "C2: PartialModel top-k encode + decode of one 11M-fp32 flattened tensor"
    return f"PartialModel top-k encode + decode of one {n}-element fp32 tensor"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks (one per GPU); default: WORLD_SIZE under a launcher, else 1")
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--n", type=int, default=None,
                   help="tensor size (default: the 64 MiB north-star tensor; C4: C2's 11M)")
    p.add_argument("--alpha", type=float, default=0.01)
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-extra", action="store_true",
                   help="skip the secondary line (C2, or 64 MiB when --n is not 64 MiB) and "
                        "the C4 gossip-round / shard objects")
    p.add_argument("--workload", choices=["c2", "c3", "c4", "c5", "e2e", "shard", "fft", "wire",
                                          "plugin"],
                   default="c2",
                   help="c2: one node's 11M tensor per GPU (default); c4: the 96-node gossip "
                        "round of eval/96_regular.edges sharded over the GPUs; c3: JWINS wavelet "
                        "25M + 16-payload decode; c5: 256 MiB, 0.1%%, fp16 values; e2e: "
                        "PCIe-inclusive rates; shard: one C5 tensor sharded over the GPUs "
                        "(bench_workloads.py)")
    p.add_argument("--rotate", type=int, default=None,
                   help="independent node states cycled per step (default: enough for > 2x L3)")
    p.add_argument("--streams", type=int, default=3,
                   help="S > 1: S independent node codecs share the GPU on S streams (as "
                        "decentralizepy runs procs_per_machine nodes per machine); the one-node "
                        "(one stream) rate is always measured beside it")
    p.add_argument("--selftest-spawn", action="store_true",
                   help="(tests) each started rank reports RANK / WORLD_SIZE / LOCAL_RANK and "
                        "exits before any GPU call")
    p.add_argument("--repeats", type=int, default=0,
                   help="timed regions of exactly --steps steps each (0: auto, enough for a "
                        "stable median at small --steps); the line reports the median region")
    return p.parse_args()


def spawn_ranks(args):
    """``bench.py --gpus N`` (N > 1) started WITHOUT a launcher: run N ranks, one process per
    GPU, under torch.distributed.run as a child process and exit with its code.  This parent
    never makes a HIP call (no GPU initialised before the ranks start); it times the CPU
    baseline first (host cores only) and hands it to rank 0 through a file, so the ranks' GPU
    work and the CPU sample never overlap."""
    import socket
    import subprocess
    import tempfile
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    path = None
    if not args.no_cpu and args.workload == "c2":
        cpu = cpu_baseline(args.n, args.alpha, args.cpu_seconds)
        fd, path = tempfile.mkstemp(prefix="dpz_cpu_", suffix=".json")
        with os.fdopen(fd, "w") as f:
            json.dump(cpu, f)
        env["DPZ_BENCH_CPU_BASELINE"] = path
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    try:
        rc = subprocess.call(cmd, env=env)
    finally:
        if path:
            os.unlink(path)
    return rc


def timed_loop(fn, reps, stream):
    """Average device time of fn() over reps launches, with HIP events on `stream`."""
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        ev0.record(stream)
        for _ in range(reps):
            fn()
        ev1.record(stream)
    ev1.synchronize()
    return ev0.elapsed_time(ev1) / reps * 1e-3  # seconds


L3_BYTES = 256 * 2 ** 20  # MI355X Infinity Cache (MI355X_MICROARCH.md § Infinity Cache)


def gpu_case(n, alpha, dev, seed, steps, warmup, world, dist, rotate=None, streams=3, repeats=9):
    """Time `steps` encode+decode steps.  Consecutive steps rotate over R independent node states
    (x, x0, counter, payload, output) so the timed working set is > 2x the 256 MiB Infinity
    Cache: every step streams its inputs from HBM, as a real round does after training.

    Step i = node state i's round: top-k encode of its model x (change vs x0, counter update)
    and the replace decode of a neighbour's payload over x (reference
    PartialModel.serialized_model + deserialized_model, whose base is the receiver's current
    state_dict): the neighbour is the state encoded S steps earlier on the same stream.  The
    decode's copy of x is written by the encoder's filter as it streams x (fused), so the step
    moves 12N + 24k bytes; the line's frac_of_hbm_peak keeps SURVEY §8(d)'s unfused B = 16N + 16k
    (decode materialised as in the reference) and the PMC traffic beside it is what moved.  The host loop over steps is native (dpz_encode_replace_batch, one
    ctypes call per R steps).  With S streams, S node codecs share the GPU (state i on stream
    i % S, its own workspace), as decentralizepy runs procs_per_machine nodes per machine; the
    one-stream (one node) rate is measured beside it and the faster of the two is the line's
    value.  Every timed encode's sampled-path status is OR-ed into its workspace's sticky word
    and checked after the loop (fell_back)."""
    from decentralizepy_amd import codec
    from decentralizepy_amd._lib import DPZ_BATCH_DECODE, DPZ_BATCH_ENCODE, DPZ_BATCH_HINT
    k = round(alpha * n)
    per_set = 4 * n * 4 + 8 * k          # x, x0, counter, out + payload
    R = rotate or max(1, math.ceil(2 * L3_BYTES / per_set) + 1)
    S = max(1, streams)
    R = -(-R // S) * S                   # a state is only ever reused by the same stream
    if S > 1:
        R = max(R, 2 * S)                # a neighbour's payload is another state's
    g = torch.Generator(device=dev).manual_seed(seed)
    sets = []
    for _ in range(R):
        x = torch.randn(n, device=dev, generator=g)
        x0 = x - 0.01 * torch.randn(n, device=dev, generator=g)
        sets.append(dict(x=x, x0=x0, counter=torch.zeros(n, dtype=torch.int32, device=dev),
                         idx=torch.empty(k, dtype=torch.int32, device=dev),
                         val=torch.empty(k, dtype=torch.float32, device=dev),
                         out=torch.empty(n, dtype=torch.float32, device=dev)))
    s_list = [torch.cuda.Stream(dev) for _ in range(S)]
    ws_list = [codec.Workspace(dev) for _ in range(S)]
    # every state's shared_parameters_counter as the PartialModel plugin keeps it (RingCounter):
    # the encodes write their payload indices into a ring slot and update no counter line; the
    # rings are folded into the counters when full and at the end of every timed region
    # (BENCH_RING=0: the counter updated inside the compact, A/B)
    from decentralizepy_amd._device import RingCounter
    rings = ([RingCounter(d["counter"]) for d in sets]
             if os.environ.get("BENCH_RING", "1") != "0" else None)
    multi = codec.NodeStepBatch(sets, n, k, s_list, ws_list, decode_src=lambda j: (j - S) % len(sets),
                                rings=rings)
    # one node on one stream decodes a neighbour's payload (the previous state's, encoded in the
    # previous step on the same stream), so its decode is co-scheduled in its encode's launches
    # its own workspace: a prior window is only taken from an encode of the same grid (the
    # S-codec batch runs the shared filter grid, DPZ_TOPK_SHARED)
    one = codec.NodeStepBatch(sets, n, k, s_list[:1], [codec.Workspace(dev)],
                              decode_src=lambda j: (j - 1) % len(sets), rings=rings)

    # every encode takes its key window from the previous encode on its stream's workspace
    # (DPZ_BATCH_HINT: a node's previous round, as PartialModel runs it; no sample launch)
    hint = DPZ_BATCH_HINT if os.environ.get("BENCH_HINT", "1") != "0" else 0  # A/B switch

    def run_steps(batch, count, what=DPZ_BATCH_ENCODE | DPZ_BATCH_DECODE | hint):
        for _ in range(count // R):
            batch.run(what)
        if count % R:
            batch.run(what, m=count % R)

    torch.cuda.synchronize()
    run_steps(multi, max(warmup, 2 * R))
    multi.flush_rings()
    torch.cuda.synchronize()
    run_steps(one, max(warmup, R))
    one.flush_rings()
    torch.cuda.synchronize()
    multi.sticky_status(clear=True)
    one.sticky_status(clear=True)

    def timed_once(batch, count):
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run_steps(batch, count)
        batch.flush_rings()  # every deferred counter update of the region, inside it
        t_host = time.perf_counter() - t0  # host enqueue time (host-bound if close to t)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        if dist is not None:
            tt = torch.tensor([t], device=dev, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            t = float(tt.item())
        return t / count, t_host / count

    def timed(batch, count):
        """`repeats` timed regions of exactly `count` steps, each bracketed by barrier +
        synchronize and max-over-ranks; the median region is the result (a 20-step region is
        under 1 ms of device time, so one host hiccup would otherwise move the line)."""
        res = sorted(timed_once(batch, count) for _ in range(repeats))
        spread.append([res[0][0], res[len(res) // 2][0], res[-1][0]])
        return res[len(res) // 2]

    spread = []
    s_multi, h_multi = timed(multi, steps)
    s_serial, h_serial = timed(one, steps)
    status = multi.sticky_status(clear=True) | one.sticky_status(clear=True)  # both loops
    fell_back = status != 0
    if dist is not None:
        st = torch.tensor([status], device=dev, dtype=torch.int32)
        dist.all_reduce(st, op=dist.ReduceOp.MAX)
        fell_back = int(st.item()) != 0
    if S > 1 and s_multi <= s_serial:
        s_step, s_host, mode = s_multi, h_multi, "multi"
    else:
        s_step, s_host, mode = s_serial, h_serial, "serial"
    # per-stage device time with events on the one launch stream (encodes only, decodes only)
    stream = s_list[0]
    reps = max(2 * R, steps // 2)

    t_enc = _stage_time(one, DPZ_BATCH_ENCODE | hint, reps, run_steps, stream)
    t_dec = _stage_time(one, DPZ_BATCH_DECODE, reps, run_steps, stream)
    # per-kernel device time: the library brackets every launch with a HIP event pair on the
    # stream it launches on.  A GPU-side spin first lets the host queue all `reps` steps, so the
    # kernels then run back-to-back (no host-launch gaps inside a pair).  Encodes and decodes are
    # queued as separate loops: a one-stream step co-schedules the decode inside the encoder's
    # launches (dpz_encode_replace_batch), which would hide the replace kernel's own duration.
    # The kernels of the one-node step as it runs (fused: the filter also writes the decode's
    # copy of x, the select launch scatters the entries), then the standalone replace decode
    # (the "fold" kernel, for the event-pair overhead below and the decode stage).
    with codec.KernelTimer() as kt:
        with torch.cuda.stream(stream):
            torch.cuda._sleep(int(200e6))  # ~0.1 s of GPU cycles while the steps are enqueued
        run_steps(one, reps)
        run_steps(one, reps, DPZ_BATCH_DECODE)
        torch.cuda.synchronize()
    kernels = {name: {"avg_us": ms / c * 1e3, "launches_per_step": c / reps}
               for name, (ms, c) in kt.result.items()}
    if "fold" in kernels:  # the standalone decode's launches are not part of the step
        kernels["fold"]["launches_per_step"] = 0.0 if fused_copy() else 1.0
    b_enc = 8 * n + 8 * k + 8 * k      # read x, x0; write idx, val; counter[idx] += 1 (r+w)
    b_dec = 8 * n + 8 * k              # read local, payload; write out
    fell_back |= (multi.sticky_status(clear=True) | one.sticky_status(clear=True)) != 0
    product = product_one_node(sets, n, k, stream, max(2 * R, min(steps, 200)), alpha=alpha)
    fell_back |= product["fell_back"]
    return dict(n=n, k=k, s_step=s_step, s_multi=s_multi, s_serial=s_serial, s_host=s_host,
                mode=mode, streams=S, fell_back=fell_back, t_enc=t_enc, t_dec=t_dec,
                b_enc=b_enc, b_dec=b_dec, kernels=kernels, rotate=R, repeats=repeats,
                product=product,
                spread_ms={"multi": [round(v * 1e3, 5) for v in spread[0]],
                           "serial": [round(v * 1e3, 5) for v in spread[1]]},
                value=world * 4 * n / s_step / 2 ** 30)


class _BenchMapping:
    """The Node's mapping as the plugins use it (get_uid only)."""

    def get_uid(self, rank, machine_id):
        return rank


class _BenchGraph:
    """A regular topology of degree ``deg`` as the plugins read it (neighbors(uid) only)."""

    def __init__(self, deg):
        self.deg = deg

    def neighbors(self, uid):
        return set(range(uid + 1, uid + 1 + self.deg))


def _bench_model(n):
    """An n-parameter fp32 model on the host with the reference Model's codec fields
    (models/Model.py:15-25); zero-initialised (the bench sets the plugin's device state)."""
    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.weight = torch.nn.Parameter(torch.zeros(n))
            self.model_change = None
            self.accumulated_changes = None
            self.shared_parameters_counter = None
    return Net()


def make_bench_plugins(count, n, alpha, deg, dev):
    """``count`` PartialModel plugins (the drop-in class, decentralizepy_amd.sharing.PartialModel)
    of an n-parameter model on a degree-``deg`` regular graph, one per rotated node state, all on
    ``dev`` (the plugin's DPZ_DEVICE override; it would otherwise pick rank mod GPUs)."""
    from decentralizepy_amd.sharing.PartialModel import PartialModel
    import tempfile
    tmp = tempfile.mkdtemp(prefix="dpz_bench_")
    prev = os.environ.get("DPZ_DEVICE")
    os.environ["DPZ_DEVICE"] = str(torch.device(dev).index or 0)
    try:
        return [PartialModel(j, 0, None, _BenchMapping(), _BenchGraph(deg), _bench_model(n), None,
                             tmp, alpha=alpha) for j in range(count)]
    finally:
        if prev is None:
            del os.environ["DPZ_DEVICE"]
        else:
            os.environ["DPZ_DEVICE"] = prev


def plugin_device_round(p, x, x0, payloads, degrees, blocking=True):
    """The device work of one PartialModel round as the plugin enqueues it, with the host legs
    (state_dict H2D, payload H2D, D2H, load_state_dict) left out: ``_pre_step`` (model_change
    kept lazily, LazyChange), ``serialized_model``'s ``_encode`` (top-k into the counter ring's
    slot, prior-round key window, keep-x; the fold base when the node has one neighbour),
    ``_averaging``'s Metro-Hastings weights and ``_fold_on_base`` / ``_fold`` (reference
    sharing/PartialModel.py:188-255, 305-331, sharing/Sharing.py:156-190), ``_post_step``.
    ``x`` / ``x0``: the node's flat model and init_model, already in HBM.  ``blocking=False``:
    the encode is only enqueued (``_encode(k, blocking=False)``: no host wait for its status;
    the caller checks the sticky status words after the loop), so back-to-back rounds keep the
    device busy — the plugin itself waits there for its payload (the D2H to the wire follows).
    Returns the encode's (idx, val) and the averaged model."""
    p.pre_share_model = x
    p.pre_share_model_transformed, p._change_dev = x, None
    p.init_model = x0
    p._fb = None
    p.model.model_change = p._model_change()
    idx, val = p._encode(round(p.alpha * p.transformed_len), blocking=blocking)
    weights = [1 / (max(len(payloads), d) + 1) for d in degrees]
    weight_total = 0
    for w in weights:
        weight_total += w
    out = p._fold_on_base(x, payloads, weights, 1 - weight_total)
    if out is None:
        out = p._fold(x, payloads, weights, 1 - weight_total)
    p._drop_model_change()  # _post_step: init_model = the averaged model (a rebinding)
    return idx, val, out


def product_one_node(sets, n, k, stream, reps, alpha=0.01):
    """``stages.product_one_node``: the device work of the drop-in PartialModel plugin's round
    (plugin_device_round: its own _model_change / _encode / _fold_on_base / _fold methods, so the
    launch sequence is the plugin's, tests/test_gpu_bench_plugin.py) for one node on one stream,
    with 1 and 3 neighbours (degree-1 / degree-3 regular graphs: the one-neighbour node takes the
    encode's fold base).  Step j is node state j mod R of the HBM-rotated states; its neighbours'
    payloads are the ones states j-1 .. j-npay sent.  Each state is its own plugin instance
    (its workspace / prior window, its counter ring).  The timed region ends with every plugin's
    counter read (RingCounter flush, the node's end-of-run dump, node/DPSGDNode.py:186-194), so
    the counter updates the rounds deferred are inside it.  Device time: HIP events around the
    whole loop on the launch stream after a GPU-side spin that lets the host queue it.
    Algorithmic bytes: encode 8N + 16k (x, x0; idx, val; counter r+w), fold 8N + 8·npay·k."""
    from decentralizepy_amd import codec
    R = len(sets)
    out = {}
    fell = False
    with torch.cuda.stream(stream):
        for npay in (1, 3):
            plugins = make_bench_plugins(R, n, alpha, npay, stream.device)
            sent = [None] * R

            def step(j, encode=True, fold=True):
                d, p = sets[j % R], plugins[j % R]
                pays = [sent[(j - q) % R] for q in range(1, npay + 1)]
                if encode and fold:
                    i, v, _ = plugin_device_round(p, d["x"], d["x0"], pays, [npay] * npay,
                                                  blocking=False)
                    sent[j % R] = (i, v)
                elif encode:  # the round's first half: pre-step + encode
                    p.pre_share_model = d["x"]
                    p.pre_share_model_transformed, p._change_dev = d["x"], None
                    p.init_model, p._fb = d["x0"], None
                    p.model.model_change = p._model_change()
                    sent[j % R] = p._encode(k, blocking=False)
                    p._fb = None  # (the fold-only loop takes the plain fold)
                else:  # the second half: the Metro-Hastings fold over the node's model
                    w = [1 / (npay + 1)] * npay
                    wt = 0
                    for v in w:
                        wt += v
                    p._fold(d["x"], pays, w, 1 - wt)

            def flush_all():
                for p in plugins:
                    p._ring.flush()

            # a timed region is one full ring per plugin (its counter flushed once, when full, as
            # in a run: RingCounter), so the deferred counter work is charged at the rate a node
            # pays it; at least `reps` steps
            ring = plugins[0]._ring
            ring_rounds = max(1, min(ring.MAX_SEGS, ring.cap_bytes // max(4 * k, 1)))
            reps = max(reps, R * ring_rounds)

            def loop(**kw):
                ev0 = torch.cuda.Event(enable_timing=True)
                ev1 = torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                torch.cuda._sleep(int(400e6))  # the host queues the loop while the GPU spins
                ev0.record(stream)
                t0 = time.perf_counter()
                for j in range(reps):
                    step(j, **kw)
                flush_all()  # every counter read once: the deferred updates are timed
                t_host = time.perf_counter() - t0
                ev1.record(stream)
                ev1.synchronize()
                return ev0.elapsed_time(ev1) / reps * 1e-3, t_host / reps

            for j in range(R):  # every state encoded once (its payload exists)
                step(j, fold=False)
            for j in range(2 * R):  # warm-up rounds (priors set, allocator warm)
                step(j)
            flush_all()
            t_step, h_step = loop()
            t_enc, _ = loop(fold=False)
            t_dec, _ = loop(encode=False)
            # per-kernel device time of the round's launches (library event pairs; the pair
            # overhead is not removed here: rocprofv3's summary under profiles/ gives the bare
            # durations)
            with codec.KernelTimer() as kt:
                loop()
            kern = {nm: {"avg_us_event_pair": round(ms / c * 1e3, 3),
                         "launches_per_step": round(c / reps, 3)}
                    for nm, (ms, c) in kt.result.items()}
            fell |= any(codec.topk_sticky_status(p.workspace, clear=True) != 0 for p in plugins)
            b_enc, b_dec = 8 * n + 16 * k, 8 * n + 8 * npay * k
            out[f"{npay}_payload"] = {
                "step_us": round(t_step * 1e6, 3), "encode_us": round(t_enc * 1e6, 3),
                "fold_us": round(t_dec * 1e6, 3), "host_enqueue_us": round(h_step * 1e6, 3),
                "fold_path": "fold base (encode writes it)" if npay == 1 else "plain fold",
                "steps_per_region": reps, "ring_rounds": ring_rounds,
                "kernels": kern,
                "alg_bytes": b_enc + b_dec,
                "GiBps": round(4 * n / t_step / 2 ** 30, 2),
                "frac_of_hbm_peak": round((b_enc + b_dec) / t_step / 1e9 / HBM_PEAK_GBS, 4)}
            del plugins, sent
    out["note"] = ("the drop-in PartialModel plugin's device round (bench.plugin_device_round: "
                   "its _model_change / _encode / _fold_on_base / _fold), host legs excluded, one "
                   "plugin per rotated node state; model_change formed on read only "
                   "(LazyChange), the counter updates deferred to a ring folded in on read "
                   "(RingCounter) — a timed region is one full ring per plugin, every counter "
                   "read (flushed) at its end, so the deferred updates are timed at the rate a "
                   "node pays them")
    out["fell_back"] = fell
    return out


def _stage_time(batch, what, reps, run_steps, stream):
    """Average device time of one step's `what` part (encode or decode), back to back on the
    batch's single stream, HIP events around the loop on that stream."""
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        torch.cuda._sleep(int(50e6))  # the host queues the loop while the GPU spins
        ev0.record(stream)
    run_steps(batch, reps, what)
    batch.flush_rings()  # (encodes: their deferred counter updates, on the batch's stream)
    ev1.record(stream)
    ev1.synchronize()
    return ev0.elapsed_time(ev1) / reps * 1e-3


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def gossip_case(n, alpha, dev, rank, world, dist, rounds, warmup, exchange="allgather",
                engine_kw=None):
    """C4: one synchronous gossip round of the 96-node regular topology (reference
    eval/96_regular.edges, copied as data under tests/golden/), nodes sharded over the ranks,
    payloads exchanged by one RCCL all-gather (decentralizepy_amd/gossip.py).  A "training"
    perturbation between rounds is excluded from the timed region.  ``engine_kw``: the engine's
    injectable steps (encode / fold / partial / combine; tests/test_cpu_bench_collectives.py runs
    this function on gloo ranks with the oracle standing in for the HIP codec)."""
    from decentralizepy_amd.gossip import GossipRound, read_edges, shard
    adj = read_edges(os.path.join(ROOT, "tests", "golden", "96_regular.edges"))
    lo, hi, _ = shard(len(adj), world, rank)
    g = torch.Generator(device=dev).manual_seed(77 + rank)
    x = torch.randn(hi - lo, n, device=dev, generator=g)
    eng = GossipRound(adj, x, alpha, rank=rank, world=world, device=dev, exchange=exchange,
                      **(engine_kw or {}))
    del x
    noise = 0.01 * torch.randn(hi - lo, n, device=dev, generator=g)
    total = 0.0
    for r in range(warmup + rounds):
        eng.x += noise
        _sync(dev)
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        eng.step()
        _sync(dev)
        if dist is not None:
            dist.barrier()
        dt = time.perf_counter() - t0
        if dist is not None:
            tt = torch.tensor([dt], device=dev, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            dt = float(tt.item())
        if r >= warmup:
            total += dt
    s_round = total / rounds
    # per-leg times (encode / exchange / fold, or the reduce-scatter legs) from two more rounds
    # with a synchronize between legs: a breakdown beside the timed rounds, not part of them
    eng.leg_times = {}
    for _ in range(2):
        eng.x += noise
        eng.step()
    legs = {nm: round(v / 2 * 1e3, 4) for nm, v in eng.leg_times.items()}
    eng.leg_times = None
    k = eng.k
    nsum = sum(len(a) for a in adj)
    # algorithmic bytes of the round: every node's encode (read x, x0; idx / val out; counter
    # r+w) and fold (read x and the payloads; the averaged model written as the node's model AND
    # as its init_model — reference Sharing.py:186-190 load_state_dict, then PartialModel.py:
    # 340-343 init_model = cat(state): both must hold it for the next round, 12N);
    # alg_bytes_8n counts the fold's output once (the round-4 convention)
    return dict(n=n, k=k, s_step=s_round, nodes=len(adj), edges=nsum // 2, legs_ms=legs,
                rs_group=getattr(eng, "rs_group", None),
                peer_recv_payloads=(eng._peer_n_recv if eng.exchange_mode == "peer" else None),
                value=len(adj) * 4 * n / s_round / 2 ** 30,
                alg_bytes=len(adj) * (8 * n + 16 * k) + len(adj) * 12 * n + nsum * 8 * k,
                alg_bytes_8n=len(adj) * (8 * n + 16 * k) + len(adj) * 8 * n + nsum * 8 * k)


def fused_copy():
    """The one-node step's decode copy is written by the encoder's filter (dpz_topk.hip
    dpz_topk_encode_replace) unless a diagnostic build (DPZ_CODEC_LIB) disables it with its A/B
    switches; the product library reads no environment."""
    if not os.environ.get("DPZ_CODEC_LIB"):
        return True
    return os.environ.get("DPZ_FUSED_COPY", "1") != "0" and \
        os.environ.get("DPZ_BATCH_COSCHED", "1") != "0"


def kernel_alg_bytes(name, n, k):
    """Algorithmic HBM bytes of one launch: the bytes the operation must move,
    not what the implementation happens to move (candidate lists, histograms are excluded)."""
    return {
        "topk_sample": 8 * 65536,          # x, x0 at the 65,536 sampled positions
        # read x, x0 once (+ write the decode's copy of x when fused)
        "topk_filter": 12 * n if fused_copy() else 8 * n,
        "topk_select": 0,                  # works on the ~1.9k candidates only
        "topk_resolve": 0,                 # works on the ~k/256 boundary entries only
        "topk_compact": 8 * k + 4 * k + 8 * k,  # write idx, val; gather vals; counter r+w
        "fold_offsets": 4 * k,             # read the payload indices
        "fold": 8 * n + 8 * k,             # read local, payload (idx, val); write out
    }.get(name, 0)


def load_pmc(kernel, n):
    """HBM traffic per launch of `kernel` from the committed rocprofv3 PMC summaries
    (profiles/pmc_latest*.json), the one collected at this tensor size (its "n"); None if none
    was."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_latest*.json"))):
        with open(path) as f:
            pmc = json.load(f)
        if pmc.get("n") != n:
            continue
        ent = pmc.get("kernels", {}).get(kernel)
        if ent:
            return ent.get("hbm_bytes_per_launch")
    return None


def _cpu_steps(n, alpha, seconds, threads):
    from oracle import ref_ops
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        g = torch.Generator().manual_seed(0)
        x = torch.randn(n, generator=g)
        x0 = x - 0.01 * torch.randn(n, generator=g)
        counter = torch.zeros(n, dtype=torch.int32)
        times = []
        t_start = time.perf_counter()
        while True:
            t0 = time.perf_counter()
            idx, vals = ref_ops.encode(x, x0, alpha, counter)
            ref_ops.decode(x0, idx, vals)
            times.append(time.perf_counter() - t0)
            if len(times) >= 3 and time.perf_counter() - t_start > seconds:
                break
    finally:
        torch.set_num_threads(prev)
    return sorted(times)[len(times) // 2], times


def cpu_baseline(n, alpha, seconds):
    """The reference's CPU op sequence on this box's host cores, on the same
    tensor as the headline: at the process's thread budget (torch's intra-op threads =
    OMP_NUM_THREADS, the cores this job may use; `value`), at every CPU in the process's
    affinity mask (`full_affinity`: the host's best figure, stated beside it), and at the
    per-node share floor(cores / 16) a 16-node machine gives each node process
    (node/DPSGDNode.py:434-439 sets floor(cores / procs_per_machine))."""
    cores = torch.get_num_threads()
    t, times = _cpu_steps(n, alpha, seconds, cores)
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    full = None
    if affinity and affinity > cores:
        tf, times_f = _cpu_steps(n, alpha, max(3.0, seconds / 3), affinity)
        full = {"threads": affinity, "value": round(4 * n / tf / 2 ** 30, 4), "unit": "GiB/s",
                "steps": len(times_f),
                "note": "every CPU in the affinity mask (torch.set_num_threads); on a shared "
                        "host these cores also serve other jobs"}
    share = max(1, cores // 16)
    t1, times1 = _cpu_steps(n, alpha, max(3.0, seconds / 3), share)
    return dict(value=4 * n / t / 2 ** 30, unit="GiB/s", cores=cores,
                host_cpu_count=os.cpu_count(), affinity_cpus=affinity,
                cores_note=(f"{cores} threads used (torch intra-op threads = this job's CPU "
                            f"share); the host reports {os.cpu_count()} logical CPUs, "
                            f"{affinity} in this process's affinity mask (timed in "
                            f"full_affinity)"),
                kind="port",
                sample=f"reference ATen-CPU op sequence (oracle/ref_ops.py), N={n}, k={round(alpha*n)}, "
                       f"median of {len(times)} encode+decode steps ({sum(times):.1f} s) at "
                       f"{cores} threads (torch.get_num_threads(), the job's CPU share)",
                full_affinity=full,
                per_node_share={"threads": share, "value": round(4 * n / t1 / 2 ** 30, 4),
                                "unit": "GiB/s", "steps": len(times1),
                                "note": "floor(cores / 16): one of 16 node processes per machine"})


def _finish(dist):
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def main():
    args = parse()
    if args.n is None:
        args.n = C2_N if args.workload == "c4" else NORTH_STAR_N
    launched = "WORLD_SIZE" in os.environ
    if args.gpus is None:  # under torchrun without --gpus: the launcher's rank count
        args.gpus = int(os.environ["WORLD_SIZE"]) if launched else 1
    if args.gpus > 1 and not launched:
        sys.exit(spawn_ranks(args))  # the parent never touches the GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.selftest_spawn:
        print(json.dumps({"rank": rank, "world": world, "local_rank": local_rank,
                          "cpu_baseline_file": bool(os.environ.get("DPZ_BENCH_CPU_BASELINE"))}),
              flush=True)
        return
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks were started")
    dist = None
    if world > 1:
        import torch.distributed as dist_mod
        torch.cuda.set_device(local_rank)
        dist_mod.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        dist = dist_mod
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    repeats = args.repeats or max(5, min(25, math.ceil(4000 / max(1, args.steps))))

    if args.workload == "c4":
        rounds = max(3, min(args.steps, 20))
        warm = max(1, min(args.warmup, 3))
        r = gossip_case(args.n, args.alpha, dev, rank, world, dist, rounds, warm)
        rs = gossip_case(args.n, args.alpha, dev, rank, world, dist, max(3, rounds // 2), warm,
                         exchange="reduce_scatter")
        pe = gossip_case(args.n, args.alpha, dev, rank, world, dist, max(3, rounds // 2), warm,
                         exchange="peer")
        cpu = None
        if rank == 0 and not args.no_cpu:
            # one node's round of the 96 (encode + the MH fold of its neighbours' payloads;
            # eval/96_regular.edges' degree ~4), x96 nodes
            import bench_workloads as bw
            torch.cuda.empty_cache()
            deg = round(2 * r["edges"] / r["nodes"])
            cpu = bw.cpu_partial_round(args.n, args.alpha, deg, 5, scale=r["nodes"], seconds=8.0,
                                       what=f"one of the {r['nodes']} nodes (degree {deg})")
            cpu["value"] = round(r["nodes"] * 4 * args.n / cpu["seconds_per_unit"] / 2 ** 30, 5)
            cpu["unit_note"] = "seconds_per_unit = one round of all 96 nodes"
        if rank == 0:
            print(json.dumps({
                "metric": "GiB/s fp32 params encoded+decoded (device-resident), 1% top-k",
                "value": round(r["value"], 3), "unit": "GiB/s", "n_gpus": world,
                "steps": rounds, "warmup": warm,
                "ms_per_step": round(r["s_step"] * 1e3, 4), "higher_is_better": True,
                "scaling": "strong", "vs_baseline": None, "dtype": "f32",
                "data": "synthetic (x ~ N(0,1), +0.01*N(0,1) per round), device-generated",
                "config": {"workload": "C4: one gossip round of eval/96_regular.edges (96 nodes, "
                                       "190 edges), every node top-k encodes and MH-folds its "
                                       "neighbours' payloads",
                           "n": r["n"], "k": r["k"], "alpha": args.alpha,
                           "parallelism": f"{r['nodes']} nodes sharded over {world} GPU(s), one "
                                          "RCCL all-gather of the payloads per round"},
                "round_alg_bytes": r["alg_bytes_8n"],
                "round_frac_of_hbm_peak": round(r["alg_bytes_8n"] / r["s_step"] / 1e9
                                                / HBM_PEAK_GBS / world, 4),
                "round_frac_of_hbm_peak_fold_12n": round(r["alg_bytes"] / r["s_step"] / 1e9
                                                         / HBM_PEAK_GBS / world, 4),
                "alg_bytes_note": "SURVEY §8(d) C4 accounting: per node encode 8N + 16k, fold 8N "
                                  "+ 8k per payload (the averaged model counted once); "
                                  "*_fold_12n also counts its second write (the node keeps it as "
                                  "model and as init_model, Sharing.py:186-190, "
                                  "PartialModel.py:340-343)",
                "legs_ms": r["legs_ms"],
                "reduce_scatter_mode": {
                    "note": "the over-HBM exchange forced (exchange='reduce_scatter'): payloads "
                            "never replicated; per destination group one batched zero-base fold "
                            "of the owned (A, B) rows, one packed RCCL reduce-scatter, the "
                            "owner's combine" + ("" if world > 1 else
                                                 " (1 GPU: no collective, the legs still run)"),
                    "ms_per_round": round(rs["s_step"] * 1e3, 4),
                    "value": round(rs["value"], 3), "legs_ms": rs["legs_ms"],
                    "rs_group": rs["rs_group"]},
                "peer_mode": {
                    "note": "exchange='peer': each rank sends each other rank only the payloads "
                            "its nodes' neighbours there fold (one all_to_all_single, uneven "
                            "splits), bit-exact fold as in the all-gather mode" +
                            ("" if world > 1 else " (1 GPU: every neighbour is local, no "
                                                  "collective)"),
                    "ms_per_round": round(pe["s_step"] * 1e3, 4),
                    "value": round(pe["value"], 3), "legs_ms": pe["legs_ms"],
                    "remote_payloads_per_rank": pe["peer_recv_payloads"]},
                "cpu_baseline": cpu,
            }), flush=True)
        _finish(dist)
        return
    if args.workload in ("c3", "c5", "e2e", "shard", "fft", "wire", "plugin"):
        import bench_workloads as bw
        cpu = not args.no_cpu
        if args.workload == "plugin":
            r = [bw.plugin_case(dev, "partial", cpu_rounds=int(cpu)),
                 bw.plugin_case(dev, "jwins", cpu_rounds=int(cpu))]
        elif args.workload == "fft":
            r = bw.fft_case(dev, steps=min(args.steps, 30), cpu=cpu)
        elif args.workload == "wire":
            r = bw.wire_case(dev)
        elif args.workload == "shard":
            r = bw.shard_case(dev, rank, world, dist, steps=min(args.steps, 40), cpu=cpu)
        elif args.workload == "c3":
            r = [bw.c3_case(dev, alpha=a, steps=min(args.steps, 40), cpu=cpu) for a in (0.01, 0.1)]
            r.append(bw.c3_case(dev, alpha=0.01, steps=min(args.steps, 40), wavelet="haar",
                                cpu=cpu))
            r.append(bw.c3_round_case(dev, rank, world, dist, rounds=min(args.steps, 10), cpu=cpu))
        elif args.workload == "c5":
            r = bw.c5_case(dev, steps=min(args.steps, 40), streams=args.streams, cpu=cpu)
        else:
            r = {"c2": bw.e2e_case(dev, 11_000_000, 0.01, streams=args.streams, cpu=cpu),
                 "64MiB": bw.e2e_case(dev, 16_777_216, 0.01, streams=args.streams, cpu=cpu),
                 "c5_fp16": bw.e2e_case(dev, 67_108_864, 0.001, fp16=True,
                                        streams=args.streams, cpu=cpu)}
        if rank == 0:
            print(json.dumps({"metric": "GiB/s fp32 params encoded+decoded", "unit": "GiB/s",
                              "workload": args.workload, "n_gpus": world, "result": r}),
                  flush=True)
        _finish(dist)
        return
    r = gpu_case(args.n, args.alpha, dev, 1234 + rank, args.steps, args.warmup, world, dist,
                 rotate=args.rotate, streams=args.streams, repeats=repeats)
    extra = None
    if not args.no_extra:
        # the other single-GPU size beside the headline (C2 when the headline is the 64 MiB
        # north-star tensor), every rank its own node's model (weak, like the headline)
        n2 = C2_N if args.n != C2_N else NORTH_STAR_N
        e = gpu_case(n2, 0.01, dev, 99 + rank, max(20, args.steps // 2), args.warmup,
                     world, dist, streams=args.streams, repeats=repeats)
        extra = None
        if rank == 0:
            b = (e["b_enc"] + e["b_dec"]) * world
            kern2, dk2, _ = kernel_table(e)
            extra = {"workload": workload_name(n2) + ", one per GPU",
                     "n": e["n"], "k": e["k"],
                     "value": round(e["value"], 2), "ms_per_step": round(e["s_step"] * 1e3, 4),
                     "frac_of_hbm_peak": round(b / e["s_step"] / 1e9 / HBM_PEAK_GBS / world, 4),
                     "launch": e["mode"],
                     "one_node_serial_ms_per_step": round(e["s_serial"] * 1e3, 4),
                     "one_node_frac_of_hbm_peak": round(b / e["s_serial"] / 1e9 / HBM_PEAK_GBS / world, 4),
                     f"{e['streams']}_node_ms_per_step": round(e["s_multi"] * 1e3, 4),
                     "host_enqueue_ms_per_step": round(e["s_host"] * 1e3, 4),
                     "roofline": roofline_obj(dk2, e["n"]),
                     "product_one_node": {k_: v for k_, v in e["product"].items() if k_ != "fell_back"},
                     "kernels": kern2,
                     "spread_ms": e["spread_ms"],
                     "fell_back": e["fell_back"]}

    # the gossip round of BASELINE.json C4 (eval/96_regular.edges) at every N: the nodes are
    # sharded over the ranks and each round's payloads cross ranks in one RCCL all-gather, so a
    # multi-GPU run of this bench also times the collective path (strong scaling, 96 nodes fixed)
    gossip = shard_line = None
    if not args.no_extra:
        gossip = gossip_line(gossip_case(C2_N, 0.01, dev, rank, world, dist, rounds=5, warmup=2),
                             world)
        torch.cuda.empty_cache()
        # one C5 tensor (256 MiB, alpha 0.001) sharded over the ranks: the sharded top-k's
        # candidate all-gather is the collective (strong scaling)
        import bench_workloads as bw
        sh = bw.shard_case(dev, rank, world, dist, steps=20)
        shard_line = {k_: (round(v, 4) if isinstance(v, float) else v) for k_, v in sh.items()}
        torch.cuda.empty_cache()

    copy_gbs = None
    if rank == 0:  # context: what a plain device-to-device copy reaches on this box
        a = torch.empty(64 * 2 ** 20, dtype=torch.float32, device=dev)
        b = torch.empty_like(a)
        for _ in range(3):
            b.copy_(a)
        t_copy = timed_loop(lambda: b.copy_(a), 20, torch.cuda.current_stream(dev))
        copy_gbs = round(2 * a.numel() * 4 / t_copy / 1e9, 1)
        del a, b

    cpu = None
    if rank == 0 and not args.no_cpu:
        path = os.environ.get("DPZ_BENCH_CPU_BASELINE")
        if path and os.path.exists(path):  # timed by the spawning parent before the ranks
            with open(path) as f:
                cpu = json.load(f)
            cpu["timed_by"] = "the bench.py parent process before the GPU ranks started"
        else:
            cpu = cpu_baseline(args.n, args.alpha,
                               args.cpu_seconds if world == 1 else min(args.cpu_seconds, 8.0))
            if world > 1:
                cpu["timed_by"] = "rank 0 after the GPU legs (the other ranks wait at a barrier)"

    if rank == 0:
        t_enc, t_dec = r["t_enc"], r["t_dec"]
        dec_gbs = r["b_dec"] / t_dec / 1e9
        enc_gbs = r["b_enc"] / t_enc / 1e9
        step_gbs = (r["b_enc"] + r["b_dec"]) / r["s_step"] / 1e9
        serial_b = r["b_enc"] + r["b_dec"]
        kern, dk, _ = kernel_table(r)
        line = {
            "metric": "GiB/s fp32 params encoded+decoded (device-resident), 1% top-k",
            "value": round(r["value"], 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(r["s_step"] * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (x ~ N(0,1), x0 = x - 0.01*N(0,1), device-generated)",
            "config": {
                "workload": workload_name(r["n"]),
                "n": r["n"], "k": r["k"], "alpha": args.alpha,
                "parallelism": (f"{world} GPU(s) x {r['streams']} concurrent node codecs (one "
                                f"stream each), no collective" if r["mode"] == "multi" else
                                f"{world} GPU(s) x 1 node codec, no collective"),
                "launch": ("native batched enqueue (dpz_encode_replace_batch, DPZ_BATCH_HINT: "
                           "each encode's key window from the previous encode's exact threshold "
                           "on its stream's workspace, no sample launch); step i = encode "
                           f"of node state i with the replace decode of state i - {r['streams']}'s "
                           f"payload over its x fused in, on stream i % {r['streams']}; "
                           "counters as the PartialModel plugin keeps them (RingCounter: payload "
                           "indices into a ring slot, folded into the counter when the ring is "
                           "full and at the end of every timed region, inside it)"
                           if r["mode"] == "multi" else
                           "native batched enqueue (dpz_encode_replace_batch, DPZ_BATCH_HINT), "
                           "one stream; "
                           "step i = encode of node state i with the replace decode of state "
                           "i - 1's payload over state i's x fused into the encoder's launches "
                           "(filter writes the copy of x, select scatters the entries)"),
                "rotated_states": r["rotate"],
                "timing": (f"median of {r['repeats']} timed regions of exactly {args.steps} "
                           f"steps (each: barrier + synchronize on both sides, max over ranks)"),
            },
            "spread_ms_per_step": r["spread_ms"],
            "roofline": roofline_obj(dk, r["n"]),
            "stages": {
                "encode": {"avg_us": round(t_enc * 1e6, 3), "alg_bytes": r["b_enc"],
                           "GBps": round(enc_gbs, 1), "frac": round(enc_gbs / HBM_PEAK_GBS, 4),
                           "sampled_path_fell_back": r["fell_back"]},
                "decode": {"avg_us": round(t_dec * 1e6, 3), "alg_bytes": r["b_dec"],
                           "GBps": round(dec_gbs, 1), "frac": round(dec_gbs / HBM_PEAK_GBS, 4)},
                "step_frac_of_hbm_peak": round(step_gbs / HBM_PEAK_GBS, 4),
                "one_node_serial_ms_per_step": round(r["s_serial"] * 1e3, 5),
                "one_node_frac_of_hbm_peak": round(serial_b / r["s_serial"] / 1e9 / HBM_PEAK_GBS, 4),
                f"{r['streams']}_node_ms_per_step": round(r["s_multi"] * 1e3, 5),
                "host_enqueue_ms_per_step": round(r["s_host"] * 1e3, 5),
                "product_one_node": {k_: v for k_, v in r["product"].items() if k_ != "fell_back"},
                "kernels": kern,
                "torch_copy_GBps_256MiB": copy_gbs,
            },
            "cpu_baseline": cpu,
            "secondary": extra,
            "gossip_round": gossip,
            "shard": shard_line,
        }
        print(json.dumps(line), flush=True)
    _finish(dist)


def kernel_table(r):
    """Per-kernel averages of the one-node step with the per-launch HIP event-pair overhead
    removed, and the dominant kernel (most device time per step).  The overhead is measured on
    the replace decode (the one kernel also timed back to back: event-pair average -
    back-to-back average) and subtracted from every kernel's event-pair average, so the
    averages are what rocprofv3 --kernel-trace reports (profiles/)."""
    kern = {nm: dict(v) for nm, v in r["kernels"].items()}
    t_dec = r["t_dec"]
    bias = 0.0
    if "fold" in kern:
        bias = max(0.0, kern["fold"]["avg_us"] - t_dec * 1e6)
    for name, kv in kern.items():
        b = kernel_alg_bytes(name, r["n"], r["k"])
        kv["avg_us_event_pair"] = round(kv["avg_us"], 3)
        kv["avg_us"] = max(kv["avg_us"] - bias, 1e-3)
        kv["alg_bytes"] = b
        kv["GBps"] = round(b / (kv["avg_us"] * 1e-6) / 1e9, 1) if b else 0.0
        kv["avg_us"] = round(kv["avg_us"], 3)
    dom = max(kern, key=lambda nm: kern[nm]["avg_us"] * kern[nm]["launches_per_step"])
    dk = dict(kern[dom])
    dk["name"] = dom
    dk["timing"] = (f"per-launch HIP event pair (library KernelTimer) minus the event-pair "
                    f"overhead {bias:.3f} us (replace kernel: event-pair avg - back-to-back avg)")
    if dom == "fold" and kern[dom]["launches_per_step"] == 1.0:
        # the decode is this one launch: its back-to-back average on the launch stream (HIP
        # events around the whole loop) has no per-launch event overhead
        dk["avg_us"] = round(t_dec * 1e6, 3)
        dk["GBps"] = round(dk["alg_bytes"] / t_dec / 1e9, 1)
        dk["timing"] = "back-to-back launches, HIP events around the loop on the launch stream"
    return kern, dk, bias


def load_rocprof(kernel, n):
    """(avg launch us, source) of `kernel` from the committed rocprofv3 --stats summary of the
    bench's own one-stream command at this tensor size (profiles/rocprof_latest*.json, written by
    tools/kstats2json.py), or (None, None)."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "rocprof_latest*.json"))):
        with open(path) as f:
            doc = json.load(f)
        if doc.get("n") != n:
            continue
        ent = doc.get("kernels", {}).get(kernel)
        if ent:
            return ent["avg_us"], os.path.relpath(path, ROOT)
    return None, None


def roofline_obj(dk, n):
    """The line's `roofline` object for the dominant kernel `dk` (kernel_table) at size n, with
    the HBM traffic of the committed PMC pass at the same n (profiles/pmc_latest*.json).  The
    live launch time (event pairs, calibrated) is quoted beside the committed rocprofv3 summary
    of the same command (profiles/rocprof_latest*.json); `frac` takes the slower of the two, so
    the line never claims more than the profile shows."""
    rp_us, rp_src = load_rocprof(dk["name"], n)
    live_frac = dk["GBps"] / HBM_PEAK_GBS
    frac, achieved, basis = live_frac, dk["GBps"], "live"
    if rp_us:
        rp_gbps = dk["alg_bytes"] / (rp_us * 1e-6) / 1e9
        if rp_gbps < dk["GBps"]:
            frac, achieved, basis = rp_gbps / HBM_PEAK_GBS, round(rp_gbps, 1), "rocprof"
    return {
        "bound": "hbm",
        "kernel": dk["name"],
        "achieved": achieved,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(frac, 4),
        "frac_basis": basis,
        "traffic": load_pmc(dk["name"], n),
        "alg_bytes_per_launch": dk["alg_bytes"],
        "avg_launch_us": dk["avg_us"],
        "live_frac": round(live_frac, 4),
        "rocprof_avg_launch_us": rp_us,
        "rocprof_summary": rp_src,
        "timing": dk["timing"],
    }


def gossip_line(gr, world):
    return {"workload": "C4: one gossip round of eval/96_regular.edges (96 nodes, 190 "
                        "edges): every node top-k encodes, payloads all-gathered over RCCL, "
                        "every node MH-folds its neighbours' payloads",
            "n": gr["n"], "k": gr["k"],
            "value": round(gr["value"], 3), "unit": "GiB/s",
            "ms_per_round": round(gr["s_step"] * 1e3, 4), "scaling": "strong",
            "parallelism": f"{gr['nodes']} nodes sharded over {world} GPU(s), "
                           + ("one RCCL all-gather of the payloads per round" if world > 1
                              else "no collective on one GPU"),
            "legs_ms": gr["legs_ms"],
            "round_alg_bytes": gr["alg_bytes_8n"],
            "round_frac_of_hbm_peak": round(gr["alg_bytes_8n"] / gr["s_step"] / 1e9
                                            / HBM_PEAK_GBS / world, 4),
            "round_frac_of_hbm_peak_fold_12n": round(gr["alg_bytes"] / gr["s_step"] / 1e9
                                                     / HBM_PEAK_GBS / world, 4),
            "alg_bytes_note": "SURVEY §8(d) C4 accounting: per node encode 8N + 16k, fold 8N + 8k "
                              "per payload (the averaged model counted once); *_fold_12n also "
                              "counts its second write (model and init_model, Sharing.py:186-190, "
                              "PartialModel.py:340-343)"}

if __name__ == "__main__":
    main()
