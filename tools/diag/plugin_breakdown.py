"""Diagnostic: stamped parts of a node's plugin round (bench_workloads.plugin_case: PartialModel +
Elias at C2, or with argv[1] == "jwins" JWINS + EliasFpzip at 25 M).  Every listed method is
wrapped with a timer that synchronises the device on entry and exit, so each part's time includes
its own device work; nested parts are reported inclusive.  One JSON line: per part the median ms
per round and the call count per round."""
import json
import os
import pickle
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench_workloads as bw  # noqa: E402
from decentralizepy_amd import codec  # noqa: E402
from decentralizepy_amd.compression import Elias, EliasFpzip  # noqa: E402
from decentralizepy_amd.sharing import PartialModel, Sharing  # noqa: E402
from decentralizepy_amd.sharing.JWINS import Wavelet  # noqa: E402

if os.environ.get("LOAD_FLAT_OLD") == "1":  # A/B: the unpipelined D2H + load_state_dict
    from decentralizepy_amd._device import to_host

    def _load_flat_old(self, out_dev):
        flat = to_host(out_dev, self.staging, "result", own=False)
        self.model.load_state_dict(self._unflatten(flat))
    Sharing.Sharing._load_flat = _load_flat_old

kind = sys.argv[1] if len(sys.argv) > 1 else "jwins"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 6
acc = defaultdict(list)
cur = defaultdict(float)
cnt = defaultdict(int)
allocs = []


# NOSYNC=1: host time only (no device synchronisation around a part: the asynchronous receive
# path is timed as it runs; a part then shows the host work plus whatever it waits on)
SYNC = os.environ.get("NOSYNC") != "1"
if os.environ.get("ASYNC") == "0":  # A/B: the synchronous payload decodes
    Elias.Elias.async_decode = False


def wrap(owner, name, label):
    fn = getattr(owner, name)

    def timed(*a, **kw):
        if SYNC:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn(*a, **kw)
        if SYNC:
            torch.cuda.synchronize()
        cur[label] += time.perf_counter() - t0
        cnt[label] += 1
        return r
    setattr(owner, name, timed)


S, P, W = Sharing.Sharing, PartialModel.PartialModel, Wavelet.Wavelet
for owner, name, label in [
        (S, "get_data_to_send", "send.total"), (S, "_pre_step", "send.pre_step"),
        (P, "_pre_step", "send.pre_step"), (P, "_encode", "send.encode"),
        (W, "_encode", "send.encode"), (W, "_full_share", "send.full_share"),
        (P, "compress_data", "send.compress"),
        (W, "_averaging", "recv.total"), (S, "_averaging", "recv.total"),
        (S, "_pop_payloads", "recv.pop_payloads"), (P, "decompress_data", "recv.decompress"),
        (S, "decompress_data", "recv.decompress"),
        (Elias.Elias, "decompress_device", "recv.elias_decode"),
        (EliasFpzip.EliasFpzip, "decompress_float_device", "recv.float_decode"),
        (P, "_device_payload", "recv.h2d_payload"), (S, "_device_payload", "recv.h2d_payload"),
        (S, "_fold", "recv.fold"), (S, "_local_flat_device", "recv.local_flat"),
        (S, "_load_flat", "recv.load_flat"), (P, "_load_flat", "recv.load_flat"),
        (P, "_post_step", "recv.post_step"),
        (codec, "waverec", "recv.waverec")]:
    wrap(owner, name, label)
from decentralizepy_amd import _device  # noqa: E402

def _get_stamped(self, name, n, dtype):
    """Staging.get with its two waits stamped apart: the event of the buffer's previous DMA and
    a page-locked allocation (a growth), per buffer name."""
    key = (name, dtype)
    ev = self._events.pop(key, None)
    t0 = time.perf_counter()
    if ev is not None:
        ev.synchronize()
    t1 = time.perf_counter()
    cur["stage.get_event_wait"] += t1 - t0
    cur[f"stage.get_event_wait[{name}]"] += t1 - t0
    buf = self._bufs.get(key)
    grow = buf is None or buf.numel() < n
    if ev is not None:
        self._events[key] = ev
    r = _get_orig(self, name, n, dtype)
    t2 = time.perf_counter()
    if grow:
        allocs.append((name, int(n), None if buf is None else int(buf.numel()),
                       round(1e3 * (t2 - t1), 3)))
        cur["stage.get_alloc"] += t2 - t1
        cur[f"stage.get_alloc[{name}]"] += t2 - t1
        cnt["stage.get_alloc"] += 1
    return r


_get_orig = _device.Staging.get
_device.Staging.get = _get_stamped
for owner, name, label in [  # the staging and launch pieces of the receive decodes (Elias, "host_copy_into", "stage.host_copy"),
        (EliasFpzip, "host_copy_into", "stage.host_copy"), (codec, "fpz_decode", "stage.fpz_decode"),
        (codec, "elias_decode_async", "stage.elias_decode_async"),
        (codec, "elias_decode", "stage.elias_decode_sync")]:
    wrap(owner, name, label)
for mod in (Sharing, PartialModel, Wavelet):  # the modules' own to_host bindings
    wrap(mod, "to_host", "any.to_host")

# plugin_case's own round loop, with the pickle legs stamped too
_dumps, _loads = pickle.dumps, pickle.loads


def dumps(o, *a, **kw):
    t0 = time.perf_counter()
    r = _dumps(o, *a, **kw)
    cur["wire.pickle_dumps"] += time.perf_counter() - t0
    return r


def loads(b, *a, **kw):
    t0 = time.perf_counter()
    r = _loads(b, *a, **kw)
    cur["wire.pickle_loads"] += time.perf_counter() - t0
    return r


pickle.dumps, pickle.loads = dumps, loads
dev = torch.device("cuda", 0)
bw.plugin_case(dev, kind, rounds=1, warmup=1, cpu_rounds=0)  # warm
cur.clear()
cnt.clear()


def _warm():
    allocs.clear()
    cur.clear()
    cnt.clear()


# counters from the first timed round on, after 3 warm rounds of the same plugins (their pinned
# buffers grown to the payload sizes the alpha draws produce)
res = bw.plugin_case(dev, kind, rounds=rounds, warmup=3, cpu_rounds=0, on_warm=_warm)
# the neighbours' rounds (3 get_data_to_send per round) are inside the same counters: report the
# node's own parts per round by dividing the send parts by 4 plugins and the rest by rounds
out = {"kind": kind, "rounds": rounds, "round": res, "sync_wrapped": SYNC,
       "async_decode": Elias.Elias.async_decode,
       "note": "send.* parts are summed over the node and its 3 neighbours' get_data_to_send "
               "(4 calls per round); recv.* and wire.pickle_loads are the node's own; "
               "ms per round"}
out["parts_ms_per_round"] = {k: round(v / rounds * 1e3, 3) for k, v in sorted(cur.items())}
out["pinned_allocs_timed_rounds"] = allocs
out["calls_per_round"] = {k: round(v / rounds, 2) for k, v in sorted(cnt.items())}
print(json.dumps(out))
