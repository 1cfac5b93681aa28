"""Host -> device ways for a received wire leg (a Python bytes object from pickle.loads), timed on
the GPU box: (a) torch's parallel copy into a kept pinned buffer, then an async DMA (the plugin's
path); (b) a pageable tensor's .to(device); (c) hipHostRegister of the bytes' own pages, a DMA
straight from them, unregister; (d) numpy's single-threaded copy into the pinned buffer.
Prints one JSON line per size: median ms of each way and the host-copy rate."""
import ctypes
import json
import sys
import time
import warnings

import numpy as np
import torch


def med(f, reps=9):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return 1e3 * sorted(ts)[len(ts) // 2]


def main():
    dev = torch.device("cuda:0")
    torch.cuda.init()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    out = []
    for mb in [float(a) for a in sys.argv[1:]] or [4.0, 16.0, 48.0]:
        n = int(mb * 2 ** 20)
        src = np.random.default_rng(1).integers(0, 255, n, dtype=np.uint8).tobytes()
        a = np.frombuffer(src, dtype=np.uint8)
        pin = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        dst = torch.empty(n, dtype=torch.uint8, device=dev)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            ta_view = torch.from_numpy(a)

        def way_a():
            pin.copy_(ta_view)
            dst.copy_(pin, non_blocking=True)
            torch.cuda.synchronize()

        def host_only():
            pin.copy_(ta_view)

        def way_b():
            dst.copy_(ta_view)
            torch.cuda.synchronize()

        def way_c():
            p = a.ctypes.data
            rc = hip.hipHostRegister(p, n, 0)
            if rc != 0:
                raise RuntimeError(f"hipHostRegister rc={rc}")
            try:
                dst.copy_(ta_view, non_blocking=True)
                torch.cuda.synchronize()
            finally:
                hip.hipHostUnregister(p)

        def way_d():
            np.copyto(pin.numpy(), a)

        def dma_only():
            dst.copy_(pin, non_blocking=True)
            torch.cuda.synchronize()

        r = {"MiB": mb, "threads": torch.get_num_threads()}
        for name, f in (("a_pinned_copy_then_dma", way_a), ("host_copy_torch", host_only),
                        ("host_copy_numpy", way_d), ("dma_from_pinned", dma_only),
                        ("b_pageable_to", way_b)):
            r[name + "_ms"] = round(med(f), 3)
        try:
            r["c_register_dma_unregister_ms"] = round(med(way_c), 3)
        except Exception as e:  # noqa: BLE001
            r["c_error"] = repr(e)
        t0 = torch.get_num_threads()
        for t in (1, 4, 8, 32):
            torch.set_num_threads(t)
            r[f"host_copy_torch_{t}t_ms"] = round(med(host_only), 3)
        torch.set_num_threads(t0)
        # cold: a fresh bytes object every repetition (what pickle.loads hands the receiver)
        import pickle
        wire = pickle.dumps({"b": src})

        def cold(way):
            ts = []
            for _ in range(7):
                fresh = pickle.loads(wire)["b"]
                fa = np.frombuffer(fresh, dtype=np.uint8)
                with warnings.catch_warnings():
                    warnings.simplefilter("ignore")
                    ft = torch.from_numpy(fa)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                if way == "a":
                    pin.copy_(ft)
                    dst.copy_(pin, non_blocking=True)
                elif way == "a_host":
                    pin.copy_(ft)
                elif way == "b":
                    dst.copy_(ft)
                else:
                    hip.hipHostRegister(fa.ctypes.data, n, 0)
                    dst.copy_(ft, non_blocking=True)
                    torch.cuda.synchronize()
                    hip.hipHostUnregister(fa.ctypes.data)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t1)
            return round(1e3 * sorted(ts)[len(ts) // 2], 3)

        for w in ("a", "a_host", "b", "c"):
            r[f"cold_{w}_ms"] = cold(w)
        r["host_copy_torch_GBps"] = round(n / r["host_copy_torch_ms"] / 1e6, 2)
        r["host_copy_numpy_GBps"] = round(n / r["host_copy_numpy_ms"] / 1e6, 2)
        out.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
