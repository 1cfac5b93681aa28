"""Diagnostic A/B: per-kernel device time of one node's encode (top-k + counter) and replace
decode on HBM-rotated C2 / 64 MiB states, for each library build named on the command line
(tools/diag/variants/lib_<name>.so; "cur" = the in-tree build).  Each build runs in its own
process; the builds alternate twice so box drift shows."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(n):
    import torch
    sys.path.insert(0, ROOT)
    from decentralizepy_amd import codec
    from decentralizepy_amd._lib import DPZ_BATCH_DECODE, DPZ_BATCH_ENCODE
    dev = torch.device("cuda", 0)
    k = round(0.01 * n)
    R = 6
    g = torch.Generator(device=dev).manual_seed(3)
    sets = []
    for _ in range(R):
        x = torch.randn(n, device=dev, generator=g)
        sets.append(dict(x=x, x0=x - 0.01 * torch.randn(n, device=dev, generator=g),
                         counter=torch.zeros(n, dtype=torch.int32, device=dev),
                         idx=torch.empty(k, dtype=torch.int32, device=dev),
                         val=torch.empty(k, device=dev), out=torch.empty(n, device=dev)))
    st = torch.cuda.Stream(dev)
    b = codec.NodeStepBatch(sets, n, k, [st], [codec.Workspace(dev)])
    for _ in range(3):
        b.run()
    torch.cuda.synchronize()
    res = {}
    with codec.KernelTimer() as kt:
        with torch.cuda.stream(st):
            torch.cuda._sleep(int(100e6))
        for _ in range(10):
            b.run()
        torch.cuda.synchronize()
    res.update({kk: round(v[0] / v[1] * 1e3, 2) for kk, v in kt.result.items()})
    for what, nm in ((DPZ_BATCH_ENCODE, "enc_loop"), (DPZ_BATCH_DECODE, "dec_loop"),
                     (DPZ_BATCH_ENCODE | DPZ_BATCH_DECODE, "step_loop")):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        with torch.cuda.stream(st):
            torch.cuda._sleep(int(100e6))
            e0.record(st)
        for _ in range(10):
            b.run(what)
        e1.record(st)
        e1.synchronize()
        res[nm] = round(e0.elapsed_time(e1) / (10 * R) * 1e3, 2)
    res["sticky"] = b.sticky_status(clear=True)
    print(json.dumps(res))


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(int(sys.argv[2]))
        sys.exit(0)
    names = sys.argv[1:]
    for n in (11_000_000, 16_777_216):
        for rep in range(2):
            for nm in names:
                env = dict(os.environ)
                if nm != "cur":
                    env["DPZ_CODEC_LIB"] = os.path.join(ROOT, "tools", "diag", "variants",
                                                        f"lib_{nm}.so")
                r = subprocess.run([sys.executable, __file__, "--child", str(n)], env=env,
                                   capture_output=True, text=True, timeout=120)
                line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-300:]
                print(f"n={n} {nm:>10}: {line}", flush=True)
