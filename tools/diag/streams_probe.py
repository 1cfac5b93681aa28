"""Do two torch streams run kernels concurrently on this box, and what does a cross-stream event
wait cost?  (diagnostic only)"""
import time
import torch

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
hi = torch.cuda.Stream(dev, priority=-1)
cyc = int(50e6)
torch.cuda._sleep(cyc)
torch.cuda.synchronize()


def timeit(fn, reps=3):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3


def one():
    with torch.cuda.stream(s1):
        torch.cuda._sleep(cyc)


def two_same():
    with torch.cuda.stream(s1):
        torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)


def two_par(a=s1, b=s2):
    with torch.cuda.stream(a):
        torch.cuda._sleep(cyc)
    with torch.cuda.stream(b):
        torch.cuda._sleep(cyc)


print("streams", s1.cuda_stream, s2.cuda_stream, hi.cuda_stream)
print("one sleep ms", timeit(one))
print("two same-stream ms", timeit(two_same))
print("two parallel ms", timeit(two_par))
print("two parallel (hi prio) ms", timeit(lambda: two_par(s1, hi)))
# ping-pong chain of tiny kernels with cross-stream waits
x = torch.zeros(1, device=dev)
ev = [torch.cuda.Event() for _ in range(2)]


def pingpong(n=200):
    for i in range(n):
        s = s1 if i % 2 == 0 else s2
        with torch.cuda.stream(s):
            if i:
                s.wait_event(ev[(i - 1) % 2])
            x.add_(1)
            ev[i % 2].record(s)


def chain(n=200):
    with torch.cuda.stream(s1):
        for i in range(n):
            x.add_(1)


print("200 tiny kernels one stream us/kernel", timeit(chain) * 1e3 / 200)
print("200 tiny kernels ping-pong us/kernel", timeit(pingpong) * 1e3 / 200)
# bandwidth-bound kernels on two streams: copies of 256 MiB
a = torch.empty(64 * 2 ** 20, device=dev)
b = torch.empty_like(a)
c = torch.empty_like(a)
d = torch.empty_like(a)


def cp1():
    with torch.cuda.stream(s1):
        b.copy_(a)
        d.copy_(c)


def cp2():
    with torch.cuda.stream(s1):
        b.copy_(a)
    with torch.cuda.stream(s2):
        d.copy_(c)


print("2 copies one stream ms", timeit(cp1), "two streams ms", timeit(cp2))
