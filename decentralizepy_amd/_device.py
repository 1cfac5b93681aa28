"""Device plumbing for the Sharing plugins: device choice, pinned host staging, host views.

The reference runs one node per OS process with the model on the CPU (node/Node.py,
eval/testing.py:54-80).  The plugins keep the codec state on the GPU chosen by the node's local
rank and move only the flat model and the payloads across PCIe, through pinned staging buffers.
"""
import functools
import os
import warnings

import numpy as np
import torch


def pick_device(rank):
    """GPU for a node process: DPZ_DEVICE overrides, else local rank modulo the visible GPUs."""
    if not torch.cuda.is_available():
        raise RuntimeError("decentralizepy_amd needs a ROCm GPU (MI355X); none is visible. "
                           "There is no CPU path.")
    env = os.environ.get("DPZ_DEVICE")
    if env is not None:
        return torch.device("cuda", int(env))
    return torch.device("cuda", int(rank) % torch.cuda.device_count())


def _pinned_cap():
    """Pinned host bytes one plugin may hold (DPZ_PINNED_MB, default 1024 MiB).  decentralizepy
    runs procs_per_machine node processes per host (16 in the tutorial), each with its own
    staging, so the cap bounds the page-locked total per machine."""
    return int(float(os.environ.get("DPZ_PINNED_MB", "1024")) * 2 ** 20)


class Staging:
    """Reusable pinned host buffers keyed by (name, dtype); grown on demand, within a byte cap.

    A buffer handed out again waits for the last asynchronous copy that read it (``mark``),
    so a pinned source is never overwritten while its DMA is in flight.  ``get`` returns None
    when a buffer would take the total past ``cap_bytes``: the caller then copies through
    pageable memory (synchronous, correct, slower)."""

    def __init__(self, cap_bytes=None):
        self._bufs = {}
        self._events = {}
        self.cap = _pinned_cap() if cap_bytes is None else int(cap_bytes)
        self.total = 0

    def get(self, name, n, dtype):
        key = (name, dtype)
        ev = self._events.pop(key, None)
        if ev is not None:
            ev.synchronize()
        buf = self._bufs.get(key)
        if buf is None or buf.numel() < n:
            esz = torch.empty(0, dtype=dtype).element_size()
            old = 0 if buf is None else buf.numel() * buf.element_size()
            # exact the first time (the model-sized buffers never grow); a buffer that grows is
            # grown to the next power of two (payload sizes vary round to round and each growth
            # is a page-locked allocation, ~1 ms per 10 MB on the box: it grows a few times in
            # its life, not every round), exact if that would pass the cap
            want = max(int(n), 1) if buf is None else 1 << max(int(n) - 1, 1).bit_length()
            if self.total - old + want * esz > self.cap:
                want = max(int(n), 1)
            size = want * esz
            if self.total - old + size > self.cap:
                return None
            self._bufs.pop(key, None)
            del buf
            buf = torch.empty(want, dtype=dtype, pin_memory=True)
            self._bufs[key] = buf
            self.total += size - old
        return buf[:n]

    def mark(self, name, dtype, stream):
        ev = torch.cuda.Event()
        ev.record(stream)
        self._events[(name, dtype)] = ev


def _as_cpu_tensor(src):
    """A CPU tensor view (no copy) of a bytes-like object, numpy array or CPU tensor.  A
    read-only buffer (a bytes object from pickle.loads) is only read, so torch's warning about
    non-writable memory does not apply."""
    if isinstance(src, torch.Tensor):
        return src
    if isinstance(src, (bytes, bytearray, memoryview)):
        a = np.frombuffer(memoryview(src), dtype=np.uint8)
    else:
        a = np.ascontiguousarray(src)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return torch.from_numpy(a)


def host_copy_into(dst, src):
    """``dst[:] = src`` for a CPU (pinned staging) tensor with torch's parallel copy (its intra-op
    threads: the node process's CPU share) instead of numpy's single-threaded slice assignment —
    the receive path stages tens of MB of payload bytes per round (JWINS)."""
    t = _as_cpu_tensor(src).reshape(-1)
    if t.dtype != dst.dtype:
        t = t.view(dst.dtype) if t.element_size() == dst.element_size() else t.to(dst.dtype)
    dst.view(-1)[:t.numel()].copy_(t)
    return dst


def host_owned(t):
    """A numpy array owning a copy of the CPU tensor ``t`` (pinned staging about to be reused),
    made with torch's parallel copy."""
    return torch.empty(t.shape, dtype=t.dtype).copy_(t).numpy()


def flatten_state(state_dict):
    """``torch.cat`` of the flattened state tensors (reference sharing/Sharing.py:93-112)."""
    return torch.cat([v.flatten() for v in state_dict.values()])


def state_version(state_dict):
    """In-place modification stamp of a state_dict (torch version counters of its tensors)."""
    return tuple(v._version for v in state_dict.values())


def state_to_device(state_dict, device, staging, name):
    """``flatten_state`` + H2D in one host pass: the state tensors are concatenated straight
    into the pinned staging buffer (``torch.cat(..., out=pinned)``), then one async DMA — no
    intermediate flat copy of the model on the host (the reference's ``torch.cat``,
    sharing/PartialModel.py:312-316, is this concatenation)."""
    vals = [v.flatten() for v in state_dict.values()]
    # the dtype the reference's torch.cat produces (type promotion: int buffers such as
    # BatchNorm's num_batches_tracked, or fp16 tensors beside fp32 ones, become fp32)
    dt = functools.reduce(torch.promote_types, [v.dtype for v in vals], torch.bool)
    if dt != torch.float32:
        raise NotImplementedError(
            f"the flattened model is {dt}; the HIP codec handles fp32 models only")
    n = sum(v.numel() for v in vals)
    host = staging.get(name, n, torch.float32)
    if host is None:  # over the pinned cap: pageable copy
        return torch.cat(vals).to(device)
    torch.cat(vals, out=host)
    out = host.to(device, non_blocking=True)
    staging.mark(name, torch.float32, torch.cuda.current_stream(device))
    return out


def to_device_flat(flat_cpu, device, staging, name):
    """H2D of a host fp32 vector through a pinned buffer."""
    if flat_cpu.dtype != torch.float32:
        raise NotImplementedError(
            f"the flattened model is {flat_cpu.dtype}; the HIP codec handles fp32 models only")
    host = staging.get(name, flat_cpu.numel(), torch.float32)
    if host is None:  # over the pinned cap: pageable copy
        return flat_cpu.to(device)
    host.copy_(flat_cpu)
    out = host.to(device, non_blocking=True)
    staging.mark(name, torch.float32, torch.cuda.current_stream(device))
    return out


def h2d_array(arr, dtype, device, staging, name):
    """H2D of a host numpy array (a received payload leg) through the pinned buffer ``name``:
    the host copy into pinned memory, then an asynchronous DMA on the current stream, so the
    caller's host work on the next payload (unpickled dict, decompression) overlaps this DMA
    (reference wire boundary: node/DPSGDNode.py receive -> Sharing._averaging).  The buffer is
    not reused before its DMA has completed (Staging events)."""
    a = np.ascontiguousarray(arr, dtype=dtype)
    tdt = torch.from_numpy(a[:0]).dtype
    host = staging.get(name, a.size, tdt)
    if host is None:  # over the pinned cap: pageable copy
        return torch.from_numpy(a.reshape(-1)).to(device)
    host_copy_into(host, a)
    out = host.to(device, non_blocking=True)
    staging.mark(name, tdt, torch.cuda.current_stream(device))
    return out


def load_flat(model, flat_dev, staging, name, chunk=1 << 22):
    """``model.load_state_dict(unflatten(flat_dev))`` (reference sharing/Sharing.py:186-190) with
    the D2H pipelined against the host copy: the flat vector comes back in chunks of ``chunk``
    elements (asynchronous DMAs into one pinned buffer, an event each), and each state tensor's
    range is copied into the tensor as soon as its chunks have landed, so the copy of chunk i
    overlaps the DMA of chunk i + 1.  Values, dtype conversion (``copy_``) and the tensors written
    are those of ``load_state_dict``; a model with load_state_dict hooks, a flat size that does
    not match, or a buffer over the pinned cap takes ``load_state_dict`` itself."""
    sd = model.state_dict()
    n = flat_dev.numel()
    hooks = any(m._load_state_dict_pre_hooks or m._load_state_dict_post_hooks
                for m in model.modules())
    host = None if hooks or sum(v.numel() for v in sd.values()) != n else \
        staging.get(name, n, torch.float32)
    if host is None:
        flat = flat_dev.cpu()
        out, start = {}, 0
        for key, v in sd.items():
            out[key] = flat[start:start + v.numel()].view(v.shape)
            start += v.numel()
        model.load_state_dict(out)
        return
    stream = torch.cuda.current_stream(flat_dev.device)
    chunk = max(int(chunk), 1)
    landed = []
    for s0 in range(0, n, chunk):
        e0 = min(n, s0 + chunk)
        host[s0:e0].copy_(flat_dev[s0:e0], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(stream)
        landed.append((e0, ev))
    ci, done = 0, 0

    def wait_to(end):
        nonlocal ci, done
        while done < end:
            e0, ev = landed[ci]
            ev.synchronize()
            done, ci = e0, ci + 1

    with torch.no_grad():
        start = 0
        for v in sd.values():
            end = start + v.numel()
            if v.is_cuda:  # a device-resident model: one device copy
                v.copy_(flat_dev[start:end].view(v.shape))
            elif v.is_contiguous():
                flat_v = v.view(-1)
                a = start
                while a < end:  # the tensor's range chunk by chunk, as the chunks land
                    b = min(end, (a // chunk + 1) * chunk)
                    wait_to(b)
                    flat_v[a - start:b - start].copy_(host[a:b])
                    a = b
            else:
                wait_to(end)
                v.copy_(host[start:end].view(v.shape))
            start = end
    wait_to(n)  # the pinned buffer is free for the next call


class PayloadNames:
    """Pinned-buffer names for received payload legs: a ring of ``slots`` names, so consecutive
    legs use distinct buffers and a reused buffer waits only for its own earlier DMA (Staging).
    A few slots cover the legs in flight (the next payload's host work overlaps the previous
    DMA); more would only pin more memory: a full-model payload (Sharing, Choco) pins 4N bytes
    per slot, within the Staging cap."""

    def __init__(self, slots=8):
        self.i = 0
        self.slots = slots

    def __call__(self, leg):
        self.i = (self.i + 1) % self.slots
        return f"pay{self.i}_{leg}"


def to_host(t, staging, name, own=True):
    """D2H into a pinned buffer; returns a numpy array that owns its memory, or with
    ``own=False`` a view of the pinned buffer, valid until the next ``to_host`` of ``name`` (for
    a result consumed at once: the averaged model ``load_state_dict`` copies into the model)."""
    host = staging.get(name, t.numel(), t.dtype)
    if host is None:  # over the pinned cap: pageable copy
        return t.cpu().numpy().copy()
    host.copy_(t, non_blocking=True)
    torch.cuda.current_stream(t.device).synchronize()
    return host_owned(host) if own else host.numpy()


class DeviceCounter:
    """Host-visible view of the device-resident ``shared_parameters_counter``.

    The reference keeps the counter as a CPU int32 tensor on the model
    (sharing/PartialModel.py:143-145) and the node dumps it with ``.numpy().tolist()`` at the end
    of a run (node/DPSGDNode.py:186-194); this view offers the same calls, copying on demand.
    """

    def __init__(self, t):
        self.device_tensor = t

    def numpy(self):
        return self.device_tensor.cpu().numpy()

    def cpu(self):
        return self.device_tensor.cpu()

    def tolist(self):
        return self.numpy().tolist()

    @property
    def shape(self):
        return self.device_tensor.shape

    def __len__(self):
        return self.device_tensor.numel()

    def __getitem__(self, item):
        """Index on the device and copy only the selection (a CPU tensor, as indexing the
        reference's CPU counter returns); host index arrays are moved to the device first."""
        if isinstance(item, (np.ndarray, list)):
            item = torch.as_tensor(np.asarray(item), device=self.device_tensor.device)
        elif isinstance(item, torch.Tensor):
            item = item.to(self.device_tensor.device)
        return self.device_tensor[item].cpu()

    def __array__(self, dtype=None):
        a = self.numpy()
        return a if dtype is None else a.astype(dtype)


class RingCounter(DeviceCounter):
    """``shared_parameters_counter`` with each round's ``counter[indices] += 1``
    (sharing/PartialModel.py:205-207) applied on read: the encode writes the round's payload
    indices into a slot of a device ring (:meth:`slot`, the payload itself, so nothing extra is
    written), and the ring is folded into the int32 counter (dpz_counter_flush: scattered atomics
    for a few rounds, one coalesced sweep of the counter for many) before any read — the node's
    end-of-run dump (node/DPSGDNode.py:186-194), indexing, ``numpy`` — or when it is full.  The
    encode itself then touches no counter line (its scattered read-modify-writes were 5.7x the
    compact launch's payload traffic at 1 % top-k)."""

    MAX_SEGS = 64  # rounds per ring (the flush passes their offsets as kernel arguments)

    def __init__(self, t, cap_bytes=64 * 2 ** 20):
        self._t = t
        self.n = t.numel()
        self.cap_bytes = int(cap_bytes)
        self.ring = None
        self.segs = [0]
        self._ws = None  # the flush's scratch (allocated with the ring)

    def slot(self, k):
        """int32[k] device view for this round's payload indices (commit with :meth:`commit`)."""
        k = int(k)
        if self.ring is None or self.ring.numel() < k:
            self.flush()
            rounds = max(1, min(self.MAX_SEGS, self.cap_bytes // max(4 * k, 1)))
            self.ring = torch.empty(max(k * rounds, 1), dtype=torch.int32, device=self._t.device)
            if self._ws is None:
                from . import _lib
                self._ws = torch.empty(
                    int(_lib.lib().dpz_counter_flush_workspace_bytes(self.n)), dtype=torch.uint8,
                    device=self._t.device)
        if self.segs[-1] + k > self.ring.numel() or len(self.segs) > self.MAX_SEGS:
            self.flush()
        return self.ring[self.segs[-1]:self.segs[-1] + k]

    def commit(self, k):
        """The slot handed out last holds a final payload (sorted, unique): count it."""
        self.segs.append(self.segs[-1] + int(k))

    def pending_rounds(self):
        return len(self.segs) - 1

    def flush(self):
        if len(self.segs) > 1:
            from . import codec
            codec.counter_flush(self._t, self.ring, self.segs, workspace=self._ws)
            self.segs = [0]
        return self._t

    @property
    def device_tensor(self):
        return self.flush()


class LazyChange:
    """``model.model_change`` (sharing/PartialModel.py:317-331: T(x - init_model), plus the
    accumulated changes with accumulation) formed only when something reads it.  The reference
    sets it every round, but its only readers are ``extract_top_gradients``, which the fused
    encode replaces, and ``save_change`` (:385-390, with ``save_accumulated``); forming it eagerly
    cost one full elementwise pass (12 bytes per element) per round.  ``build`` forms the value from
    tensors the round does not modify in place before ``_post_step`` drops the attribute; a writer
    that would (DeviceAccumulator) materialises it first.  Reads behave like the tensor: torch
    functions, methods and attributes, indexing, operators, ``numpy`` / ``tolist``."""

    def __init__(self, build):
        self._build = build
        self._t = None

    @property
    def materialized(self):
        return self._t is not None

    def materialize(self):
        if self._t is None:
            self._t = self._build()
            self._build = None
        return self._t

    def __getattr__(self, name):
        if name.startswith("__") or name in ("_t", "_build"):
            raise AttributeError(name)
        return getattr(self.materialize(), name)

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        def unwrap(a):
            if isinstance(a, LazyChange):
                return a.materialize()
            if isinstance(a, (list, tuple)):
                return type(a)(unwrap(v) for v in a)
            return a
        return func(*unwrap(tuple(args)), **{k: unwrap(v) for k, v in (kwargs or {}).items()})

    def __getitem__(self, item):
        return self.materialize()[item]

    def __len__(self):
        return len(self.materialize())

    def __array__(self, dtype=None):
        a = self.materialize().cpu().numpy()
        return a if dtype is None else a.astype(dtype)

    __hash__ = object.__hash__


def _lazy_op(name):
    def op(self, *args):
        return getattr(self.materialize(), name)(*args)
    op.__name__ = name
    return op


for _name in ("__add__", "__radd__", "__sub__", "__rsub__", "__mul__", "__rmul__",
              "__truediv__", "__rtruediv__", "__neg__", "__abs__", "__pow__", "__eq__", "__ne__",
              "__lt__", "__le__", "__gt__", "__ge__", "__iter__", "__bool__", "__float__"):
    setattr(LazyChange, _name, _lazy_op(_name))


class SlicedCounter(DeviceCounter):
    """``shared_parameters_counter`` kept as 32 bit planes (dpz_topk_encode_sliced adds the
    selection to them with coalesced word updates); every read materialises the int32 vector
    (dpz_counter_unslice), so the node's end-of-run dump (node/DPSGDNode.py:186-194) and any
    indexing see the reference's counter."""

    def __init__(self, planes, n):
        self.planes = planes
        self.n = int(n)

    @property
    def device_tensor(self):
        from . import codec
        return codec.counter_unslice(self.planes, self.n)

    @property
    def shape(self):
        return torch.Size([self.n])

    def __len__(self):
        return self.n


class DeviceAccumulator:
    """``model.accumulated_changes`` when the encode's rewind is deferred
    (dpz_topk_encode_sliced): ``device_tensor`` is the accumulator as the encode left it and
    ``pending`` the selection mask whose rewind (reference models/Model.py:53-64,
    ``accumulated_changes[indices] = 0``) the post-step applies as it adds the averaging change
    (dpz_dwt_sym2_rewind).  Any read in between (``cpu``, ``numpy``, indexing, ``clone``)
    settles it first — applies the rewind in place — so it always shows the reference's value."""

    def __init__(self, t):
        self.device_tensor = t
        self.pending = None
        self._readers = []  # LazyChange values formed from device_tensor (watch)

    def watch(self, lazy):
        """``lazy`` (a LazyChange) reads device_tensor when it materialises: any in-place write
        through this wrapper forms it first."""
        self._readers.append(lazy)

    def unwatch(self):
        self._readers = []

    def _before_write(self):
        for lz in self._readers:
            lz.materialize()
        self._readers = []

    def settle(self):
        if self.pending is not None:
            from . import codec
            self._before_write()
            codec.rewind_apply(self.device_tensor, self.pending)
            self.pending = None
        return self.device_tensor

    def zero_(self):
        self._before_write()
        self.pending = None
        self.device_tensor.zero_()
        return self

    def cpu(self):
        return self.settle().cpu()

    def numpy(self):
        return self.cpu().numpy()

    def tolist(self):
        return self.numpy().tolist()

    def clone(self):
        return self.settle().clone()

    def view(self, *args):
        return self.settle().view(*args)

    @property
    def shape(self):
        return self.device_tensor.shape

    def numel(self):
        return self.device_tensor.numel()

    def __len__(self):
        return self.device_tensor.numel()

    def __getitem__(self, item):
        return self.settle()[item]

    def __setitem__(self, item, value):
        """Reference-style writes (models/Model.py:53-64 ``accumulated_changes[indices] = 0``):
        settle the pending rewind, then assign on the device tensor (host index arrays and
        values are moved to its device)."""
        t = self.settle()
        self._before_write()
        if isinstance(item, (np.ndarray, list)):
            item = torch.as_tensor(np.asarray(item), device=t.device)
        elif isinstance(item, torch.Tensor):
            item = item.to(t.device)
        if isinstance(value, (np.ndarray, torch.Tensor)):
            value = torch.as_tensor(value).to(t.device)
        t[item] = value

    def __iadd__(self, other):
        """``acc += change`` (PartialModel.py:346-349): settle, then add in place."""
        if isinstance(other, DeviceAccumulator):
            other = other.settle()
        self.settle()
        self._before_write()
        self.device_tensor.add_(torch.as_tensor(other).to(self.device_tensor.device))
        return self

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        """Any torch function handed the wrapper (``torch.zeros_like(acc)``, ``acc + t``,
        ``torch.cat([acc, ...])``) sees the settled device tensor."""
        def unwrap(a):
            if isinstance(a, DeviceAccumulator):
                return a.settle()
            if isinstance(a, (list, tuple)):
                return type(a)(unwrap(v) for v in a)
            return a
        return func(*unwrap(tuple(args)), **{k: unwrap(v) for k, v in (kwargs or {}).items()})

    def __array__(self, dtype=None):
        a = self.numpy()
        return a if dtype is None else a.astype(dtype)


def np_int32(a):
    return np.ascontiguousarray(np.asarray(a), dtype=np.int32)
