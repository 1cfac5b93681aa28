"""Top-k encode of ONE tensor split over ranks ("one tensor, top-k encode: yes,
one small exchange step"; the C5 shape: a 256 MiB model on 8 MI355X).

Rank r holds the contiguous slice [offset_r, offset_r + n_r) of the flat model (and of init_model,
shared_parameters_counter).  The global top-k under the reference's rule (k largest |x - x0|,
ties to the lowest index; sharing/PartialModel.py:164-186) is found with ONE collective:

  1. every rank selects its local top-k (the full k, not k / world) with the HIP encoder — the
     global top-k is contained in the union: a rank contributes at most k entries, and those are
     its k largest with the lowest local (= lowest global) indices among ties;
  2. one all-gather of the k candidates of every rank (global index, change, value: 12 B each,
     10 B with fp16 values; 6.4 / 5.4 MB for C5 on 8 ranks) over RCCL;
  3. every rank runs the same top-k over the world * k gathered changes (their concatenation is
     in global index order, so the encoder's lowest-position tie rule is the lowest global index)
     and gathers the winners' indices and values — identical on every rank, no second exchange;
  4. each rank applies counter[idx] += 1 to the winners inside its own slice.

The result is bit-identical to a one-GPU encode of the whole tensor (tests/test_gpu_shard.py,
tests/test_cpu_shard.py).  Only the all-gather crosses xGMI; no reduce-scatter is needed.
"""
import torch

from . import _lib, codec
from .codec import _ptr, _stream


def _gather_change(x, x0, idx):
    out = torch.empty(idx.numel(), dtype=torch.float32, device=x.device)
    rc = _lib.lib().dpz_gather_change(_ptr(x), _ptr(x0), x.numel(), _ptr(idx), idx.numel(),
                                      _ptr(out), _stream(x.device))
    _lib.check(rc, "dpz_gather_change")
    return out


def _gather_u32(src, pos):
    out = torch.empty(pos.numel(), dtype=src.dtype, device=src.device)
    if src.element_size() == 2:  # fp16 payload values
        rc = _lib.lib().dpz_gather_u16(_ptr(src), src.numel(), _ptr(pos), pos.numel(), _ptr(out),
                                       _stream(src.device))
        _lib.check(rc, "dpz_gather_u16")
        return out
    rc = _lib.lib().dpz_gather_u32(_ptr(src), src.numel(), _ptr(pos), pos.numel(), _ptr(out),
                                   _stream(src.device))
    _lib.check(rc, "dpz_gather_u32")
    return out


def _scatter_add(counter, idx, offset):
    rc = _lib.lib().dpz_scatter_add_i32(_ptr(counter), counter.numel(), _ptr(idx), idx.numel(),
                                        int(offset), 1, _stream(counter.device))
    _lib.check(rc, "dpz_scatter_add_i32")


class HipShardOps:
    """Device implementation of the per-rank steps (the HIP codec).  The encodes are enqueued
    optimistically (no host sync); their sampled-path status words travel with the candidates
    and the caller re-runs the round exactly in the rare case one of them missed."""

    def __init__(self, device):
        self.ws = codec.Workspace(device)
        self.ws_merge = codec.Workspace(device)

    def local_candidates(self, x, x0, k, offset, exact=False, val_fp16=False):
        idx, val = codec.topk_encode(x, k, x0=x0, workspace=self.ws, asynchronous=not exact,
                                     exact=exact, val_fp16=val_fp16)
        chg = _gather_change(x, x0, idx)
        return (idx + int(offset)).to(torch.int32), chg, val

    def local_status(self):
        """This rank's sampled-path status word (device int32[1]; 0 = the result is final)."""
        return self.ws.buf[8:12].view(torch.int32)

    def merge(self, gidx, gchg, gval, k, exact=False):
        # positions of the k winners among the gathered changes, in ascending position order
        pos, _ = codec.topk_encode(gchg, k, workspace=self.ws_merge, asynchronous=not exact,
                                   exact=exact)
        return _gather_u32(gidx, pos), _gather_u32(gval, pos)

    def merge_status(self):
        return self.ws_merge.buf[8:12].view(torch.int32)

    def count(self, counter, idx, offset):
        _scatter_add(counter, idx, offset)

    def replace_slice(self, local_slice, offset, idx, vals, out):
        rc = _lib.lib().dpz_replace_slice(_ptr(local_slice), local_slice.numel(), int(offset),
                                          _ptr(idx), _ptr(vals), idx.numel(), _ptr(out),
                                          _stream(local_slice.device))
        _lib.check(rc, "dpz_replace_slice")


def sharded_topk_encode(x, x0, k, offset, counter=None, group=None, ops=None, val_fp16=False):
    """Global top-k of a tensor sharded over the ranks of `group`.

    x, x0: this rank's slice (flat fp32); offset: the slice's first global index; k: the GLOBAL
    k (every slice must hold at least k elements).  Returns ``(idx int32[k] global ascending,
    val fp32[k])`` — the whole payload, identical on every rank.  ``counter`` (this rank's slice
    of shared_parameters_counter) gets += 1 at the winners inside the slice.  ``val_fp16``: the
    values are packed to fp16 (round to nearest even) by the local encodes themselves
    (DPZ_TOPK_VAL_FP16, BASELINE config 5) and travel as fp16: ``val`` is float16[k].
    """
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    # collectives with more than one rank, or with an explicit group (one rank: RCCL loopback)
    coll = dist.is_initialized() and (world > 1 or group is not None)
    if x.numel() < k:
        raise ValueError("every shard must hold at least k elements")
    ops = ops or HipShardOps(x.device)
    for exact in (False, True):
        if val_fp16:
            idx, chg, val = ops.local_candidates(x, x0, k, offset, exact=exact, val_fp16=True)
        else:
            idx, chg, val = ops.local_candidates(x, x0, k, offset, exact=exact)
        st = (ops.local_status() if hasattr(ops, "local_status")
              else torch.zeros(1, dtype=torch.int32, device=idx.device))
        if coll:
            # one exchange: the candidate arrays and the status word, packed as bytes
            # (index, change: 4 B; value: 4 or 2 B) in ONE all-gather.  The value section is
            # padded to a multiple of 4 bytes so every section of every row starts 4-byte
            # aligned (odd k with fp16 values; the int32 / fp32 views below need it even when
            # a one-rank gather hands back a view without a copy)
            vb = val.element_size()
            vpad = -(-vb * k // 4) * 4
            row = 8 * k + vpad + 4
            parts = [idx.view(torch.uint8), chg.view(torch.uint8), val.view(torch.uint8)]
            if vpad != vb * k:
                parts.append(torch.zeros(vpad - vb * k, dtype=torch.uint8, device=idx.device))
            pack = torch.cat(parts + [st.view(torch.uint8)])
            gflat = torch.empty(world * row, dtype=torch.uint8, device=idx.device)
            dist.all_gather_into_tensor(gflat, pack, group=group)
            gpack = gflat.view(world, row)
            gidx = gpack[:, :4 * k].reshape(-1).contiguous().view(torch.int32)
            gchg = gpack[:, 4 * k:8 * k].reshape(-1).contiguous().view(torch.float32)
            gval = gpack[:, 8 * k:8 * k + vb * k].reshape(-1).contiguous().view(val.dtype)
            gst = gpack[:, row - 4:].reshape(-1).contiguous().view(torch.int32)
        else:
            gidx, gchg, gval, gst = idx, chg, val, st
        widx, wval = ops.merge(gidx, gchg, gval, k, exact=exact)
        mst = (ops.merge_status() if hasattr(ops, "merge_status")
               else torch.zeros(1, dtype=torch.int32, device=idx.device))
        # every rank sees the same gathered statuses and the same merge: the same decision
        if exact or int(gst.abs().sum().item()) + int(mst.abs().sum().item()) == 0:
            break
    if counter is not None:
        ops.count(counter, widx, offset)
    return widx, wval


# ---------------------------------------------------------------------------------------------
# One tensor's sym2 DWT / IDWT over ranks (SURVEY.md §8e "wavelet DWT/IDWT: yes, with a halo").
#
# The model is cut into IDWT tiles of V = 4096 outputs; rank r owns the contiguous tiles
# [u_lo, u_hi) = its model slice [lo, hi).  The forward tiles (W = 128 level-L outputs, 2^L * W
# inputs) of that slice start at t_lo = lo / (2^L W): a rank's forward tiles read only its own
# slice plus a LEFT halo of 2 (2^L - 1) inputs (30 at level 4; 32 kept, see halo_len), the tail
# of rank r - 1's slice,
# exchanged with one small all-gather.  Every rank writes the coefficients its tiles own (one
# range per level) and one all-gather of those owned ranges gives every rank the whole
# [cA_L, cD_L, ..., cD_1] array (what the fold and the IDWT read).  The inverse needs no exchange
# once the coefficients are whole: each rank rebuilds its own slice.  Bit-identical to the
# one-GPU transform (tests/test_gpu_shard.py; the exchange logic: tests/test_cpu_shard.py).

def _level_lengths(n, level):
    lens = [n]
    for _ in range(level):
        lens.append((lens[-1] + 3) // 2)
    return lens


def wavelet_slice(n, level, world, rank, dwt_tile=128, idwt_tile=4096):
    """Rank `rank`'s model slice [lo, hi) and its forward / inverse tile ranges.

    The forward tiles past the last whole span (the model's tail) belong to the rank whose slice
    holds element n - 1; a rank with an empty slice (more ranks than inverse tiles) owns no tile
    of either kind."""
    span = (1 << level) * dwt_tile
    if idwt_tile % span:
        raise ValueError("level too deep for the shared tiling (needs 2^level * dwt_tile | "
                         "idwt_tile)")
    lens = _level_lengths(n, level)
    n_fwd = -(-lens[level] // dwt_tile)
    n_inv = -(-n // idwt_tile)
    per = -(-n_inv // world)
    u_lo, u_hi = min(rank * per, n_inv), min((rank + 1) * per, n_inv)
    lo, hi = min(u_lo * idwt_tile, n), min(u_hi * idwt_tile, n)
    if lo >= hi:  # empty slice
        return dict(lo=lo, hi=lo, t_lo=n_fwd, t_hi=n_fwd, u_lo=u_hi, u_hi=u_hi)
    t_lo = min(lo // span, n_fwd)
    t_hi = n_fwd if hi == n else min(hi // span, n_fwd)
    return dict(lo=lo, hi=hi, t_lo=t_lo, t_hi=t_hi, u_lo=u_lo, u_hi=u_hi)


def owned_coeff_ranges(n, level, t_lo, t_hi, dwt_tile=128):
    """[start, end) ranges of the coefficient array written by forward tiles [t_lo, t_hi) (the
    last tile, t_hi == the tile count, also owns each detail level's tail)."""
    lens = _level_lengths(n, level)
    n_fwd = -(-lens[level] // dwt_tile)
    last = t_hi == n_fwd and t_lo < t_hi
    out = [(min(t_lo * dwt_tile, lens[level]), min(t_hi * dwt_tile, lens[level]))]  # cA_L
    off = lens[level]
    for lv in range(level, 0, -1):
        s = min(t_lo * dwt_tile << (level - lv), lens[lv])
        e = lens[lv] if last else min(t_hi * dwt_tile << (level - lv), lens[lv])
        out.append((off + s, off + max(s, e)))
        off += lens[lv]
    return out


def tile_widths():
    """(forward, inverse) tile widths of the built kernels (dpz_dwt_tile_width /
    dpz_idwt_tile_width): every slice and owned-range computation uses these."""
    L = _lib.lib()
    return int(L.dpz_dwt_tile_width()), int(L.dpz_idwt_tile_width())


def halo_len(level):
    """Left halo a forward slice needs: 2 (2^L - 1) inputs, rounded up to 4 so that the halo'd
    buffer keeps the kernel's float4 groups (which start at a multiple of 4) aligned and inside
    the buffer."""
    return (2 * ((1 << level) - 1) + 3) // 4 * 4


def _virtual(t, first_index):
    """Address of global element 0 for a buffer holding elements from `first_index` on."""
    return t.data_ptr() - int(first_index) * t.element_size()


def dwt_rank_part(xbuf, x0buf, buf_first, n, level, t_lo, t_hi, cx, cd, accumulate=False):
    """Forward tiles [t_lo, t_hi) from a halo'd slice buffer whose element 0 is global element
    `buf_first`; writes the owned coefficients into the full-length cx / cd (may be None)."""
    dev = xbuf.device
    rc = _lib.lib().dpz_dwt_sym2_tiles(
        _virtual(xbuf, buf_first), _virtual(x0buf, buf_first) if x0buf is not None else None,
        n, level, t_lo, t_hi, _ptr(cx) if cx is not None else None,
        _ptr(cd) if cd is not None else None, 1 if accumulate else 0, _stream(dev))
    _lib.check(rc, "dpz_dwt_sym2_tiles")


def _exchange_owned(arrs, n, level, world, rank, group, dist, widths):
    """All-gather every rank's owned coefficient ranges of each array in `arrs` (in place)."""
    dw, iw = widths
    parts = []
    for r in range(world):
        sl = wavelet_slice(n, level, world, r, dw, iw)
        parts.append(owned_coeff_ranges(n, level, sl["t_lo"], sl["t_hi"], dw))
    sizes = [sum(e - s for s, e in p) for p in parts]
    cap = max(1, max(sizes))
    dev = arrs[0].device
    send = torch.zeros(len(arrs) * cap, dtype=torch.float32, device=dev)
    o = 0
    for s, e in parts[rank]:
        for a_i, a in enumerate(arrs):
            send[a_i * cap + o:a_i * cap + o + (e - s)] = a[s:e]
        o += e - s
    recv = torch.empty(world * len(arrs) * cap, dtype=torch.float32, device=dev)
    dist.all_gather_into_tensor(recv, send, group=group)
    recv = recv.view(world, len(arrs), cap)
    for r in range(world):
        if r == rank:
            continue
        o = 0
        for s, e in parts[r]:
            for a_i, a in enumerate(arrs):
                a[s:e] = recv[r, a_i, o:o + (e - s)]
            o += e - s


# the per-rank transforms (dwt_rank_part) are module attributes so the CPU exchange tests can
# replace them with the oracle; those tests also lift the device requirement below
_DEVICE_ONLY = True


def _check_f32(t, name, numel=None, device=None):
    if _DEVICE_ONLY if device is None else device:
        codec._require(t, torch.float32, name)
    elif t.dtype != torch.float32 or not t.is_contiguous():
        raise ValueError(f"{name} must be a contiguous float32 tensor")
    if numel is not None and t.numel() != numel:
        raise ValueError(f"{name} must hold {numel} elements, got {t.numel()}")


def _halo_buffer(t, H):
    """A (buffer, first-offset) pair holding H elements before `t`'s first element and then `t`:
    `t` itself viewed with its headroom when it came from alloc_wavelet_slice (no copy; only
    that buffer's reserved headroom is ever written), otherwise a fresh copy."""
    so = t.storage_offset()
    if getattr(t, "_dpz_halo", 0) >= H and so >= H:
        buf = torch.empty(0, dtype=t.dtype, device=t.device)
        buf.set_(t.untyped_storage(), so - H, (H + t.numel(),), (1,))
        return buf, False
    return torch.cat([torch.empty(H, dtype=t.dtype, device=t.device), t]), True


def alloc_wavelet_slice(n, level, world, rank, device):
    """This rank's x (or x0) slice buffer for sharded_wavedec: a view of a buffer with room for
    the left halo in front, so the halo exchange writes halo_len(level) elements, not a copy of
    the whole slice."""
    dw, iw = tile_widths()
    sl = wavelet_slice(n, level, world, rank, dw, iw)
    H = halo_len(level)
    base = torch.empty(H + sl["hi"] - sl["lo"], dtype=torch.float32, device=device)
    view = base[H:]
    view._dpz_halo = H  # the H elements in front are this buffer's own, free for the halo
    return view


def sharded_wavedec(x_slice, x0_slice, n, level, group=None, accumulate_into=None):
    """W(x) and W(x - x0) of a tensor sharded over the ranks of `group` (rank r holds its
    wavelet_slice [lo, hi) of x and x0).  Returns the whole coefficient arrays on every rank
    (W(x), W(x - x0) — or, with ``accumulate_into``, that array += W(x - x0) and W(x)).
    Slices from alloc_wavelet_slice get their halo written in place (no slice copy)."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    widths = tile_widths()
    sl = wavelet_slice(n, level, world, rank, *widths)
    # every check happens before the first collective, so every rank fails the same way
    m_len = codec.wavedec_len(n, level)
    _check_f32(x_slice, "x_slice", sl["hi"] - sl["lo"])
    _check_f32(x0_slice, "x0_slice", sl["hi"] - sl["lo"])
    if accumulate_into is not None:
        _check_f32(accumulate_into, "accumulate_into", m_len)
    H = halo_len(level)
    for r in range(world):
        s = wavelet_slice(n, level, world, r, *widths)
        if 0 < s["hi"] - s["lo"] < H:
            raise ValueError("tensor too small for this many ranks (a slice is shorter than the "
                             "halo)")
    dev = x_slice.device
    xb, x0b, first = x_slice, x0_slice, sl["lo"]
    coll = dist.is_initialized() and (world > 1 or group is not None)  # as sharded_topk_encode
    if coll:
        # the left halo: the last H elements of the previous non-empty slice (x and x0), one
        # all-gather; an empty slice sends nothing useful and receives nothing
        tail = torch.zeros(2 * H, dtype=torch.float32, device=dev)
        m = min(H, x_slice.numel())
        if m:
            tail[H - m:H] = x_slice[x_slice.numel() - m:]
            tail[2 * H - m:] = x0_slice[x0_slice.numel() - m:]
        tails = torch.empty(world * 2 * H, dtype=torch.float32, device=dev)
        dist.all_gather_into_tensor(tails, tail, group=group)
        if rank > 0 and sl["lo"] < sl["hi"]:
            prev = tails.view(world, 2 * H)[rank - 1]
            xb, _ = _halo_buffer(x_slice, H)
            x0b, _ = _halo_buffer(x0_slice, H)
            xb[:H] = prev[:H]
            x0b[:H] = prev[H:]
            first = sl["lo"] - H
    cx = torch.zeros(m_len, dtype=torch.float32, device=dev)
    cd = accumulate_into if accumulate_into is not None else torch.zeros_like(cx)
    if sl["t_lo"] < sl["t_hi"]:
        dwt_rank_part(xb, x0b, first, n, level, sl["t_lo"], sl["t_hi"], cx, cd,
                      accumulate=accumulate_into is not None)
    if coll:
        _exchange_owned([cx, cd], n, level, world, rank, group, dist, widths)
    return cx, cd


def idwt_rank_part(coeffs, n, level, u_lo, u_hi, out_slice, lo):
    """Inverse tiles [u_lo, u_hi) of the whole coefficient array into out_slice (global [lo, ..))."""
    rc = _lib.lib().dpz_idwt_sym2_tiles(_ptr(coeffs), n, level, u_lo, u_hi,
                                        _virtual(out_slice, lo), _stream(coeffs.device))
    _lib.check(rc, "dpz_idwt_sym2_tiles")


def sharded_waverec(coeffs, n, level, group=None):
    """This rank's slice [lo, hi) of the inverse transform of the whole coefficient array."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    _check_f32(coeffs, "coeffs", codec.wavedec_len(n, level))
    sl = wavelet_slice(n, level, world, rank, *tile_widths())
    out = torch.empty(sl["hi"] - sl["lo"], dtype=torch.float32, device=coeffs.device)
    if out.numel():
        idwt_rank_part(coeffs, n, level, sl["u_lo"], sl["u_hi"], out, sl["lo"])
    return out


# ---------------------------------------------------------------------------------------------
# One tensor's decode over ranks (SURVEY.md §8e "one tensor, decode: yes, no collective"): the
# payload's indices are global and sorted; each rank replaces the entries that fall inside its
# slice [offset, offset + n) and skips the rest, in one launch (dpz_replace_slice).

def sharded_replace(local_slice, offset, idx, vals, out=None, ops=None):
    """``T = local.clone(); T[idx] = vals`` (reference PartialModel.py:292-295) restricted to this
    rank's slice: local_slice holds global elements [offset, offset + len); idx / vals is the
    WHOLE payload (global ascending indices, e.g. from sharded_topk_encode).  No collective."""
    ops = ops or HipShardOps(local_slice.device)
    hip = isinstance(ops, HipShardOps)  # the device kernel needs device tensors
    _check_f32(local_slice, "local_slice", device=hip)
    if hip:
        codec._require(idx, torch.int32, "idx")
    if idx.dtype != torch.int32 or idx.dim() != 1:
        raise ValueError("idx must be a 1-D int32 tensor")
    _check_f32(vals, "vals", idx.numel(), device=hip)
    if out is None:
        out = torch.empty_like(local_slice)
    _check_f32(out, "out", local_slice.numel(), device=hip)
    if int(offset) < 0:
        raise ValueError("offset must be >= 0")
    ops.replace_slice(local_slice, int(offset), idx, vals, out)
    return out
