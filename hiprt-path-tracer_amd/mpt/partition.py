"""Framebuffer row partition across GPUs.

Rank ``k`` of ``n`` owns the interleaved bands ``y // band_height ≡ k (mod n)``; its
framebuffer holds those rows in increasing y ("band-major compact layout", the layout
of ``mpt_get_framebuffer``).  Every pixel's RNG stream depends only on (pixel index,
sample number, seed), so any partition renders the same pixels bit-identically.
"""
from __future__ import annotations

import numpy as np


def rows_of(res_y: int, band_height: int, band_index: int, band_count: int) -> np.ndarray:
    y = np.arange(res_y)
    return y[(y // band_height) % band_count == band_index]


def max_rows(res_y: int, band_height: int, band_count: int) -> int:
    return max(len(rows_of(res_y, band_height, k, band_count)) for k in range(band_count))


def assemble(parts, res_y: int, band_height: int):
    """parts[k]: rank k's compact rows (rows_k[, padding], W, C) -> full (res_y, W, C).
    Works on numpy arrays and torch tensors (the gathered padded buffers)."""
    n = len(parts)
    first = parts[0]
    if hasattr(first, "new_zeros"):          # torch
        out = first.new_zeros((res_y,) + tuple(first.shape[1:]))
        import torch
        for k, p in enumerate(parts):
            ys = rows_of(res_y, band_height, k, n)
            out[torch.as_tensor(ys, device=p.device)] = p[: len(ys)]
        return out
    out = np.zeros((res_y,) + first.shape[1:], first.dtype)
    for k, p in enumerate(parts):
        ys = rows_of(res_y, band_height, k, n)
        out[ys] = p[: len(ys)]
    return out


def gather_frame(local, res_y: int, band_height: int, dist, group=None):
    """Collective gather of every rank's compact rows (torch tensor [rows, W, C]) and
    re-interleave into the full frame on every rank.  With the nccl backend this is one
    RCCL all-gather over xGMI of the padded row buffers; with gloo (CPU tests) the same
    code path runs on host tensors."""
    world = dist.get_world_size(group)
    mr = max_rows(res_y, band_height, world)
    padded = local.new_zeros((mr,) + tuple(local.shape[1:]))
    padded[: local.shape[0]] = local
    parts = [local.new_empty(padded.shape) for _ in range(world)]
    dist.all_gather(parts, padded, group=group)
    return assemble(parts, res_y, band_height)


# ---- ReSTIR DI across a row partition: contiguous bands + halo exchange --------------
# The reuse passes read neighbours' G-buffer entries and reservoirs, so a
# ReSTIR context renders ONE contiguous band of rows and the library asks the host, through
# the mpt_set_halo_exchange callback, to fill the rows around the band from their owners
# after the G-buffer pass and before every reuse pass (include/mpt.h MptHaloExchange).

def contiguous_band(res_y: int, band_count: int, band_index: int):
    """(band_height, band_index, band_count) of band_index's contiguous band: rank k owns rows
    [k * band_height, min(res_y, (k + 1) * band_height)) -- the MptFrame band fields."""
    bh = -(-res_y // band_count)
    return bh, band_index, band_count


def band_range(res_y: int, band_height: int, k: int):
    y0 = min(res_y, k * band_height)
    return y0, min(res_y, y0 + band_height)


def _overlap(a0, a1, b0, b1):
    lo, hi = max(a0, b0), min(a1, b1)
    return (lo, hi) if lo < hi else None


def halo_plan(res_y: int, band_height: int, band_count: int, rank: int, halo_rows: int):
    """Row ranges a rank exchanges: (sends, recvs), lists of (peer, y0, y1) sorted by
    (peer, y0).  recvs: the rows of [y0 - halo, y0) and [y1, y1 + halo) (clipped) owned by
    peer; sends: the rows of this rank's band inside a peer's halo.  Both sides derive
    the same ranges in the same order, so point-to-point operations pair up."""
    def need(k):
        a, b = band_range(res_y, band_height, k)
        if a >= b:
            return []
        return [(max(0, a - halo_rows), a), (b, min(res_y, b + halo_rows))]

    my0, my1 = band_range(res_y, band_height, rank)
    sends, recvs = [], []
    for p in range(band_count):
        if p == rank:
            continue
        p0, p1 = band_range(res_y, band_height, p)
        for (n0, n1) in need(rank):
            o = _overlap(n0, n1, p0, p1)
            if o:
                recvs.append((p, o[0], o[1]))
        for (n0, n1) in need(p):
            o = _overlap(n0, n1, my0, my1)
            if o:
                sends.append((p, o[0], o[1]))
    return sorted(sends), sorted(recvs)


HALO_GBUFFER = 0      # include/mpt.h MPT_HALO_GBUFFER: the phase that agrees on the halo


class _DevBytes:
    """A device allocation of the library exposed through __cuda_array_interface__ so torch
    can alias it (no copy)."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False), "version": 3}


def _row_views(x, torch, device):
    """The halo buffers of an abi.HaloExchange as uint8 tensors [res_y, res_x * bpp]."""
    out = []
    for i in range(x.n_buffers):
        row = x.res_x * x.bytes_per_pixel[i]
        t = torch.as_tensor(_DevBytes(x.buffers[i], x.res_y * row), device=device)
        out.append(t.view(x.res_y, row))
    return out


class TorchHaloExchange:
    """Halo exchange over torch.distributed, one process per GPU.  With the nccl backend
    (RCCL over xGMI) the point-to-point sends/receives are enqueued on the library's own
    stream (no host synchronisation); with gloo (CPU transport: tests, or hosts without
    RCCL) the rows are staged through host memory."""

    def __init__(self, dist, band_height: int, group=None, device=None):
        import torch
        self.torch = torch
        self.dist = dist
        self.group = group
        self.band_height = band_height
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if device is None and torch.cuda.is_available():
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self.nccl = dist.get_backend(group) == "nccl"
        self.bytes_moved = 0
        self.calls = 0

    def _peer(self, p):
        return p if self.group is None else self.dist.get_global_rank(self.group, p)

    def agree(self, halo_rows: int) -> int:
        """The halo every rank uses this frame: the maximum of what the ranks need."""
        torch, dist = self.torch, self.dist
        dev = self.device if self.nccl else "cpu"
        t = torch.tensor([int(halo_rows)], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return int(t.item())

    def __call__(self, x):
        torch = self.torch
        if x.phase == HALO_GBUFFER and not x.halo_agreed:   # (agreed: a still camera, same halo everywhere)
            x.halo_rows = self.agree(x.halo_rows)
        stream = torch.cuda.ExternalStream(x.stream, device=self.device) if x.stream else torch.cuda.current_stream(self.device)
        self.exchange_views(_row_views(x, torch, self.device), x.res_y, x.halo_rows, stream)

    def exchange_views(self, views, res_y: int, halo_rows: int, stream=None):
        """Fills rows of every view ([res_y, row_bytes] tensors) around this rank's band from
        their owners.  CUDA views + nccl: enqueued on `stream`; otherwise staged through
        host memory (CPU views need no staging: the gloo path of the CPU tests)."""
        torch, dist = self.torch, self.dist
        sends, recvs = halo_plan(res_y, self.band_height, self.world, self.rank, halo_rows)
        self.calls += 1
        on_dev = bool(views) and views[0].is_cuda
        if self.nccl and on_dev:
            with torch.cuda.stream(stream):
                ops = []
                for v in views:
                    for (p, a, b) in sends:
                        ops.append(dist.P2POp(dist.isend, v[a:b], self._peer(p), self.group))
                    for (p, a, b) in recvs:
                        ops.append(dist.P2POp(dist.irecv, v[a:b], self._peer(p), self.group))
                if ops:
                    for w in dist.batch_isend_irecv(ops):
                        w.wait()       # the library's stream waits; the host does not
        else:
            if on_dev:
                stream.synchronize()
            ops, staged = [], []
            for v in views:
                for (p, a, b) in sends:
                    ops.append(dist.P2POp(dist.isend, v[a:b].cpu().contiguous(), self._peer(p), self.group))
                for (p, a, b) in recvs:
                    buf = torch.empty((b - a, v.shape[1]), dtype=v.dtype)
                    staged.append((v, a, b, buf))
                    ops.append(dist.P2POp(dist.irecv, buf, self._peer(p), self.group))
            if ops:
                for w in dist.batch_isend_irecv(ops):
                    w.wait()
            if on_dev:
                with torch.cuda.stream(stream):
                    for (v, a, b, buf) in staged:
                        v[a:b].copy_(buf)
                stream.synchronize()
            else:
                for (v, a, b, buf) in staged:
                    v[a:b].copy_(buf)
        self.bytes_moved += sum(v.shape[1] * v.element_size() * (b - a) for v in views for (_, a, b) in recvs)


class LocalHaloGroup:
    """Halo exchange between the contexts of ONE process (one host thread per context, e.g.
    one process driving several GPUs, or several bands on one GPU).  Each context's callback
    publishes its buffers, waits for the others, copies its halo rows from the owners'
    buffers (device-to-device, peer copies across GPUs) and waits again so that no owner
    overwrites rows still being read."""

    def __init__(self, band_height: int, band_count: int, devices=None):
        import threading
        import torch
        self.torch = torch
        self.band_height = band_height
        self.band_count = band_count
        self.devices = devices or [torch.device("cuda", 0)] * band_count
        self.barrier = threading.Barrier(band_count, timeout=120)   # a failed member breaks it
        self.published = [None] * band_count
        self.need = [0] * band_count

    def member(self, rank: int):
        def exchange(x):
            try:
                _exchange(x)
            except BaseException:
                self.barrier.abort()     # no other member waits for this one's rows
                raise

        def _exchange(x):
            torch = self.torch
            dev = self.devices[rank]
            views = _row_views(x, torch, dev)
            stream = torch.cuda.ExternalStream(x.stream, device=dev)
            stream.synchronize()             # this band's rows are final
            self.published[rank] = views
            self.need[rank] = x.halo_rows
            self.barrier.wait()
            if x.phase == HALO_GBUFFER:
                x.halo_rows = max(self.need)
            _, recvs = halo_plan(x.res_y, self.band_height, self.band_count, rank, x.halo_rows)
            with torch.cuda.stream(stream):
                for i, v in enumerate(views):
                    for (p, a, b) in recvs:
                        v[a:b].copy_(self.published[p][i][a:b])
            stream.synchronize()
            self.barrier.wait()
        return exchange
