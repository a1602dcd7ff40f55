"""Row-band sharding of one image pair across GPUs.

Output row h of the cost volume reads only image rows h-o .. h+a (o = k//2,
a = k-1-o; o = a = r for odd k; custma/src/stereo_matching_kernel.cu:44,60),
so the path shards by row band with no data-path collective: rank g owns rows
[b_g, e_g) of both images and of the volume, and needs o halo rows from the
rank above and a from the rank below.

* forward: one neighbour exchange of r x W pixels per image per side
  (``torch.distributed.batch_isend_irecv`` -- RCCL point-to-point over xGMI
  with the ``nccl`` backend), then the band kernel computes exactly the
  owned volume rows (custma_forward_band).  The volume stays sharded.
* backward: the band kernel returns image gradients for the owned rows
  AND the halo rows (partial sums of patches centred in this band); one
  exchange sends each halo partial to the neighbour that owns those rows,
  which adds it (a halo reduce of r x W floats per side).
* disparity: local per band, no communication beyond the halo.

The whole exchange is latency-bound (r*W*4 bytes, e.g. 5 x 8192 x 4 B =
160 KB at k = 11); ring collectives are not needed and not used.

A ``backend`` object computes the band ops; the default is the HIP library.
Tests on CPU (gloo) inject the oracle as the backend; the product never does.
"""
from __future__ import annotations

import os
import weakref
from typing import Optional, Tuple

import torch
import torch.distributed as dist


def band_bounds(H: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced split of H rows over `world` ranks."""
    base, extra = divmod(H, world)
    b = rank * base + min(rank, extra)
    return b, b + base + (1 if rank < extra else 0)


class HipBackend:
    """Band ops on the HIP library (custma_*_band)."""

    supports_out = True  # forward() writes into a preallocated slice of the band's volume

    def forward(self, cam, proj, D, k, layout, precision, rows, out=None):
        from .stereo_matching_wrapper import cost_volume_forward

        return cost_volume_forward(cam, proj, D, k, layout, precision, rows=rows, out=out)

    def backward(self, grad, cam, proj, D, k, layout, rows, want_cam, want_proj, vol=None):
        from .stereo_matching_wrapper import cost_volume_backward

        return cost_volume_backward(grad, cam, proj, k, layout, D, camera_grad=want_cam,
                                    projector_grad=want_proj, rows=rows, cost_volume=vol)

    def disparity(self, cam, proj, D, k, layout, rows):
        from .disparity import stereo_disparity

        return stereo_disparity(cam, proj, D, k, layout, rows=rows)


# ---- optional timing of the exchanges (bench.py at N > 1): CUDA events on the op's stream ----
_TIMING = {"on": False, "events": []}


def enable_timing(on: bool = True) -> None:
    """Record, per exchange, the time the op's stream waited for it (device tensors only):
    ``fwd_exposed`` = from the post of the exchange (CUSTMA_ROWBAND_OVERLAP=1: from the end of the
    interior-row forward launch) to the halo's arrival, ``bwd`` = the whole halo reduce."""
    _TIMING["on"] = on
    _TIMING["events"] = []


def timing_summary() -> dict:
    """Mean milliseconds per exchange kind recorded since enable_timing()."""
    torch.cuda.synchronize()
    acc = {}
    for kind, a, b in _TIMING["events"]:
        acc.setdefault(kind, []).append(a.elapsed_time(b))
    return {f"{k}_ms": round(sum(v) / len(v), 4) for k, v in acc.items()} | {
        f"{k}_n": len(v) for k, v in acc.items()}


def _event(t: torch.Tensor):
    if not (_TIMING["on"] and t.is_cuda):
        return None
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


def _record(kind, a, t: torch.Tensor):
    if a is not None:
        _TIMING["events"].append((kind, a, _event(t)))


class _Pending:
    """An exchange in flight: ``wait()`` makes the current stream wait for the received halo
    (nccl), or blocks for the gloo requests and copies the staged host buffers to the device."""

    def __init__(self, works, staged):
        self.works, self.staged = works, staged

    def wait(self):
        for w in self.works:
            w.wait()
        for dst, src in self.staged:
            dst.copy_(src)
        self.works, self.staged = [], []


class RowBandGroup:
    """Rank/world/halo bookkeeping plus the two halo primitives.

    The halo must come from the immediate neighbour, so every band needs at
    least max(o, a) rows.  That is checked for ALL ranks, collectively, before
    any point-to-point call: one MIN all-reduce of (band height, -mismatch),
    where mismatch says that this rank's height differs from
    ``band_bounds(H, world, rank)`` when the global ``H`` is given.  So a band
    that is too thin, or a split that is not ``band_bounds``'s, raises on
    EVERY rank instead of leaving the others waiting in ``batch_isend_irecv``.
    With ``H`` alone (no ``n``) the bands are ``band_bounds``'s by definition
    and nothing is communicated.  A group can be built once and reused for
    every op on the same bands (``rbg=``); the per-call check then compares
    the band height with the one the collective check saw."""

    def __init__(self, kernel_size: int, group=None, n: Optional[int] = None, H: Optional[int] = None,
                 device=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.k = kernel_size
        self.o = kernel_size // 2
        self.a = kernel_size - 1 - self.o
        self.n = None if n is None else int(n)
        need = max(self.o, self.a)
        if self.world > 1 and need > 0:
            if self.n is not None:
                mismatch = 0
                if H is not None:
                    b0, e0 = band_bounds(H, self.world, self.rank)
                    mismatch = int(self.n != e0 - b0)
                dev = device if dist.get_backend(group) == "nccl" else "cpu"
                t = torch.tensor([self.n, -mismatch], dtype=torch.int64, device=dev)
                dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
                thinnest, bad = int(t[0].item()), int(t[1].item()) < 0
                if bad:
                    raise ValueError(f"some rank's band height differs from band_bounds({H}, {self.world}, rank) "
                                     f"(this rank holds {self.n} rows): pass H=None for a custom row split")
            elif H is not None:
                thinnest = min(e - b for b, e in (band_bounds(H, self.world, q) for q in range(self.world)))
            else:
                thinnest = None
            if thinnest is not None and thinnest < need:
                raise ValueError(f"the thinnest row band has {thinnest} rows, fewer than the {need} halo rows "
                                 f"kernel_size {kernel_size} needs from a neighbour")

    def _peer(self, rank):
        return dist.get_global_rank(self.group, rank) if self.group is not None else rank

    def _p2p_start(self, sends, recvs) -> _Pending:
        """Post one batch_isend_irecv of (tensor, group rank) pairs.  Device tensors on a gloo
        group (CPU-only transport, e.g. a single-GPU rehearsal) are staged through host
        memory; with nccl (RCCL over xGMI) they go device to device on RCCL's stream."""
        stage = dist.get_backend(self.group) == "gloo" and any(t.is_cuda for t, _ in sends + recvs)
        hs = [(t.cpu() if stage else t, q) for t, q in sends]
        hr = [(torch.empty(t.shape, dtype=t.dtype) if stage else t, q) for t, q in recvs]
        # zero-row parts (k = 2: no rows below the patch centre) are not sent at all
        ops = [dist.P2POp(dist.isend, t.contiguous(), self._peer(q), self.group) for t, q in hs if t.numel()]
        ops += [dist.P2POp(dist.irecv, t, self._peer(q), self.group) for t, q in hr if t.numel()]
        works = dist.batch_isend_irecv(ops) if ops else []
        staged = [(dst, src) for (dst, _), (src, _) in zip(recvs, hr)] if stage else []
        return _Pending(works, staged)

    def _p2p(self, sends, recvs):
        self._p2p_start(sends, recvs).wait()

    def halo_sizes(self) -> Tuple[int, int]:
        """Rows received from the rank above (o) and from the rank below (a)."""
        top = self.o if self.rank > 0 else 0
        bot = self.a if self.rank < self.world - 1 else 0
        return top, bot

    def exchange_halo_start(self, band: torch.Tensor) -> Tuple[torch.Tensor, Optional[_Pending]]:
        """[n, W] owned rows -> ([top + n + bot, W] buffer with the owned rows in place, the
        exchange filling the halo rows, still in flight)."""
        top, bot = self.halo_sizes()
        if self.world == 1 or self.o + self.a == 0:
            return band, None
        n = band.shape[0]
        if n < max(self.o, self.a):
            raise ValueError(f"row band of {n} rows is thinner than the halo ({self.o} / {self.a} rows)")
        out = torch.empty((top + n + bot,) + tuple(band.shape[1:]), dtype=band.dtype, device=band.device)
        out[top:top + n].copy_(band)
        sends, recvs = [], []
        # the rank above needs my first a rows (its bottom halo); the rank below my last o rows
        if self.rank > 0:
            sends.append((band[:self.a], self.rank - 1))
            recvs.append((out[:top], self.rank - 1))
        if self.rank < self.world - 1:
            sends.append((band[n - self.o:], self.rank + 1))
            recvs.append((out[top + n:], self.rank + 1))
        return out, self._p2p_start(sends, recvs)

    def exchange_halo(self, band: torch.Tensor) -> torch.Tensor:
        """[n, W] owned rows -> [top + n + bot, W] with the neighbours' edge rows."""
        out, pend = self.exchange_halo_start(band)
        if pend is not None:
            pend.wait()
        return out

    def interior(self, n: int) -> Tuple[int, int]:
        """Owned volume rows [i0, i1) whose patches lie inside the owned image rows: they can be
        computed while the halo is in flight (rank 0 / the last rank have image edges, not halos)."""
        top, bot = self.halo_sizes()
        i0 = self.o if top else 0
        i1 = n - self.a if bot else n
        return (i0, i1) if i0 < i1 else (0, 0)

    def reduce_halo(self, buf: torch.Tensor, n: int) -> torch.Tensor:
        """[top + n + bot, W] partial gradients -> [n, W] owned rows with the
        neighbours' halo partials added (each neighbour sends the partials of
        rows this rank owns)."""
        top, bot = self.halo_sizes()
        own = buf[top:top + n]
        if self.world == 1 or self.o + self.a == 0:
            return own.contiguous()
        own = own.clone()
        sends, recvs = [], []
        # partials of my first a rows come from the rank above, of my last o rows from the rank below
        from_up = torch.empty((self.a,) + tuple(buf.shape[1:]), dtype=buf.dtype, device=buf.device)
        from_dn = torch.empty((self.o,) + tuple(buf.shape[1:]), dtype=buf.dtype, device=buf.device)
        if self.rank > 0:
            sends.append((buf[:top], self.rank - 1))
            recvs.append((from_up, self.rank - 1))
        if self.rank < self.world - 1:
            sends.append((buf[top + n:], self.rank + 1))
            recvs.append((from_dn, self.rank + 1))
        e0 = _event(buf)
        self._p2p(sends, recvs)
        _record("bwd_exchange", e0, buf)
        if self.rank > 0 and self.a:
            own[:self.a] += from_up
        if self.rank < self.world - 1 and self.o:
            own[n - self.o:] += from_dn
        return own


def _forward_band(backend, ch, ph, D, k, layout, precision, lo, hi, vol, top):
    """Volume rows [lo, hi) of the band (owned-row indices) into vol[lo:hi]."""
    if hi <= lo:
        return
    dst = vol[lo:hi]
    if getattr(backend, "supports_out", False):
        backend.forward(ch, ph, D, k, layout, precision, (top + lo, top + hi), out=dst)
    else:
        dst.copy_(backend.forward(ch, ph, D, k, layout, precision, (top + lo, top + hi)))


# The forward of a band with halos: by default the halos land first and the band is ONE forward (one
# statistics pass, one sweep launch).  CUSTMA_ROWBAND_OVERLAP=1 computes the interior rows while the
# halos are in flight and the two edges afterwards -- three statistics passes and three sweeps per rank,
# the edge sweeps shorter than their k - 1 warm-up rows; at C5 / 8 ranks the exchange is ~330 KB, a few
# microseconds over xGMI, less than the two extra launch pairs.
def _overlap_interior() -> bool:
    return os.environ.get("CUSTMA_ROWBAND_OVERLAP", "0") == "1"


class _RowBandStereoMatching(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cam_band, proj_band, D, kernel_size, layout, precision, rbg, backend):
        # Post both images' halo exchanges; then either wait for them and run one band forward, or
        # (CUSTMA_ROWBAND_OVERLAP=1) compute the interior volume rows (patches inside the owned rows) while they
        # are in flight and the edge rows once the halos have landed.
        ch, pc = rbg.exchange_halo_start(cam_band.contiguous())
        ph, pp = rbg.exchange_halo_start(proj_band.contiguous())
        top, _ = rbg.halo_sizes()
        n = cam_band.shape[0]
        if pc is None:
            vol = backend.forward(ch, ph, D, kernel_size, layout, precision, (top, top + n))
        elif not _overlap_interior():
            e0 = _event(cam_band)
            pc.wait()
            pp.wait()
            _record("fwd_exposed", e0, cam_band)
            vol = backend.forward(ch, ph, D, kernel_size, layout, precision, (top, top + n))
        else:
            W = ch.shape[1]
            dims = (W, W) if layout == "full" else (W - int(D), int(D) + 1)  # [H, W, W] / [H, W-D, D+1]
            vol = torch.empty((n,) + dims, dtype=torch.float32, device=ch.device)
            i0, i1 = rbg.interior(n)
            _forward_band(backend, ch, ph, D, kernel_size, layout, precision, i0, i1, vol, top)
            e0 = _event(vol)
            pc.wait()
            pp.wait()
            _record("fwd_exposed", e0, vol)
            if i1 > i0:
                _forward_band(backend, ch, ph, D, kernel_size, layout, precision, 0, i0, vol, top)
                _forward_band(backend, ch, ph, D, kernel_size, layout, precision, i1, n, vol, top)
            else:
                _forward_band(backend, ch, ph, D, kernel_size, layout, precision, 0, n, vol, top)
        # the haloed images are saved; the returned volume only weakly (see _StereoMatching)
        ctx.save_for_backward(ch, ph)
        ctx.vol_ref = weakref.ref(vol)
        ctx.vol_version = vol._version
        ctx.meta = (D, kernel_size, layout, precision, rbg, backend, top, n)
        return vol

    @staticmethod
    def backward(ctx, grad):
        ch, ph = ctx.saved_tensors
        vol = ctx.vol_ref()
        vol = vol.detach() if vol is not None and vol._version == ctx.vol_version else None
        D, k, layout, precision, rbg, backend, top, n = ctx.meta
        if vol is None:  # dropped or edited in place: recompute with the forward's own arithmetic
            vol = backend.forward(ch, ph, D, k, layout, precision, (top, top + n))
        want_c, want_p = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        gc, gp = backend.backward(grad.contiguous(), ch, ph, D, k, layout, (top, top + n), want_c, want_p, vol)
        gc = rbg.reduce_halo(gc, n) if gc is not None else None
        gp = rbg.reduce_halo(gp, n) if gp is not None else None
        return gc, gp, None, None, None, None, None, None


# Groups built for a given global H, reused by later calls with the same (group, k, band height, H,
# device): the collective band check then runs once per such key instead of once per call (its MIN
# all-reduce and host sync would sit in front of every op's halo exchange).  Only with H given: every
# rank's key then changes together (H is global and band_bounds fixes each rank's height), so all
# ranks run the check on the same calls.  A custom split (H=None) checks on every call, or takes rbg=.
_GROUPS: dict = {}


def _group_for(rbg, kernel_size, group, n, H, device):
    if rbg is None:
        if H is None:
            return RowBandGroup(kernel_size, group, n=n, H=H, device=device)
        # keyed on the resolved group object and this rank's place in it: after destroy_process_group()
        # and a re-init, WORLD is a new object (and rank / size may differ), so a RowBandGroup built for
        # the old group is never reused
        pg = dist.group.WORLD if group is None else group
        key = (id(pg), dist.get_rank(pg), dist.get_world_size(pg), kernel_size, int(n), int(H), str(device))
        hit = _GROUPS.get(key)
        if hit is None or hit.pg is not pg:
            hit = RowBandGroup(kernel_size, group, n=n, H=H, device=device)
            hit.pg = pg
            if len(_GROUPS) >= 64:
                _GROUPS.clear()
            _GROUPS[key] = hit
        return hit
    if rbg.k != kernel_size or (rbg.n is not None and rbg.n != n):
        raise ValueError(f"rbg was built for kernel_size {rbg.k} and {rbg.n} rows, called with {kernel_size} / {n}")
    return rbg


def stereo_matching_rowband(cam_band: torch.Tensor, proj_band: torch.Tensor, D: int, kernel_size: int,
                            layout: str = "full", precision: Optional[str] = None, group=None,
                            backend=None, H: Optional[int] = None, rbg: Optional[RowBandGroup] = None
                            ) -> torch.Tensor:
    """Distributed ``stereo_matching``: every rank passes its own row band of
    both images (rows ``band_bounds(H, world, rank)``) and gets the matching
    rows of the cost volume; ``backward`` yields gradients of its own rows.
    ``H`` (the global height) also checks that the bands are ``band_bounds``'s.
    ``rbg``: a RowBandGroup built once for these bands (skips the per-call check's
    all-reduce; every rank must pass the same kind of argument)."""
    rbg = _group_for(rbg, kernel_size, group, cam_band.shape[0], H, cam_band.device)
    return _RowBandStereoMatching.apply(cam_band, proj_band, D, kernel_size, layout, precision, rbg,
                                        backend or HipBackend())


def stereo_disparity_rowband(cam_band, proj_band, D, kernel_size, layout="full", group=None, backend=None,
                             H: Optional[int] = None, rbg: Optional[RowBandGroup] = None):
    """Distributed fused disparity for the owned rows (halo exchange only)."""
    rbg = _group_for(rbg, kernel_size, group, cam_band.shape[0], H, cam_band.device)
    ch = rbg.exchange_halo(cam_band.contiguous())
    ph = rbg.exchange_halo(proj_band.contiguous())
    top, _ = rbg.halo_sizes()
    n = cam_band.shape[0]
    return (backend or HipBackend()).disparity(ch, ph, D, kernel_size, layout, (top, top + n))
