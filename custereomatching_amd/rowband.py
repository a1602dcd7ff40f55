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

    def forward(self, cam, proj, D, k, layout, precision, rows):
        from .stereo_matching_wrapper import cost_volume_forward

        return cost_volume_forward(cam, proj, D, k, layout, precision, rows=rows)

    def backward(self, grad, cam, proj, D, k, layout, rows, want_cam, want_proj, vol=None):
        from .stereo_matching_wrapper import cost_volume_backward

        return cost_volume_backward(grad, cam, proj, k, layout, D, camera_grad=want_cam,
                                    projector_grad=want_proj, rows=rows, cost_volume=vol)

    def disparity(self, cam, proj, D, k, layout, rows):
        from .disparity import stereo_disparity

        return stereo_disparity(cam, proj, D, k, layout, rows=rows)


class RowBandGroup:
    """Rank/world/halo bookkeeping plus the two halo primitives.

    The halo must come from the immediate neighbour, so every band needs at
    least max(o, a) rows.  That is checked for ALL ranks before any
    point-to-point call, so every rank raises together instead of the thin
    ranks raising while their neighbours wait in ``batch_isend_irecv``: from
    ``H`` (the global height, bands = ``band_bounds``) without communication,
    or else with one MIN all-reduce of the band heights."""

    def __init__(self, kernel_size: int, group=None, n: Optional[int] = None, H: Optional[int] = None,
                 device=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.o = kernel_size // 2
        self.a = kernel_size - 1 - self.o
        need = max(self.o, self.a)
        if self.world > 1 and need > 0:
            if H is not None:
                b0, e0 = band_bounds(H, self.world, self.rank)
                if n is not None and int(n) != e0 - b0:
                    raise ValueError(f"rank {self.rank} holds {int(n)} rows but band_bounds({H}, {self.world}, "
                                     f"{self.rank}) gives {e0 - b0}: pass H=None for a custom row split (the band "
                                     f"check then runs a MIN all-reduce)")
                thinnest = min(e - b for b, e in (band_bounds(H, self.world, q) for q in range(self.world)))
            elif n is not None:
                t = torch.tensor([int(n)], dtype=torch.int64, device=device)
                dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
                thinnest = int(t.item())
            else:
                thinnest = None
            if thinnest is not None and thinnest < need:
                raise ValueError(f"the thinnest row band has {thinnest} rows, fewer than the {need} halo rows "
                                 f"kernel_size {kernel_size} needs from a neighbour")

    def _peer(self, rank):
        return dist.get_global_rank(self.group, rank) if self.group is not None else rank

    def _p2p(self, sends, recvs):
        """One batch_isend_irecv of (tensor, group rank) pairs.  Device tensors on a gloo
        group (CPU-only transport, e.g. a single-GPU rehearsal) are staged through host
        memory; with nccl (RCCL over xGMI) they go device to device."""
        stage = dist.get_backend(self.group) == "gloo" and any(t.is_cuda for t, _ in sends + recvs)
        hs = [(t.cpu() if stage else t, q) for t, q in sends]
        hr = [(torch.empty(t.shape, dtype=t.dtype) if stage else t, q) for t, q in recvs]
        # zero-row parts (k = 2: no rows below the patch centre) are not sent at all
        ops = [dist.P2POp(dist.isend, t.contiguous(), self._peer(q), self.group) for t, q in hs if t.numel()]
        ops += [dist.P2POp(dist.irecv, t, self._peer(q), self.group) for t, q in hr if t.numel()]
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        if stage:
            for (dst, _), (src, _) in zip(recvs, hr):
                dst.copy_(src)

    def halo_sizes(self) -> Tuple[int, int]:
        """Rows received from the rank above (o) and from the rank below (a)."""
        top = self.o if self.rank > 0 else 0
        bot = self.a if self.rank < self.world - 1 else 0
        return top, bot

    def exchange_halo(self, band: torch.Tensor) -> torch.Tensor:
        """[n, W] owned rows -> [top + n + bot, W] with the neighbours' edge rows."""
        top, bot = self.halo_sizes()
        if self.world == 1 or self.o + self.a == 0:
            return band
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
        self._p2p(sends, recvs)
        return out

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
        self._p2p(sends, recvs)
        if self.rank > 0 and self.a:
            own[:self.a] += from_up
        if self.rank < self.world - 1 and self.o:
            own[n - self.o:] += from_dn
        return own


class _RowBandStereoMatching(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cam_band, proj_band, D, kernel_size, layout, precision, rbg, backend):
        ch = rbg.exchange_halo(cam_band.contiguous())
        ph = rbg.exchange_halo(proj_band.contiguous())
        top, _ = rbg.halo_sizes()
        n = cam_band.shape[0]
        vol = backend.forward(ch, ph, D, kernel_size, layout, precision, (top, top + n))
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


def stereo_matching_rowband(cam_band: torch.Tensor, proj_band: torch.Tensor, D: int, kernel_size: int,
                            layout: str = "full", precision: Optional[str] = None, group=None,
                            backend=None, H: Optional[int] = None) -> torch.Tensor:
    """Distributed ``stereo_matching``: every rank passes its own row band of
    both images (rows ``band_bounds(H, world, rank)``) and gets the matching
    rows of the cost volume; ``backward`` yields gradients of its own rows.
    ``H`` (the global height) lets the band-thickness check skip its all-reduce."""
    rbg = RowBandGroup(kernel_size, group, n=cam_band.shape[0], H=H, device=cam_band.device)
    return _RowBandStereoMatching.apply(cam_band, proj_band, D, kernel_size, layout, precision, rbg,
                                        backend or HipBackend())


def stereo_disparity_rowband(cam_band, proj_band, D, kernel_size, layout="full", group=None, backend=None,
                             H: Optional[int] = None):
    """Distributed fused disparity for the owned rows (halo exchange only)."""
    rbg = RowBandGroup(kernel_size, group, n=cam_band.shape[0], H=H, device=cam_band.device)
    ch = rbg.exchange_halo(cam_band.contiguous())
    ph = rbg.exchange_halo(proj_band.contiguous())
    top, _ = rbg.halo_sizes()
    n = cam_band.shape[0]
    return (backend or HipBackend()).disparity(ch, ph, D, kernel_size, layout, (top, top + n))
