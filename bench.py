#!/usr/bin/env python3
"""Benchmark: ZNCC stereo cost volume, forward + backward (grad wrt both images).

BASELINE.json metric: "cost-volume Mvoxels/s (H x W x D) fwd+bwd at 1/2/4/8
MI355X; % HBM roofline".  Workload = BASELINE configs[2]: 1024 x 1024 fp32
image pair per GPU, D = 128, window 9, forward + backward with gradients
w.r.t. both images.  Layout "full" is what the reference op returns
([H, W, W]; D ignored, custma/src/stereo_matching_kernel.cu:14,200), so a
voxel is one element of that volume (1.07e9 per step per GPU).

One step = forward (volume written to HBM) + backward (synthetic upstream
gradient read from HBM, both image gradients written), through the drop-in
autograd op.  N > 1 GPUs (launched by torch.distributed.run): weak scaling by
row bands -- each rank owns a 1024-row band of a (1024 N)-row image pair and
exchanges k//2 halo rows with its neighbours over RCCL (custereomatching_amd.
rowband); no other collective on the data path.

Prints ONE JSON line (rank 0).  Extra objects:
  roofline      dominant kernel (the backward sweep, k_bwd_coop) -- algorithmic
                bytes / its average duration from HIP events around its launches in
                the timed region; "kernels" has the same for the forward sweep
  cpu_baseline  the reference's torch CPU path (oracle/torch_ref.py restating
                examples/verify.py:81-133) on a bounded row band, rank 0, N=1
  north_star    BASELINE configs[3]: 2048 x 2048 fp16, D = 256, k = 11, window
                layout forward, % of HBM roofline
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--H", type=int, default=1024, help="rows per GPU")
    ap.add_argument("--W", type=int, default=1024)
    ap.add_argument("--k", type=int, default=9)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--layout", default="full", choices=["full", "window"])
    ap.add_argument("--precision", default="fast", choices=["fast", "exact"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-north-star", action="store_true")
    ap.add_argument("--cpu-rows", type=int, default=96, help="row band timed for the CPU baseline")
    return ap.parse_args()


def synth_pair(H, W, D, seed, device, dtype=torch.float32):
    """Seeded speckle projector, camera = projector shifted by a per-16-row
    disparity in [0, D) + N(0, 0.01) noise."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    proj = torch.rand(H, W, generator=g)
    disp = torch.randint(0, max(D, 1), ((H + 15) // 16,), generator=g).repeat_interleave(16)[:H]
    cols = (torch.arange(W)[None, :] + disp[:, None]).clamp(max=W - 1)
    cam = torch.gather(proj, 1, cols) + 0.01 * torch.randn(H, W, generator=g)
    cam = cam.clamp(0, 1)
    return cam.to(device=device, dtype=dtype).contiguous(), proj.to(device=device, dtype=dtype).contiguous()


class EventTimer:
    """HIP-event timing on torch's current stream (where the library launches)."""

    def __init__(self):
        self.pairs = []

    def record(self, fn):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        out = fn()
        e.record()
        self.pairs.append((s, e))
        return out

    def mean_ms(self):
        torch.cuda.synchronize()
        return sum(s.elapsed_time(e) for s, e in self.pairs) / max(1, len(self.pairs))


def cpu_baseline(args, k):
    """Reference torch path on CPU, bounded sample (rank 0, N = 1 only)."""
    from oracle import torch_ref

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, os.cpu_count() or 1))
    torch.set_num_threads(threads)
    rows = args.cpu_rows
    r = k // 2
    cam, proj = synth_pair(rows + 2 * r, args.W, args.D, 1234, "cpu")
    best = float("inf")
    t_end = time.time() + 25.0
    runs = 0
    torch_ref.forward_backward(cam[: 2 * r + 8], proj[: 2 * r + 8], k)  # warm-up (allocator, threads)
    while runs < 3 and (runs == 0 or time.time() < t_end):
        t0 = time.perf_counter()
        _, gc, gp = torch_ref.forward_backward(cam, proj, k, proj_grad=True)
        best = min(best, time.perf_counter() - t0)
        runs += 1
    vox = (rows + 2 * r) * args.W * args.W
    return {
        "value": round(vox / best / 1e6, 2),
        "unit": "Mvoxels/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"torch CPU restatement of examples/verify.py:81-133 (unfold+bmm+autograd, fp32, "
                   f"camera+projector grads) on a {rows + 2 * r}x{args.W} band, k={k}, full [H,W,W] "
                   f"volume = {vox / 1e6:.1f} Mvox per run, best of {runs}; cpu={_cpu_model()}"),
    }


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def north_star(steps, warmup):
    """BASELINE configs[3]: 2048x2048 fp16, D=256, window 11, window layout forward."""
    import custereomatching_amd as cm
    from custereomatching_amd import _lib

    H = W = 2048
    k, D = 11, 256
    cam, proj = synth_pair(H, W, D, 77, "cuda", torch.float16)
    out = cm.cost_volume_forward(cam, proj, D, k, "window", "fast")
    for _ in range(warmup):
        cm.cost_volume_forward(cam, proj, D, k, "window", "fast", out=out)
    et = EventTimer()
    _lib.profile_enable(True)
    for _ in range(steps):
        et.record(lambda: cm.cost_volume_forward(cam, proj, D, k, "window", "fast", out=out))
    ms = et.mean_ms()
    kms, _ = _lib.profile_mean_ms(_lib.PROF_FWD)
    _lib.profile_enable(False)
    nvox = out.numel()
    nbytes = nvox * 4 + 2 * H * W * 2
    gbps = nbytes / (ms * 1e-3) / 1e9
    kgbps = nbytes / (kms * 1e-3) / 1e9
    return {"config": "2048x2048 fp16, D=256, k=11, window [H, W-D, D+1] forward (fast)",
            "voxels": nvox, "op_ms": round(ms, 4), "Mvoxels_per_s": round(nvox / (ms * 1e-3) / 1e6, 1),
            "achieved_GBps": round(gbps, 1), "frac_of_8TBps": round(gbps / HBM_PEAK_GBPS, 4),
            "sweep_kernel_ms": round(kms, 4), "sweep_kernel_GBps": round(kgbps, 1),
            "sweep_kernel_frac": round(kgbps / HBM_PEAK_GBPS, 4), "target_frac": 0.60}


def main():
    args = parse()
    world = args.gpus
    distributed = world > 1
    if distributed:
        rank = int(os.environ["RANK"])
        local = int(os.environ.get("LOCAL_RANK", rank))
        torch.cuda.set_device(local)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        rank, local = 0, 0
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local)

    import custereomatching_amd as cm
    from custereomatching_amd import _lib
    from custereomatching_amd.rowband import stereo_matching_rowband

    H, W, k, D = args.H, args.W, args.k, args.D
    cam, proj = synth_pair(H, W, D, 1000 + rank, dev)
    cam.requires_grad_(True)
    proj.requires_grad_(True)
    WO = W if args.layout == "full" else W - D
    DO = W if args.layout == "full" else D + 1
    g = torch.empty(H, WO, DO, device=dev)
    g.uniform_(-1.0, 1.0, generator=torch.Generator(device=dev).manual_seed(7 + rank))

    def op():
        if distributed:
            return stereo_matching_rowband(cam, proj, D, k, args.layout, args.precision)
        return cm.stereo_matching(cam, proj, D, k, args.layout, args.precision)

    def step():
        cam.grad = None
        proj.grad = None
        vol = op()
        vol.backward(g)
        return vol

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    # HIP events around the two sweep kernels of every op in the timed region (recorded by the
    # library on the op's stream; custma_profile_*), for the roofline figures
    _lib.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    fwd_kms, n_fk = _lib.profile_mean_ms(_lib.PROF_FWD)
    bwd_kms, n_bk = _lib.profile_mean_ms(_lib.PROF_BWD)
    _lib.profile_enable(False)
    if distributed:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    nvox_rank = H * WO * DO
    value = world * nvox_rank * args.steps / elapsed / 1e6
    ms_step = elapsed / args.steps * 1e3

    # Per-op HIP-event timing (same stream as the kernels), outside the timed region.
    et_f, et_b = EventTimer(), EventTimer()
    vol = cm.cost_volume_forward(cam.detach(), proj.detach(), D, k, args.layout, args.precision)
    for _ in range(max(3, args.steps // 2)):
        with torch.no_grad():
            et_f.record(lambda: cm.cost_volume_forward(cam.detach(), proj.detach(), D, k, args.layout,
                                                       args.precision, out=vol))
        et_b.record(lambda: cm.cost_volume_backward(g, cam.detach(), proj.detach(), k, args.layout, D,
                                                    camera_grad=True, projector_grad=True, cost_volume=vol))
    del vol
    fwd_ms, bwd_ms = et_f.mean_ms(), et_b.mean_ms()
    # Algorithmic bytes per launch:
    #   forward sweep  : volume written once + both images read
    #   backward sweep : upstream gradient + saved volume read once each, both images read,
    #                    both image gradients written
    img = 2 * H * W * 4
    fwd_bytes = nvox_rank * 4 + img
    bwd_bytes = 2 * nvox_rank * 4 + img + img
    # forward sweep kernel by layout (sweep_wave.hip launch_fwd_fast): full -> k_sweep_fwd, window -> k_fwd_wave
    fwd_name = "k_sweep_fwd" if args.layout == "full" else "k_fwd_wave"
    kern = {
        fwd_name: {"avg_launch_ms": round(fwd_kms, 4), "launches": n_fk, "algorithmic_bytes": fwd_bytes,
                        "achieved_GBps": round(fwd_bytes / (fwd_kms * 1e-3) / 1e9, 1) if fwd_kms else None},
        "k_bwd_coop": {"avg_launch_ms": round(bwd_kms, 4), "launches": n_bk, "algorithmic_bytes": bwd_bytes,
                        "achieved_GBps": round(bwd_bytes / (bwd_kms * 1e-3) / 1e9, 1) if bwd_kms else None},
    }
    dom = "k_bwd_coop" if bwd_kms >= fwd_kms else fwd_name
    dk = kern[dom]
    achieved = dk["achieved_GBps"] or 0.0

    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_{dom}_c2_{args.layout}.json")
    if os.path.exists(pmc_path):
        try:
            traffic = json.load(open(pmc_path)).get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    result = {
        "metric": "cost-volume Mvoxels/s (H x W x D) fwd+bwd",
        "value": round(value, 1),
        "unit": "Mvoxels/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded speckle pair, camera = shifted projector + noise; uniform upstream grad)",
        "config": {
            "workload": ("BASELINE configs[2]: fwd+bwd (grads wrt both images) of the reference op's "
                         f"{args.layout} volume, {H}x{W} fp32 pair per GPU, D={D}, window k={k}"),
            "H_per_gpu": H, "W": W, "k": k, "D": D, "layout": args.layout, "precision": args.precision,
            "voxels_per_gpu_per_step": nvox_rank, "global_H": H * world,
            "parallelism": f"rowband{world}" if distributed else "single",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": dom,
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "algorithmic_bytes_per_launch": dk["algorithmic_bytes"],
            "avg_launch_ms": dk["avg_launch_ms"],
            "timing": "HIP events around each launch of the kernel on the op's stream, over the timed steps",
        },
        "kernels": kern,
        "breakdown": {
            "fwd_op_ms": round(fwd_ms, 4), "bwd_op_ms": round(bwd_ms, 4),
            "fwd_Mvox_s": round(nvox_rank / (fwd_ms * 1e-3) / 1e6, 1),
            "bwd_Mvox_s": round(nvox_rank / (bwd_ms * 1e-3) / 1e6, 1),
        },
    }
    del g
    torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_north_star:
        result["north_star"] = north_star(max(5, args.steps), 2)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, k)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
