#!/usr/bin/env python3
"""Benchmark: ZNCC stereo cost volume, forward + backward (grad wrt both images).

BASELINE.json metric: "cost-volume Mvoxels/s (H x W x D) fwd+bwd at 1/2/4/8
MI355X; % HBM roofline".  One step = forward (volume written to HBM) +
backward (synthetic upstream gradient read from HBM, both image gradients
written) through the drop-in autograd op; a voxel is one element of the
returned volume.  Workloads (--workload):

  c5 (default)  BASELINE configs[4]: 4096 x 8192 fp16 pair, D = 256, k = 11,
                window layout [H, W-D, D+1] (8.35e9 voxels per step).  STRONG
                scaling: N ranks split the rows (custereomatching_amd.rowband,
                band_bounds), exchanging k//2 halo rows with their neighbours over
                RCCL (torch.distributed "nccl"); no other collective on the data path.
  c2            BASELINE configs[2]: 1024 x 1024 fp32, D = 128, k = 9, the reference's
                full [H, W, W] volume; WEAK scaling, one 1024-row band per GPU.

`python bench.py --gpus N` with N > 1 and no launcher environment starts
`torch.distributed.run` itself (a child process, before any GPU call) and exits
with its status; under torchrun it reads RANK / LOCAL_RANK / WORLD_SIZE.

Prints ONE JSON line (rank 0).  Extra objects:
  roofline      dominant kernel of the step -- algorithmic bytes / its average
                duration from HIP events around its launches in the timed region;
                `traffic` = HBM bytes per launch from rocprofv3 PMC passes
                (FETCH_SIZE, WRITE_SIZE; separate passes, gfx950 corrections) run
                by this process on the same workload (rank 0, N = 1)
  kernels       the same figures for the forward and backward sweeps
  north_star    BASELINE configs[3]: 2048 x 2048 fp16, D = 256, k = 11, window
                forward, fraction of the 8 TB/s HBM roofline (N = 1)
  config2       the c2 workload's fwd+bwd step at N = 1 (context across rounds)
  cpu_baseline  the reference's torch CPU path (oracle/torch_ref.py restating
                examples/verify.py:81-133) on a bounded row band of the same
                workload, rank 0, N = 1
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

WORKLOADS = {
    "c5": dict(H=4096, W=8192, k=11, D=256, layout="window", dtype=torch.float16, scaling="strong",
               desc="BASELINE configs[4]: fwd+bwd (grads wrt both images), 4096x8192 fp16 pair, D=256, "
                    "window k=11, window layout [H, W-D, D+1]; strong scaling over row bands"),
    "c2": dict(H=1024, W=1024, k=9, D=128, layout="full", dtype=torch.float32, scaling="weak",
               desc="BASELINE configs[2]: fwd+bwd (grads wrt both images) of the reference op's full volume, "
                    "1024x1024 fp32 pair per GPU, D=128, window k=9; weak scaling (1024 rows per GPU)"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c5", choices=sorted(WORKLOADS))
    ap.add_argument("--precision", default="fast", choices=["fast", "exact"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-north-star", action="store_true")
    ap.add_argument("--no-config2", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the PMC traffic passes")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearsal of N ranks on fewer GPUs (halo staged through host memory)")
    ap.add_argument("--pmc-child", default=None, choices=["fwd", "bwd"], help=argparse.SUPPRESS)
    ap.add_argument("--cpu-rows", type=int, default=None, help="rows of the CPU-baseline sample")
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


def fwd_kernel_name(layout, W, D):
    """The forward sweep the library launches (sweep_wave.hip launch_fwd_fast)."""
    if layout == "full":
        return "k_sweep_fwd"
    return "k_fwd_tile" if D + 1 <= 257 else "k_fwd_wave"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(wl, rows):
    """Reference torch path on CPU, bounded sample of the workload (rank 0, N = 1 only)."""
    from oracle import torch_ref

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, os.cpu_count() or 1))
    torch.set_num_threads(threads)
    k, D, W, layout = wl["k"], wl["D"], wl["W"], wl["layout"]
    halo = k - 1
    # fp16 workloads: the reference torch path is fp32; it runs on the fp16 images widened
    cam, proj = synth_pair(rows + halo, W, D, 1234, "cpu", wl["dtype"])
    cam, proj = cam.float(), proj.float()
    torch_ref.forward_backward(cam[: halo + 2], proj[: halo + 2], k, layout=layout, D=D)  # warm-up
    best, runs, t_end = float("inf"), 0, time.time() + 25.0
    while runs < 3 and (runs == 0 or time.time() < t_end):
        t0 = time.perf_counter()
        torch_ref.forward_backward(cam, proj, k, proj_grad=True, layout=layout, D=D)
        best = min(best, time.perf_counter() - t0)
        runs += 1
    WO, DO = (W, W) if layout == "full" else (W - D, D + 1)
    vox = (rows + halo) * WO * DO
    what = "unfold+bmm" if layout == "full" else "unfold + blocked bmm with the window's diagonals read out"
    return {
        "value": round(vox / best / 1e6, 2),
        "unit": "Mvoxels/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"torch CPU restatement of examples/verify.py:81-133 ({what} + autograd, fp32, camera + "
                   f"projector grads) on a {rows + halo}x{W} band of the workload, k={k}, {layout} volume = "
                   f"{vox / 1e6:.1f} Mvox per run, best of {runs}; cpu={_cpu_model()}"),
    }


def north_star(steps, warmup):
    """BASELINE configs[3]: 2048x2048 fp16, D=256, window 11, window layout forward."""
    import custereomatching_amd as cm
    from custereomatching_amd import _lib

    H = W = 2048
    k, D = 11, 256
    cam, proj = synth_pair(H, W, D, 77, "cuda", torch.float16)
    out = cm.cost_volume_forward(cam, proj, D, k, "window", "fast")
    # Warm up to the steady state: the GPU's clocks ramp up over the first ~20 back-to-back launches
    # after any idle gap (1.3-1.5 ms per op, settling at ~1.0 ms; scripts/throttle_probe.py,
    # profiles/r03/dpm/), so at least `warmup` launches AND 0.25 s of back-to-back launches first.
    t0 = time.perf_counter()
    n = 0
    while n < warmup or time.perf_counter() - t0 < 0.25:
        cm.cost_volume_forward(cam, proj, D, k, "window", "fast", out=out)
        n += 1
        if n % 8 == 0:
            torch.cuda.synchronize()
    et = EventTimer()
    _lib.profile_enable(True)
    for _ in range(steps):
        et.record(lambda: cm.cost_volume_forward(cam, proj, D, k, "window", "fast", out=out))
    ms = et.mean_ms()
    kms, nk = _lib.profile_mean_ms(_lib.PROF_FWD)
    _lib.profile_enable(False)
    nvox = out.numel()
    nbytes = nvox * 4 + 2 * H * W * 2
    gbps = nbytes / (ms * 1e-3) / 1e9
    # one statistics launch + one sweep launch per op (a sweep split into overlapping launches would make
    # only op_ms a rate figure: then no per-launch rate is reported)
    per_op = nk / max(1, steps)
    res = {"config": "2048x2048 fp16, D=256, k=11, window [H, W-D, D+1] forward (fast)",
           "kernel": fwd_kernel_name("window", W, D),
           "voxels": nvox, "op_ms": round(ms, 4), "Mvoxels_per_s": round(nvox / (ms * 1e-3) / 1e6, 1),
           "achieved_GBps": round(gbps, 1), "frac_of_8TBps": round(gbps / HBM_PEAK_GBPS, 4),
           "sweep_launches_per_op": round(per_op, 2), "sweep_launch_ms": round(kms, 4), "target_frac": 0.60}
    if round(per_op) == 1:
        kgbps = nbytes / (kms * 1e-3) / 1e9
        res.update(sweep_launch_GBps=round(kgbps, 1), sweep_launch_frac=round(kgbps / HBM_PEAK_GBPS, 4))
    # The fields above count the voxels the window layout writes (H (W - D) (D + 1)).  SURVEY §8(d)'s C3 row
    # prices the target on the nominal H x W x D volume instead (4 B/voxel + both images = 4.31 GB: 60 % of
    # 8 TB/s is <= 0.90 ms, >= 1.2e6 Mvox/s); both are reported, neither replaces the other.
    nom_vox = H * W * D
    nom_bytes = nom_vox * 4 + 2 * H * W * 2
    nom = {"voxels": nom_vox, "bytes": nom_bytes, "Mvoxels_per_s": round(nom_vox / (ms * 1e-3) / 1e6, 1),
           "op_frac": round(nom_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
           "target_ms": round(nom_bytes / (0.60 * HBM_PEAK_GBPS * 1e9) * 1e3, 4)}
    if round(per_op) == 1:
        nom["sweep_launch_frac"] = round(nom_bytes / (kms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
    res["survey_nominal"] = nom
    return res


def config2_step(steps):
    """configs[2] fwd+bwd at N = 1 (the previous rounds' headline workload), HIP events."""
    import custereomatching_amd as cm

    wl = WORKLOADS["c2"]
    H, W, k, D = wl["H"], wl["W"], wl["k"], wl["D"]
    cam, proj = synth_pair(H, W, D, 1000, "cuda")
    cam.requires_grad_(True)
    proj.requires_grad_(True)
    g = torch.empty(H, W, W, device="cuda").uniform_(-1.0, 1.0)

    def step():
        cam.grad = None
        proj.grad = None
        cm.stereo_matching(cam, proj, D, k).backward(g)

    # steady-state clocks first (see north_star): 0.25 s of back-to-back steps
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.25:
        step()
        torch.cuda.synchronize()
    et = EventTimer()
    for _ in range(steps):
        et.record(step)
    ms = et.mean_ms()
    return {"config": wl["desc"], "ms_per_step": round(ms, 4),
            "Mvoxels_per_s": round(H * W * W / (ms * 1e-3) / 1e6, 1)}


def make_inputs(wl, rank, world, dev):
    """Images (band of the global image for strong scaling; own image for weak) + upstream grad."""
    from custereomatching_amd.rowband import band_bounds

    H, W, D = wl["H"], wl["W"], wl["D"]
    if wl["scaling"] == "strong":
        cam, proj = synth_pair(H, W, D, 1000, "cpu", wl["dtype"])
        b, e = band_bounds(H, world, rank)
        cam, proj = cam[b:e].contiguous().to(dev), proj[b:e].contiguous().to(dev)
    else:
        cam, proj = synth_pair(H, W, D, 1000 + rank, dev, wl["dtype"])
    rows = cam.shape[0]
    WO, DO = (W, W) if wl["layout"] == "full" else (W - D, D + 1)
    g = torch.empty(rows, WO, DO, device=dev)
    g.uniform_(-1.0, 1.0, generator=torch.Generator(device=dev).manual_seed(7 + rank))
    return cam, proj, g


def pmc_child(args):
    """Child of a rocprofv3 --pmc pass: the workload's dominant op, a few launches, nothing else."""
    import custereomatching_amd as cm

    wl = WORKLOADS[args.workload]
    torch.cuda.set_device(0)
    cam, proj, g = make_inputs(wl, 0, 1, torch.device("cuda", 0))
    k, D, lay = wl["k"], wl["D"], wl["layout"]
    vol = cm.cost_volume_forward(cam, proj, D, k, lay, args.precision)
    for _ in range(3):
        if args.pmc_child == "fwd":
            cm.cost_volume_forward(cam, proj, D, k, lay, args.precision, out=vol)
        else:
            cm.cost_volume_backward(g, cam, proj, k, lay, D, camera_grad=True, projector_grad=True,
                                    cost_volume=vol)
    torch.cuda.synchronize()


def _pmc_pass(args, which, kernel, counters, out):
    """One rocprofv3 --pmc pass over a child running the op; mean value per `kernel` launch."""
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    d = os.path.join(out, counters[0])
    cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--pmc", *counters, "-d", d, "-o", "run",
           "--output-format", "csv", "--", sys.executable, os.path.abspath(__file__), "--workload",
           args.workload, "--precision", args.precision, "--pmc-child", which]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True)
    if r.returncode != 0:
        return None, f"rocprofv3 --pmc {' '.join(counters)} failed (rc {r.returncode}): {r.stderr[-300:]}"
    xs = {c: [] for c in counters}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] in xs:
                xs[row["Counter_Name"]].append(float(row["Counter_Value"]))
    if not all(xs.values()):
        return None, f"no {counters} samples for {kernel}"
    return {c: sum(v) / len(v) for c, v in xs.items()}, None


def pmc_traffic(args, which, kernel):
    """HBM bytes per launch of `kernel`: two rocprofv3 passes over a child running the op
    (FETCH_SIZE and WRITE_SIZE cannot share a pass; MI355X_MICROARCH.md §HBM/rocprofv3:
    both in KiB, FETCH_SIZE reports half the bytes on gfx950 -> x2048 and x1024 B/unit),
    plus one SQ pass for the instruction mix (wave-instructions per launch)."""
    out = tempfile.mkdtemp(prefix="custma_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    vals = {}
    for counter, scale in (("FETCH_SIZE", 2048.0), ("WRITE_SIZE", 1024.0)):
        v, err = _pmc_pass(args, which, kernel, [counter], out)
        if v is None:
            return None, err
        vals[counter] = v[counter] * scale
    sq, _ = _pmc_pass(args, which, kernel, ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES"], out)
    src = (f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ_INSTS_* passes (separate) over `bench.py --pmc-child "
           f"{which}` (same workload), mean per {kernel} launch; FETCH x2048 B, WRITE x1024 B per unit")
    return {"read": vals["FETCH_SIZE"], "write": vals["WRITE_SIZE"],
            "total": vals["FETCH_SIZE"] + vals["WRITE_SIZE"], "sq": sq}, src


def main():
    args = parse()
    if args.pmc_child:
        pmc_child(args)
        return
    world = args.gpus
    if world > 1 and "RANK" not in os.environ:
        # no launcher: start one (child process; nothing has touched the GPU yet) and pass its status on
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__),
               *sys.argv[1:]]
        sys.exit(subprocess.run(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1")).returncode)

    import torch.distributed as dist

    distributed = world > 1
    if distributed:
        rank = int(os.environ["RANK"])
        local = int(os.environ.get("LOCAL_RANK", rank))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            local = local % max(1, torch.cuda.device_count())
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
    else:
        rank, local = 0, 0
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local)

    import custereomatching_amd as cm
    from custereomatching_amd import _lib
    from custereomatching_amd import rowband

    wl = WORKLOADS[args.workload]
    H, W, k, D, layout = wl["H"], wl["W"], wl["k"], wl["D"], wl["layout"]
    cam, proj, g = make_inputs(wl, rank, world, dev)
    cam.requires_grad_(True)
    proj.requires_grad_(True)
    global_H = H if wl["scaling"] == "strong" else H * world
    # the row-band group (halo sizes, the collective band check) once for the whole run
    rbg = rowband.RowBandGroup(k, None, n=cam.shape[0], H=global_H, device=dev) if distributed else None

    def op():
        if distributed:
            return rowband.stereo_matching_rowband(cam, proj, D, k, layout, args.precision, rbg=rbg)
        return cm.stereo_matching(cam, proj, D, k, layout, args.precision)

    spans = []  # (start, forward done, backward done) events per timed step, on the op's stream

    def step(timed=False):
        cam.grad = None
        proj.grad = None
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)] if timed else None
        if timed:
            ev[0].record()
        vol = op()
        if timed:
            ev[1].record()
        vol.backward(g)
        if timed:
            ev[2].record()
            spans.append(ev)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    # HIP events around the two sweep kernels of every op in the timed region (recorded by the
    # library on the op's stream; custma_profile_*), for the roofline figures
    _lib.profile_enable(True)
    if distributed:
        rowband.enable_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timed=True)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # the forward / backward op spans of every step (statistics, sweeps, side passes; overlapped
    # launches counted once)
    fwd_span_ms = sum(a.elapsed_time(b) for a, b, _ in spans) / len(spans)
    bwd_span_ms = sum(b.elapsed_time(c) for _, b, c in spans) / len(spans)
    fwd_kms, n_fk = _lib.profile_mean_ms(_lib.PROF_FWD)
    bwd_kms, n_bk = _lib.profile_mean_ms(_lib.PROF_BWD)
    _lib.profile_enable(False)
    per_rank = None
    if distributed:
        # per rank: sweep kernel times (HIP events; one forward sweep launch per step, three with
        # CUSTMA_ROWBAND_OVERLAP=1) and the exchange times the op's stream waited for (rowband timing)
        mine = {"rank": rank, "rows": int(cam.shape[0]), "fwd_sweep_launch_ms": round(fwd_kms, 4),
                "fwd_sweep_launches_per_step": round(n_fk / max(1, args.steps), 2),
                "bwd_sweep_launch_ms": round(bwd_kms, 4), "step_ms_local": round(elapsed / args.steps * 1e3, 4)}
        # (gloo rehearsal: the halos are staged through host memory, so these spans include the device-host
        # copies and the host wait -- a rehearsal of the bookkeeping, not an xGMI figure)
        mine.update(rowband.timing_summary())
        mine["exchange_transport"] = "rccl (device to device)" if args.dist_backend == "nccl" else "gloo (host-staged)"
        rowband.enable_timing(False)
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    rows = cam.shape[0]
    WO, DO = (W, W) if layout == "full" else (W - D, D + 1)
    nvox_rank = rows * WO * DO
    tot = torch.tensor([elapsed, float(nvox_rank)], dtype=torch.float64,
                       device=dev if args.dist_backend == "nccl" else "cpu")
    if distributed:
        t_max = tot[:1].clone()
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        v_sum = tot[1:].clone()
        dist.all_reduce(v_sum, op=dist.ReduceOp.SUM)
        elapsed, nvox_all = float(t_max.item()), float(v_sum.item())
    else:
        nvox_all = float(nvox_rank)
    # distinct GPUs the ranks actually ran on (a gloo rehearsal maps several ranks to one GPU)
    n_dev = 1
    if distributed:
        devs = [None] * world
        dist.all_gather_object(devs, (socket.gethostname(), torch.cuda.current_device()))
        n_dev = len(set(devs))
    value = nvox_all * args.steps / elapsed / 1e6
    ms_step = elapsed / args.steps * 1e3

    # Algorithmic bytes per launch, SURVEY.md §8(d) unit-of-work formulas, this rank's band:
    #   forward  : N_vox * 4 (volume written) + 2 H W sizeof(image)
    #   backward : N_vox * 4 (upstream gradient read) + 2 H W sizeof(image) + 2 H W * 4 (both gradients)
    # The backward's design also re-reads the saved volume (V = A * cost / S):
    # `design_bytes` adds that N_vox * 4; it is reported beside, never as the roofline figure.
    esz = cam.element_size()
    img = 2 * cam.numel() * esz
    fwd_bytes = nvox_rank * 4 + img
    bwd_bytes = nvox_rank * 4 + img + 2 * cam.numel() * 4
    bwd_design = bwd_bytes + nvox_rank * 4
    fwd_name = fwd_kernel_name(layout, W, D)
    # The forward's bytes are per step; at N > 1 with CUSTMA_ROWBAND_OVERLAP=1 it runs as an interior
    # launch + two edge launches (rowband), and a large band's sweep may run as two half-band launches
    # that overlap in time
    # (DESIGN.md §3.1).  So its rate is taken over the forward op's whole span per step (events on the
    # op's stream before and after the op: statistics pass included, overlapped launches counted once),
    # never over a sum of launch times.
    fwd_step_ms = fwd_span_ms
    kern = {
        fwd_name: {"avg_launch_ms": round(fwd_kms, 4), "launches_per_step": round(n_fk / max(1, args.steps), 2),
                   "op_span_ms": round(fwd_span_ms, 4), "algorithmic_bytes": fwd_bytes,
                   "achieved_GBps": round(fwd_bytes / (fwd_span_ms * 1e-3) / 1e9, 1),
                   "timing": "events around the forward op on its stream (span per step)"},
        "backward_op": {"op_span_ms": round(bwd_span_ms, 4)},
        "k_bwd_coop": {"avg_launch_ms": round(bwd_kms, 4), "launches": n_bk, "algorithmic_bytes": bwd_bytes,
                       "design_bytes": bwd_design,
                       "achieved_GBps": round(bwd_bytes / (bwd_kms * 1e-3) / 1e9, 1) if bwd_kms else None,
                       "design_GBps": round(bwd_design / (bwd_kms * 1e-3) / 1e9, 1) if bwd_kms else None},
    }
    dom = "k_bwd_coop" if bwd_kms >= fwd_step_ms else fwd_name
    dk = kern[dom]
    achieved = dk["achieved_GBps"] or 0.0
    result = {
        "metric": "cost-volume Mvoxels/s (H x W x D) fwd+bwd",
        "value": round(value, 1),
        "unit": "Mvoxels/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": wl["scaling"] if n_dev == world else "rehearsal (ranks share GPUs; not a scaling figure)",
        "vs_baseline": None,
        "dtype": "f16" if wl["dtype"] == torch.float16 else "f32",
        "data": "synthetic (seeded speckle pair, camera = shifted projector + noise; uniform upstream grad)",
        "config": {
            "workload": wl["desc"],
            "H": global_H, "W": W, "k": k, "D": D, "layout": layout, "precision": args.precision,
            "rows_per_gpu": rows, "voxels_per_step": int(nvox_all),
            "parallelism": (f"rowband{world}" + ("" if n_dev == world else f"-rehearsal-on-{n_dev}-gpu"))
                           if distributed else "single",
            "dist_backend": args.dist_backend if distributed else None,
            "distinct_gpus": n_dev,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": dom,
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": None,
            "algorithmic_bytes_per_launch": dk["algorithmic_bytes"],
            "algorithmic_formula": ("N_vox*4 + 2*H*W*sizeof(image) + 2*H*W*4 (SURVEY 8(d) backward)"
                                    if dom == "k_bwd_coop" else "N_vox*4 + 2*H*W*sizeof(image) (SURVEY 8(d) forward)"),
            "design_bytes_per_launch": dk.get("design_bytes", dk["algorithmic_bytes"]),
            "avg_launch_ms": dk["avg_launch_ms"],
            "timing": "HIP events around each launch of the kernel on the op's stream, over the timed steps",
        },
        "kernels": kern,
    }
    if per_rank is not None:
        result["per_rank"] = per_rank
    del g
    cam.grad = proj.grad = None
    torch.cuda.empty_cache()
    if rank == 0 and world == 1:
        if not args.no_north_star:
            result["north_star"] = north_star(max(20, args.steps), 40)
        if not args.no_config2 and args.workload != "c2":
            result["config2"] = config2_step(max(5, args.steps // 2))
        torch.cuda.empty_cache()
        if not args.no_pmc:
            traffic, src = pmc_traffic(args, "bwd" if dom == "k_bwd_coop" else "fwd", dom)
            if traffic is not None:
                rf = result["roofline"]
                rf["traffic"] = round(traffic["total"])
                rf["traffic_read"] = round(traffic["read"])
                rf["traffic_write"] = round(traffic["write"])
                rf["traffic_over_algorithmic"] = round(traffic["total"] / rf["algorithmic_bytes_per_launch"], 3)
                rf["traffic_over_design"] = round(traffic["total"] / rf["design_bytes_per_launch"], 3)
                sq = traffic.get("sq")
                if sq:
                    rf["sq_per_launch"] = {k: round(v) for k, v in sq.items()}
                    rf["valu_wave_insts_per_voxel"] = round(sq["SQ_INSTS_VALU"] / nvox_rank, 4)
                    rf["valu_lane_ops_per_voxel"] = round(64 * sq["SQ_INSTS_VALU"] / nvox_rank, 2)
            result["roofline"]["traffic_source"] = src
        if not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(wl, args.cpu_rows or (48 if layout == "window" else 96))
    if rank == 0:
        print(json.dumps(result), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
