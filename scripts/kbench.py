"""Quick per-op timing (HIP events) for kernel iteration. Not the contract bench."""
import argparse, json, os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import custereomatching_amd as cm
from custereomatching_amd import _lib
from bench import synth_pair, EventTimer

CFGS = {
    "c2_full": dict(H=1024, W=1024, k=9, D=128, layout="full", dtype=torch.float32),
    "c2_win": dict(H=1024, W=1024, k=9, D=128, layout="window", dtype=torch.float32),
    "c3_win": dict(H=2048, W=2048, k=11, D=256, layout="window", dtype=torch.float16),
    "c3_full": dict(H=2048, W=2048, k=11, D=256, layout="full", dtype=torch.float16),
    "c3_win_d255": dict(H=2048, W=2048, k=11, D=255, layout="window", dtype=torch.float16),
    "c5_win": dict(H=4096, W=8192, k=11, D=256, layout="window", dtype=torch.float16),
    # one rank's band of configs[4] at N = 2 / 4 / 8 (strong scaling over row bands): whole images of the haloed
    # band's height (owned rows + 2 r) stand in for the bands -- the backward's row groups then match a middle
    # rank's (33 / 65 / 129 of 16 rows)
    "c5_r2": dict(H=2058, W=8192, k=11, D=256, layout="window", dtype=torch.float16),
    "c5_r4": dict(H=1034, W=8192, k=11, D=256, layout="window", dtype=torch.float16),
    "c5_r8": dict(H=522, W=8192, k=11, D=256, layout="window", dtype=torch.float16),
    # kernel sizes without a sweep instantiation (exact forward + generic fp64 backward)
    "c3_win_k17": dict(H=2048, W=2048, k=17, D=256, layout="window", dtype=torch.float16),
    "c3_win_k16": dict(H=2048, W=2048, k=16, D=256, layout="window", dtype=torch.float16),
    "c3_win_k4": dict(H=2048, W=2048, k=4, D=256, layout="window", dtype=torch.float16),
    "c3_win_k8": dict(H=2048, W=2048, k=8, D=256, layout="window", dtype=torch.float16),
    "c3_win_k12": dict(H=2048, W=2048, k=12, D=256, layout="window", dtype=torch.float16),
    "c2_full_k10": dict(H=1024, W=1024, k=10, D=128, layout="full", dtype=torch.float32),
    "c3_win_k19": dict(H=2048, W=2048, k=19, D=256, layout="window", dtype=torch.float16),
    "c3_win_k25": dict(H=2048, W=2048, k=25, D=256, layout="window", dtype=torch.float16),
    "c3_win_k31": dict(H=2048, W=2048, k=31, D=256, layout="window", dtype=torch.float16),
    "c3_win_k18": dict(H=2048, W=2048, k=18, D=256, layout="window", dtype=torch.float16),
    "c3_win_k22": dict(H=2048, W=2048, k=22, D=256, layout="window", dtype=torch.float16),
    "c3_win_k30": dict(H=2048, W=2048, k=30, D=256, layout="window", dtype=torch.float16),
    "c3_full_k19": dict(H=2048, W=2048, k=19, D=256, layout="full", dtype=torch.float16),
    # other sweep kernel sizes at C3 size
    "c3_win_k5": dict(H=2048, W=2048, k=5, D=256, layout="window", dtype=torch.float16),
    "c3_win_k9": dict(H=2048, W=2048, k=9, D=256, layout="window", dtype=torch.float16),
    "c3_win_k13": dict(H=2048, W=2048, k=13, D=256, layout="window", dtype=torch.float16),
}

def warm(fn, secs=0.25):
    """Back-to-back launches until the clocks have ramped up (scripts/throttle_probe.py)."""
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < secs:
        fn()
        torch.cuda.synchronize()


def run(name, ops, reps):
    c = CFGS[name]
    H, W, k, D, lay, dt = c["H"], c["W"], c["k"], c["D"], c["layout"], c["dtype"]
    cam, proj = synth_pair(H, W, D, 5, "cuda", dt)
    res = {"cfg": name}
    if "fwd" in ops or "exact" in ops:
        for prec in [p for p in ("fast", "exact") if (p == "fast" and "fwd" in ops) or (p == "exact" and "exact" in ops)]:
            out = cm.cost_volume_forward(cam, proj, D, k, lay, prec)
            warm(lambda: cm.cost_volume_forward(cam, proj, D, k, lay, prec, out=out))
            et = EventTimer()
            _lib.profile_enable(True)
            for _ in range(reps):
                et.record(lambda: cm.cost_volume_forward(cam, proj, D, k, lay, prec, out=out))
            ms = et.mean_ms()
            kms, nk = _lib.profile_mean_ms(_lib.PROF_FWD)
            _lib.profile_enable(False)
            res[f"fwd_{prec}_kernel_ms"] = round(kms, 4)  # per sweep launch
            if nk != reps:
                res[f"fwd_{prec}_launches_per_op"] = round(nk / reps, 2)
            nb = out.numel() * 4 + 2 * H * W * cam.element_size()
            res[f"fwd_{prec}_ms"] = round(ms, 4)
            res[f"fwd_{prec}_GBps"] = round(nb / ms / 1e6, 1)
            del out
    if "bwd" in ops:
        vol = cm.cost_volume_forward(cam, proj, D, k, lay, "fast")
        g = torch.rand_like(vol) - 0.5
        warm(lambda: cm.cost_volume_backward(g, cam, proj, k, lay, D, projector_grad=True, cost_volume=vol))
        et = EventTimer()
        for _ in range(reps):
            et.record(lambda: cm.cost_volume_backward(g, cam, proj, k, lay, D, projector_grad=True,
                                                      cost_volume=vol))
        ms = et.mean_ms()
        res["bwd_ms"] = round(ms, 4)
        res["bwd_GBps_g_vol"] = round(2 * g.numel() * 4 / ms / 1e6, 1)
        del g, vol
    if "disp" in ops:
        warm(lambda: cm.stereo_disparity(cam, proj, D, k, lay))
        et = EventTimer()
        nre = None
        for _ in range(reps):
            nre = et.record(lambda: cm.stereo_disparity(cam, proj, D, k, lay, return_rechecked=True))
        res["disp_ms"] = round(et.mean_ms(), 4)
        res["disp_rechecked"] = int(nre[2].item())
    if "soft" in ops:
        warm(lambda: cm.stereo_disparity_soft(cam, proj, D, k, lay))
        et = EventTimer()
        for _ in range(reps):
            et.record(lambda: cm.stereo_disparity_soft(cam, proj, D, k, lay))
        res["soft_ms"] = round(et.mean_ms(), 4)
    torch.cuda.empty_cache()
    return res

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="c2_full,c3_win")
    ap.add_argument("--ops", default="fwd,bwd")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    for n in a.cfg.split(","):
        print(json.dumps(run(n, a.ops.split(","), a.reps)), flush=True)
