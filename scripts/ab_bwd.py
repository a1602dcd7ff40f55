"""Same-process interleaved A/B of backward variants selected per call by environment switches (C5 and C3
window): the default against each listed form, backward op time from HIP events around the op, the
gradients of every form bit-identical to the default's.  Forms:
  gather8=0   CUSTMA_BWD_GATHER8=0: the per-slot-pair gather loop instead of the batched-load gather
and, for the full-layout forward (C2 / C3 full), full_x4=0 (CUSTMA_FULL_X4=0: dword volume stores)
Usage: python scripts/ab_bwd.py [rounds]"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import custereomatching_amd as cm  # noqa: E402
from bench import EventTimer, synth_pair  # noqa: E402
from kbench import CFGS, warm  # noqa: E402

FORMS = {"default": {}, "gather8=0": {"CUSTMA_BWD_GATHER8": "0"}}
FWD_FORMS = {"default": {}, "full_x4=0": {"CUSTMA_FULL_X4": "0"}}
KEYS = sorted({k for env in FORMS.values() for k in env})
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
for name in ("c3_win", "c5_win"):
    c = CFGS[name]
    H, W, k, D, lay, dt = c["H"], c["W"], c["k"], c["D"], c["layout"], c["dtype"]
    cam, proj = synth_pair(H, W, D, 5, "cuda", dt)
    vol = cm.cost_volume_forward(cam, proj, D, k, lay, "fast")
    g = torch.empty_like(vol).uniform_(-1.0, 1.0)
    ref = None
    res = {f: [] for f in FORMS}
    reps = 10 if name == "c3_win" else 4

    def op():
        return cm.cost_volume_backward(g, cam, proj, k, lay, D, projector_grad=True, cost_volume=vol)

    for r in range(rounds):
        for form, env in FORMS.items():
            for key in KEYS:
                os.environ.pop(key, None)
            os.environ.update(env)
            warm(op)
            et = EventTimer()
            out = None
            for _ in range(reps):
                out = et.record(op)
            res[form].append(et.mean_ms())
            if ref is None:
                ref = out
            assert torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1]), f"{form}: gradients differ"
    for key in KEYS:
        os.environ.pop(key, None)
    line = {"cfg": name}
    for form in FORMS:
        line[form] = {"ms": [round(x, 4) for x in res[form]], "median_ms": round(statistics.median(res[form]), 4)}
    print(json.dumps(line), flush=True)
    del vol, g, ref
    torch.cuda.empty_cache()

# the full-layout forward's store form (CUSTMA_FULL_X4=0: per-lane dword stores) at configs[2] and C3 full
for name in ("c2_full", "c3_full"):
    c = CFGS[name]
    H, W, k, D, lay, dt = c["H"], c["W"], c["k"], c["D"], c["layout"], c["dtype"]
    cam, proj = synth_pair(H, W, D, 5, "cuda", dt)
    out = cm.cost_volume_forward(cam, proj, D, k, lay, "fast")
    ref = out.clone()
    res = {f: [] for f in FWD_FORMS}
    for r in range(rounds):
        for form, env in FWD_FORMS.items():
            os.environ.pop("CUSTMA_FULL_X4", None)
            os.environ.update(env)
            warm(lambda: cm.cost_volume_forward(cam, proj, D, k, lay, "fast", out=out))
            et = EventTimer()
            for _ in range(10):
                et.record(lambda: cm.cost_volume_forward(cam, proj, D, k, lay, "fast", out=out))
            res[form].append(et.mean_ms())
            assert torch.equal(out, ref), f"{form}: volume differs"
    os.environ.pop("CUSTMA_FULL_X4", None)
    line = {"cfg": name, "op": "fwd"}
    for form in FWD_FORMS:
        line[form] = {"ms": [round(x, 4) for x in res[form]], "median_ms": round(statistics.median(res[form]), 4)}
    print(json.dumps(line), flush=True)
    del out, ref
    torch.cuda.empty_cache()
