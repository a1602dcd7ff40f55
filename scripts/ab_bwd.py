"""Same-process interleaved A/B of backward variants selected per call by environment switches (C5 and C3
window): the default against each listed form, backward op time from HIP events around the op, the
gradients of every form bit-identical to the default's.  Forms:
  gather8=0   CUSTMA_BWD_GATHER8=0: the per-slot-pair gather loop instead of the batched-load gather
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
