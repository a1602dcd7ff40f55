"""Same-process interleaved A/B/C of the forward's three forms at C3 and C5 window: the fused launch
(CUSTMA_FWD_FUSED=1: statistics tiles inside the sweep's grid, `sc1` statistics loads; =2: one acquire per
sweep tile and plain loads), the split forward (CUSTMA_FWD_SPLIT=1: two
half-band sweeps on two streams) and the single stream (the default: the statistics pass, then one sweep);
both switches are read per call.  Forward op time from HIP events around the op; every form's volume must
equal the first one's bit for bit.  Usage: python scripts/ab_split.py [rounds]"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import custereomatching_amd as cm  # noqa: E402
from bench import EventTimer, synth_pair  # noqa: E402
from kbench import CFGS, warm  # noqa: E402

FORMS = {"fused": {"CUSTMA_FWD_FUSED": "1"}, "fused_acq": {"CUSTMA_FWD_FUSED": "2"}, "split": {"CUSTMA_FWD_SPLIT": "1"},
         "single": {}}
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
for name in ("c3_win", "c5_win"):
    c = CFGS[name]
    H, W, k, D, lay, dt = c["H"], c["W"], c["k"], c["D"], c["layout"], c["dtype"]
    cam, proj = synth_pair(H, W, D, 5, "cuda", dt)
    out = cm.cost_volume_forward(cam, proj, D, k, lay, "fast")
    ref = out.clone()
    res = {f: [] for f in FORMS}
    reps = 20 if name == "c3_win" else 6
    for r in range(rounds):
        for form, env in FORMS.items():
            for key in ("CUSTMA_FWD_FUSED", "CUSTMA_FWD_SPLIT"):
                os.environ.pop(key, None)
            os.environ.update(env)
            warm(lambda: cm.cost_volume_forward(cam, proj, D, k, lay, "fast", out=out))
            et = EventTimer()
            for _ in range(reps):
                et.record(lambda: cm.cost_volume_forward(cam, proj, D, k, lay, "fast", out=out))
            res[form].append(et.mean_ms())
            assert torch.equal(out, ref), f"{form}: volume differs"
    for key in ("CUSTMA_FWD_FUSED", "CUSTMA_FWD_SPLIT"):
        os.environ.pop(key, None)
    nb = out.numel() * 4 + 2 * H * W * cam.element_size()
    line = {"cfg": name}
    for form in FORMS:
        med = statistics.median(res[form])
        line[form] = {"ms": [round(x, 4) for x in res[form]], "median_ms": round(med, 4),
                      "frac_of_8TBps": round(nb / med / 1e6 / 8000, 4)}
    print(json.dumps(line), flush=True)
    del out, ref
    torch.cuda.empty_cache()
