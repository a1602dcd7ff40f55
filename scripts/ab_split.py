"""Same-process interleaved A/B of the split forward (capi.hip forward_split) against the
single-stream form (CUSTMA_FWD_SPLIT=0, read per call): forward op time (HIP events around the op)
at C3 and C5 window.  Usage: python scripts/ab_split.py [rounds]"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import custereomatching_amd as cm  # noqa: E402
from bench import EventTimer, synth_pair  # noqa: E402
from kbench import CFGS, warm  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
for name in ("c3_win", "c5_win"):
    c = CFGS[name]
    H, W, k, D, lay, dt = c["H"], c["W"], c["k"], c["D"], c["layout"], c["dtype"]
    cam, proj = synth_pair(H, W, D, 5, "cuda", dt)
    out = cm.cost_volume_forward(cam, proj, D, k, lay, "fast")
    ref = out.clone()
    res = {"1": [], "0": []}
    reps = 20 if name == "c3_win" else 6
    for r in range(rounds):
        for mode in ("1", "0"):
            os.environ["CUSTMA_FWD_SPLIT"] = mode
            warm(lambda: cm.cost_volume_forward(cam, proj, D, k, lay, "fast", out=out))
            et = EventTimer()
            for _ in range(reps):
                et.record(lambda: cm.cost_volume_forward(cam, proj, D, k, lay, "fast", out=out))
            res[mode].append(et.mean_ms())
            assert torch.equal(out, ref), "split and single-stream volumes differ"
    nb = out.numel() * 4 + 2 * H * W * cam.element_size()
    print(json.dumps({"cfg": name, "split_ms": [round(x, 4) for x in res["1"]],
                      "single_ms": [round(x, 4) for x in res["0"]],
                      "split_median": round(statistics.median(res["1"]), 4),
                      "single_median": round(statistics.median(res["0"]), 4),
                      "single_frac_of_8TBps": round(nb / statistics.median(res["0"]) / 1e6 / 8000, 4)}), flush=True)
    del out, ref
    torch.cuda.empty_cache()
