"""Clock / power probe (diagnostic): per-launch HIP-event times of the C3 window forward, back to back
and after idle gaps, with the GPU's reported clocks / power sampled around them."""
import json, os, subprocess, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import custereomatching_amd as cm
from bench import synth_pair


def smi():
    try:
        r = subprocess.run(["amd-smi", "metric", "-g", "0", "-p", "-c", "--json"], capture_output=True, text=True,
                           timeout=20)
        return r.stdout[-1500:]
    except Exception as e:  # noqa: BLE001
        return str(e)


def main():
    H, W, D, k = 2048, 2048, 256, 11
    cam, proj = synth_pair(H, W, D, 5, "cuda", torch.float16)
    out = cm.cost_volume_forward(cam, proj, D, k, "window")
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(64)]

    def burst(n):
        for i in range(n):
            ev[i][0].record()
            cm.cost_volume_forward(cam, proj, D, k, "window", out=out)
            ev[i][1].record()
        torch.cuda.synchronize()
        return [round(a.elapsed_time(b), 3) for a, b in ev[:n]]

    print("idle smi:", smi(), flush=True)
    print("burst40:", burst(40), flush=True)
    print("hot smi:", smi(), flush=True)
    for gap in (0.05, 0.2, 1.0, 3.0):
        time.sleep(gap)
        print(f"after {gap}s idle:", burst(4), flush=True)


if __name__ == "__main__":
    main()
