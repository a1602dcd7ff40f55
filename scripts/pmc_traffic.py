"""HBM traffic per launch of the two sweep kernels from rocprofv3 PMC passes (GPU box).

Runs the calibration micro-benchmark and the bench workload under separate
`rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes (never combined with tracing),
derives bytes-per-KB factors for this repo's access shape (one dword per lane) from the
calibration, and writes profiles/pmc_<kernel>_c2_<layout>.json.
Usage: python scripts/pmc_traffic.py <outdir> [layout]
"""
import csv, glob, json, os, subprocess, sys

out = sys.argv[1]
layout = sys.argv[2] if len(sys.argv) > 2 else "full"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.makedirs(out, exist_ok=True)
env = dict(os.environ, TMPDIR="/tmp")


def run(counter, tag, cmd):
    d = os.path.join(out, f"{tag}_{counter}")
    r = subprocess.run(["timeout", "-k", "10", "300", "rocprofv3", "--pmc", counter, "-d", d, "-o", "run",
                        "--output-format", "csv", "--"] + cmd, cwd=root, env=env, capture_output=True, text=True)
    if r.returncode != 0:
        print(r.stdout[-2000:], r.stderr[-2000:])
        raise SystemExit(f"rocprofv3 {counter} {tag} failed")
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            vals.setdefault(row["Kernel_Name"], []).append(float(row["Counter_Value"]))
    return vals


def mean_of(vals, key):
    v = [x for name, xs in vals.items() if key in name for x in xs]
    return sum(v) / len(v) if v else None


calib = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    calib[c] = run(c, "calib", ["./scripts/micro/fetch_calib"])
GiB = float(1 << 30)
f_rd1 = GiB / (mean_of(calib["FETCH_SIZE"], "rd1") or 1)   # bytes per FETCH_SIZE unit, dword loads
f_rd4 = GiB / (mean_of(calib["FETCH_SIZE"], "rd4") or 1)
f_wr1 = GiB / (mean_of(calib["WRITE_SIZE"], "wr1") or 1)
print(f"calibration: FETCH bytes/unit dword={f_rd1:.1f} x4={f_rd4:.1f}; WRITE bytes/unit dword={f_wr1:.1f}")

bench = ["python3", "bench.py", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-north-star",
         "--layout", layout]
meas = {c: run(c, "bench", bench) for c in ("FETCH_SIZE", "WRITE_SIZE")}
for kern in ("k_bwd_coop", "k_sweep_fwd", "k_fwd_wave"):
    fs, ws = mean_of(meas["FETCH_SIZE"], kern), mean_of(meas["WRITE_SIZE"], kern)
    if fs is None or ws is None:
        continue
    rd, wr = fs * f_rd1, ws * f_wr1
    res = {"kernel": kern, "workload": f"bench.py default (1024x1024 fp32, k=9, {layout})",
           "FETCH_SIZE_mean": fs, "WRITE_SIZE_mean": ws,
           "calibration": {"fetch_bytes_per_unit_dword_loads": f_rd1, "fetch_bytes_per_unit_16B_loads": f_rd4,
                           "write_bytes_per_unit_dword_stores": f_wr1,
                           "source": "scripts/micro/fetch_calib.hip, 1 GiB streamed per kernel"},
           "read_bytes_per_launch": rd, "write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
           "note": "fabric-side request counters (TCC_EA0): Infinity-Cache hits are counted as well"}
    p = os.path.join(out, f"pmc_{kern}_c2_{layout}.json")  # copied into profiles/ by hand
    json.dump(res, open(p, "w"), indent=1)
    print(kern, json.dumps(res))
