"""Build benchmarking variants of the HIP library into scripts/_abl/<name>/ (git-ignored);
load one with CUSTMA_LIB=scripts/_abl/<name>/libcustma_hip.so.
Usage: python scripts/build_ablations.py <name> [...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from custereomatching_amd.build import build_variant  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
BWD = ["bwd_fused.hip"]
# name: (defines, translation units they affect)
VARIANTS = {
    # (CUSTMA_BWD_DEPTH=2, the backward's loads two steps ahead, profiles/r04/a/bwd_depth_ab.txt, no longer builds:
    # its waits are runtime choices, which vmcnt_check.py cannot prove -- 7000 flagged reads in round 6)
    # knock-out (timing only, wrong results): k_bwd_coop without its volume loads -- the most an in-sweep
    # recompute of the costs could save (profiles/r06/a)
    "ko_novol": (["CUSTMA_KO_NOVOL"], BWD),
    # without the chip-filling column segments of the backward sweep (profiles/r06/g, h)
    "no_tail": (["CUSTMA_NO_TAIL"], BWD),
    # the full-layout sweep's volume stores with the default cache policy instead of nt (profiles/r06/d)
    "sweep_plain": (["CUSTMA_SWEEP_AUX=0"], ["sweep_fwd.hip"]),
    # the full-layout sweep with its round-5 dword volume stores (profiles/r06/e)
    "sweep_dword": (["CUSTMA_SWEEP_NO_X4"], ["sweep_fwd.hip"]),
    # the full-layout sweep with 96 / 128-row bands (fewer K - 1 warm-up steps per output row)
    "sweep_th96": (["CUSTMA_SWEEP_TH=96"], ["sweep_fwd.hip"]),
    "sweep_th128": (["CUSTMA_SWEEP_TH=128"], ["sweep_fwd.hip"]),
    # the window tile forward / disparity with 32-row bands (the store pattern's best band, profiles/r06/d)
    "th32": (["CUSTMA_WAVE_TH=32"], ["sweep_wave_d"]),
}
# The round-1..3 ablation / knock-out builds (CUSTMA_ABL_*, rejected variants) were pruned from the
# product sources in round 4; their measurements stay in DESIGN.md and profiles/.
for n in (sys.argv[1:] or VARIANTS):
    d, only = VARIANTS[n]
    print(build_variant(os.path.join(HERE, "_abl", n), d, only))
