"""Build benchmarking variants of the HIP library into scripts/_abl/<name>/ (git-ignored);
load one with CUSTMA_LIB=scripts/_abl/<name>/libcustma_hip.so.
Usage: python scripts/build_ablations.py <name> [...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from custereomatching_amd.build import build_variant  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
FWD = ["sweep_wave.hip", "sweep_fwd.hip"]
BWD = ["bwd_fused.hip"]
# name: (defines, translation units they affect)
VARIANTS = {
    # forward ablations (sweep_wave.hip / sweep_fwd.hip)
    "nostore": (["CUSTMA_ABL_NOSTORE"], FWD), "noupdate": (["CUSTMA_ABL_NOUPDATE"], FWD),
    "storeonly": (["CUSTMA_ABL_NOUPDATE", "CUSTMA_ABL_NOOUT"], FWD),
    "nowait": (["CUSTMA_ABL_NOWAIT"], FWD),
    "nostatsmem": (["CUSTMA_ABL_NOSTATSMEM"], FWD), "noimgmem": (["CUSTMA_ABL_NOIMGMEM"], FWD),
    "noldmem": (["CUSTMA_ABL_NOSTATSMEM", "CUSTMA_ABL_NOIMGMEM"], FWD), "nocammem": (["CUSTMA_ABL_NOCAMMEM"], FWD), "stats7": (["CUSTMA_ABL_STATS7"], FWD),
    "early": (["CUSTMA_TILE_EARLY"], FWD), "tileP3": (["CUSTMA_TILE_P=3"], FWD),
    # volume-store cache policy (gfx950 aux bits: 1 sc0, 2 nt, 16 sc1)
    "st_plain": (["CUSTMA_STORE_AUX=0"], FWD), "st_sc1": (["CUSTMA_STORE_AUX=16"], FWD),
    "st_ntsc1": (["CUSTMA_STORE_AUX=18"], FWD),
    # backward unit height / block order (bwd_fused.hip)
    "r32": (["CUSTMA_BWD_ROWS=32"], BWD),  # block order: CUSTMA_BWD_ORDER=1|2 at run time
    # backward LDS: single A buffer + 4-step flushes (k = 11: 61 -> 52 KB, 3 workgroups per CU)
    "ab1": (["CUSTMA_BWD_ABUF=1", "CUSTMA_BWD_FBC=4"], BWD),
    "ab1f8": (["CUSTMA_BWD_ABUF=1"], BWD),
    # backward loads two steps ahead (sliding columns kept)
    "bdp2": (["CUSTMA_BWD_DEPTH=2"], BWD),
    "bwdnomem": (["CUSTMA_ABL_BWD_NOMEM"], BWD),  # timing only: gradient / volume loads out of range
    # knockouts (timing only, wrong results): no lane reductions / no column slide / no halo A rows
    "ko_red": (["CUSTMA_ABL_KO_RED"], BWD), "ko_slide": (["CUSTMA_ABL_KO_SLIDE"], BWD),
    "ko_halo": (["CUSTMA_ABL_KO_HALO"], BWD), "ko_bar": (["CUSTMA_ABL_KO_BAR"], BWD),
    "ko_col": (["CUSTMA_ABL_KO_COL"], BWD),
    "ko_nomem_bar": (["CUSTMA_ABL_BWD_NOMEM", "CUSTMA_ABL_KO_BAR"], BWD),
    "ko_all": (["CUSTMA_ABL_BWD_NOMEM", "CUSTMA_ABL_KO_BAR", "CUSTMA_ABL_KO_RED", "CUSTMA_ABL_KO_SLIDE"], BWD),
    "bdp2ab1": (["CUSTMA_BWD_DEPTH=2", "CUSTMA_BWD_ABUF=1", "CUSTMA_BWD_FBC=6"], BWD),
    # backward segment width (columns per unit)
    "seg128": (["CUSTMA_BWD_SEG=128"], BWD), "seg256": (["CUSTMA_BWD_SEG=256"], BWD),
    # backward without the window layout's SGPR-offset load path
    "nowin": (["CUSTMA_BWD_NOWIN"], BWD),
    "fbc8": (["CUSTMA_BWD_FBC=8"], BWD),
    "acc64": (["CUSTMA_BWD_ACC64"], BWD),
    "wait0vseq": (["CUSTMA_BWD_WAIT0", "CUSTMA_BWD_VSEQ"], BWD),
    "noslp": (["-fno-slp-vectorize"], BWD + ["stats.hip"]),  # no packed-fp32 pairing by the compiler
    "gather1": (["CUSTMA_BWD_GATHER1"], BWD),
    "camlall": (["CUSTMA_BWD_CAMLDS_ALL"], BWD), "caml0": (["CUSTMA_BWD_CAMLDS=0"], BWD),
    # statistics tile: 32 x 32 pixels, 4 rows per thread is the default (profiles/r03/stats)
    "stats32x8": (["CUSTMA_STATS_TX=32", "CUSTMA_STATS_PR=8"], ["stats.hip"]),
    "stats16x8": (["CUSTMA_STATS_TX=16", "CUSTMA_STATS_PR=8"], ["stats.hip"]),
    "stats32x4": (["CUSTMA_STATS_TX=32", "CUSTMA_STATS_PR=4"], ["stats.hip"]),
    "stats64x2": (["CUSTMA_STATS_TX=64", "CUSTMA_STATS_PR=2"], ["stats.hip"]),
    "stats16x2": (["CUSTMA_STATS_TX=16", "CUSTMA_STATS_PR=2"], ["stats.hip"]),  # the per-pixel slot gather + 16x16 three-map combine  # round-3 step waits / vertical sum before  # fp64 per-pixel sums between gather and combine
}
for n in (sys.argv[1:] or VARIANTS):
    d, only = VARIANTS[n]
    print(build_variant(os.path.join(HERE, "_abl", n), d, only))
