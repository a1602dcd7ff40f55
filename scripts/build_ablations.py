"""Build ablation variants of the HIP library into scripts/_abl/<name>/ (git-ignored)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from custereomatching_amd.build import build_variant
HERE = os.path.dirname(os.path.abspath(__file__))
VARIANTS = {"nostore": ["CUSTMA_ABL_NOSTORE"], "noupdate": ["CUSTMA_ABL_NOUPDATE"],
            "nothing": ["CUSTMA_ABL_NOSTORE", "CUSTMA_ABL_NOUPDATE"],
            "storeonly": ["CUSTMA_ABL_NOUPDATE", "CUSTMA_ABL_NOOUT"], "skeleton": ["CUSTMA_ABL_NOUPDATE", "CUSTMA_ABL_NOOUT", "CUSTMA_ABL_NOSTORE"],
            "aux1": ["CUSTMA_STORE_AUX=1"], "aux2": ["CUSTMA_STORE_AUX=2"], "aux16": ["CUSTMA_STORE_AUX=16"],
            "aux3": ["CUSTMA_STORE_AUX=3"], "aux17": ["CUSTMA_STORE_AUX=17"], "aux18": ["CUSTMA_STORE_AUX=18"],
            "aux19": ["CUSTMA_STORE_AUX=19"],
            "nowait": ["CUSTMA_ABL_NOWAIT"], "so_nowait": ["CUSTMA_ABL_NOUPDATE", "CUSTMA_ABL_NOOUT", "CUSTMA_ABL_NOWAIT"],
            "tilep2": ["CUSTMA_TILE_P=2"], "border0": ["CUSTMA_BWD_ORDER=0"], "stats7": ["CUSTMA_ABL_STATS7"],
            "so_stats7": ["CUSTMA_ABL_NOUPDATE", "CUSTMA_ABL_NOOUT", "CUSTMA_ABL_STATS7"],
            "bnoleave": ["CUSTMA_ABL_NOLEAVE"], "bnoimg": ["CUSTMA_ABL_NOIMG"], "bnored": ["CUSTMA_ABL_NORED"],
            "pf4": ["CUSTMA_BWD_PF=4"], "pf8": ["CUSTMA_BWD_PF=8"], "pf16": ["CUSTMA_BWD_PF=16"],
            "pf8noall": ["CUSTMA_BWD_PF=8", "CUSTMA_ABL_NOLEAVE", "CUSTMA_ABL_NOIMG", "CUSTMA_ABL_NORED"],
            "bnoall": ["CUSTMA_ABL_NOLEAVE", "CUSTMA_ABL_NOIMG", "CUSTMA_ABL_NORED"]}
for n in (sys.argv[1:] or VARIANTS):
    print(build_variant(os.path.join(HERE, "_abl", n), VARIANTS[n]))
