"""Debug helper: run shapes on the GPU (fast and general paths) and report where outputs differ
from the oracle (rows / columns / counts)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

import libiqo_amd  # noqa: E402
import oracle_lib as ol  # noqa: E402

SHAPES = [("lanczos", 2, 640, 480, 320, 240, 1), ("lanczos", 3, 3840, 2160, 1920, 1080, 1),
          ("lanczos", 3, 384, 216, 192, 108, 1)]
for shp in SHAPES:
    m, d, sw, sh, dw, dh, px = shp
    src = ol.gen("g1", sw, sh)
    exp = ol.run_oracle(m, d, sw, sh, dw, dh, px, src)
    for fg in (0, 1):
        r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
        r.set_option("force_general", fg)
        out = np.zeros((dh, dw), np.uint8)
        r.resize(sw, src, dw, out)
        bad = np.argwhere(out != exp)
        rows = sorted(set(bad[:, 0].tolist())) if bad.size else []
        cols = sorted(set(bad[:, 1].tolist())) if bad.size else []
        print(shp, "general" if fg else r.describe()["kernel"], "mismatches", len(bad),
              "rows", rows[:12], len(rows), "cols", cols[:12], len(cols))
        if bad.size:
            y, x = bad[0]
            print("  first", (int(y), int(x)), "got", int(out[y, x]), "exp", int(exp[y, x]))
