"""Debug: where the tile kernel differs from the oracle (row/column pattern) for one shape."""
import sys
import numpy as np
import torch
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import oracle_lib as ol
import libiqo_amd

m, d, sw, sh, dw, dh, px = sys.argv[1], int(sys.argv[2]), *map(int, sys.argv[3:8])
frame = ol.gen("g1", sw, sh, 0)
exp = ol.run_oracle(m, d, sw, sh, dw, dh, px, frame)
for tile in (1, 0):
    r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    r.set_option("tile", tile)
    out = r.resize_tensor(torch.from_numpy(frame).cuda()).cpu().numpy()
    bad = np.argwhere(out != exp)
    print("tile", tile, r.describe()["kernel"], "bad", len(bad))
    if len(bad):
        rows = np.unique(bad[:, 0]); cols = np.unique(bad[:, 1])
        print(" rows", rows[:20], len(rows), " cols", cols[:20], len(cols))
        for y, x in bad[:5]:
            print("  ", y, x, out[y, x], exp[y, x])
    host = np.zeros((dh, dw), np.uint8)
    r.resize(sw, frame, dw, host)
    print(" host path bad", int((host != exp).sum()))
