"""Debug: tile kernel with byte-aligned sources/destinations vs the oracle; prints mismatch pattern."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import libiqo_amd
import oracle_lib as ol

m, d, sw, sh, dw, dh = "lanczos", 3, 1920, 1080, 1280, 720
src = ol.gen("noise", sw, sh, 5)
exp = ol.run_oracle(m, d, sw, sh, dw, dh, 1, src)
r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, 1)
for off, pad in [(0, 0), (0, 1), (0, 2), (0, 3), (1, 0), (1, 3), (2, 0), (3, 0), (0, 4), (1, 4)]:
    sst = sw + pad
    sbuf = torch.zeros(sh * sst + 64, dtype=torch.uint8, device="cuda")
    sview = sbuf[off:off + sh * sst].view(sh, sst)
    sview[:, :sw] = torch.from_numpy(src).cuda()
    dbuf = torch.zeros(dh * dw, dtype=torch.uint8, device="cuda")
    r.resize_device(1, sst, sh * sst, sview.data_ptr(), dw, dh * dw, dbuf.data_ptr())
    got = dbuf.view(dh, dw).cpu().numpy()
    bad = np.argwhere(got != exp)
    print("off", off, "pad", pad, "bad", len(bad), bad[:6].tolist(), flush=True)
# detail for one failing layout
sst = sw + 1
sbuf = torch.zeros(sh * sst + 64, dtype=torch.uint8, device="cuda")
sview = sbuf[:sh * sst].view(sh, sst)
sview[:, :sw] = torch.from_numpy(src).cuda()
dbuf = torch.zeros(dh * dw, dtype=torch.uint8, device="cuda")
r.resize_device(1, sst, sh * sst, sview.data_ptr(), dw, dh * dw, dbuf.data_ptr())
got = dbuf.view(dh, dw).cpu().numpy()
bad = np.argwhere(got != exp)
rows = np.unique(bad[:, 0]); cols = np.unique(bad[:, 1])
print("rows", rows[:40].tolist(), len(rows), "cols", cols[:8].tolist(), len(cols))
