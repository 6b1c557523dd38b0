import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np
import oracle_lib as ol
exe = os.path.join(ROOT, "libiqo_amd", "build", "iqo_benchmark")
for m, iw, ih, ow, oh in [("lanczos2", 640, 480, 320, 240), ("lanczos3", 3840, 2160, 1920, 1080), ("area", 7680, 4320, 1920, 1080), ("linear", 1920, 1080, 3840, 2160)]:
    for extra in ([], ["-reuse", "1"]):
        r = subprocess.run([exe, "-m", m, "-iw", str(iw), "-ih", str(ih), "-ow", str(ow), "-oh", str(oh), "-cycles", "2", "-check", "/tmp/y.raw"] + extra, capture_output=True, text=True)
        got = np.fromfile("/tmp/y.raw", dtype=np.uint8).reshape(oh, ow)
        method = "lanczos" if m.startswith("lanczos") else m
        exp = ol.run_oracle(method, int(m[7]) if method == "lanczos" else 0, iw, ih, ow, oh, 1, ol.gen("mt19937", iw, ih))
        bad = np.argwhere(got != exp)
        print(m, extra, r.returncode, "mismatch", len(bad), "rows", sorted(set(bad[:, 0].tolist()))[:10] if len(bad) else [], "cols", sorted(set(bad[:, 1].tolist()))[:10] if len(bad) else [], r.stdout.strip().splitlines()[-1])
