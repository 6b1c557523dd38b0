#!/usr/bin/env python3
"""List the kernels whose ISA touches scratch (register spills or a dynamically indexed register
array).  Run after `make -C libiqo_amd asm`:  python scripts/check_scratch.py
Round 5 found the 2x/3x Lanczos streamer 2-3x slower because one select of two window rows let
the compiler move the whole register window to scratch; this makes such regressions visible."""
import re
import sys

ASMS = sys.argv[1:] or ["libiqo_amd/build/%s-hip-amdgcn-amd-amdhsa-gfx950.s" % k for k in ("kernels", "kernels_ratio")]
cur, counts = None, {}
for line in (ln for f in ASMS for ln in open(f)):
    m = re.match(r"^(_Z\S+):", line)
    if m:
        cur = m.group(1)
        counts.setdefault(cur, [0, 0])
        continue
    if cur and "scratch_load" in line:
        counts[cur][0] += 1
    elif cur and "scratch_store" in line:
        counts[cur][1] += 1
bad = {k: v for k, v in counts.items() if v[0] or v[1]}
for k, (ld, st) in sorted(bad.items()):
    print("%4d loads %4d stores  %s" % (ld, st, k))
print("%d of %d kernels touch scratch" % (len(bad), len(counts)))
