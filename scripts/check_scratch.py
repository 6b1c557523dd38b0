#!/usr/bin/env python3
"""List the kernels whose ISA touches scratch (register spills or a dynamically indexed register
array).  Run after `make -C libiqo_amd asm`:  python scripts/check_scratch.py
Round 5 found the 2x/3x Lanczos streamer 2-3x slower because one select of two window rows let
the compiler move the whole register window to scratch; this makes such regressions visible."""
import re
import sys

ASM = sys.argv[1] if len(sys.argv) > 1 else "libiqo_amd/build/kernels-hip-amdgcn-amd-amdhsa-gfx950.s"
cur, counts = None, {}
for line in open(ASM):
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
