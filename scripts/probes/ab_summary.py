#!/usr/bin/env python3
"""One line per steady_ab.py result: config, and per arm median ms / frac / bit-exact."""
import json
import sys

for fn in sys.argv[1:]:
    for line in open(fn):
        if line.startswith("{"):
            d = json.loads(line)
            arms = ", ".join("%s %.4f ms %.3f%s" % (k, v["median_ms"], v["frac_median"], "" if v["bit_exact_frame0"] else " MISMATCH")
                             for k, v in d["arms"].items())
            print("%-4s %s" % (d["config"], arms))
