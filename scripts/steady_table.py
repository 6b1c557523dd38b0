#!/usr/bin/env python3
"""Markdown rows (config, kernel, frames, ms per launch, frac) from a bench_lines jsonl file
(scripts/gpu_ci.sh benchlines), for DESIGN.md's steady-clock table.
  python scripts/steady_table.py profiles/r05/bench_lines_final.jsonl"""
import json
import sys

for line in open(sys.argv[1]):
    d = json.loads(line)
    r = d["roofline"]
    label = d["config"]["workload"]
    print("| %s | `%s` | %d | %.4f | %.3f%s |" % (label, d["config"].get("kernel", "?"), d["config"]["frames_per_gpu"],
                                              r["kernel_ms_per_launch"], r["frac"],
                                              "" if "bit-exact" in d.get("parity", "") else " NOT BIT-EXACT"))
