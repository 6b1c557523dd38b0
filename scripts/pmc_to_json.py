#!/usr/bin/env python3
"""Turn the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of scripts/gpu_ci.sh (pmc) into
profiles/pmc_<cfg>.json, which bench.py reads for roofline.traffic.

HBM bytes per launch follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE counts exactly 1/2 of the bytes of a wide coalesced streaming read, so
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
The two counters come from separate passes (they do not fit one TCC pass); each is the median
over the profiled dispatches of the hot kernel.

  python scripts/pmc_to_json.py gpurun_out c2 c3 c4 [--round r01]
"""
import csv
import glob
import json
import os
import statistics
import sys

KERNELS = {"lanczos_stream": "lanczos_s", "area_int": "area_int_kernel",  # lanczos_s: symb / sym / stream
           "linear_up2": "linear_up2_kernel", "general": "general_kernel", "tile": "tile_kernel",
           "walk": "walk_kernel", "lanczos_up2": "lanczos_up2_kernel", "lanczos_d32": "lanczos_d32_kernel",
           "area_d32": "area_d32_kernel", "lanczos_d31": "lanczos_d31_kernel", "ryx": "ryx_kernel"}
BENCH = {"c2": ("lanczos_stream", 1024), "c3": ("area_int", 64), "c4": ("linear_up2", 256), "c1": ("lanczos_stream", 4096),
         "g1": ("lanczos_d32", 128), "g2": ("lanczos_up2", 32), "g3": ("area_d32", 128),
         "g4": ("lanczos_d31", 128), "g5": ("ryx", 256), "g6": ("area_int", 128),
         "h1": ("area_int", 128, "linear_d2_kernel"), "h2": ("ryx", 128), "h3": ("lanczos_stream", 128), "h4": ("lanczos_up2", 64),
         "h5": ("linear_up2", 64), "h6": ("ryx", 128),
         # round 6: the general-row kernels (upscale rows on ryu_kernel, 3..4:1 downscale rows on ryg_kernel)
         "u1": ("ryx", 256), "u2": ("ryg", 256, "ryu_kernel"), "u3": ("ryg", 256, "ryu_kernel"),
         "w6": ("ryg", 128, "ryg_kernel"), "w4": ("ryg", 128, "ryg_kernel"), "w1": ("ryg", 256, "ryg_kernel")}


def per_dispatch(dirname, counter, kname):
    files = glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter or kname not in row.get("Kernel_Name", ""):
                    continue
                d = row.get("Dispatch_Id") or row.get("Correlation_Id")
                vals[d] = vals.get(d, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    rnd = "r01"
    if "--round" in sys.argv:
        rnd = sys.argv[sys.argv.index("--round") + 1]
        args.remove(rnd)
    out_dir, cfgs = args[0], args[1:]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for c in cfgs:
        kernel, frames = BENCH[c][:2]
        kname = BENCH[c][2] if len(BENCH[c]) > 2 else KERNELS[kernel]  # (Linear 2:1 runs area_int's linear_d2_kernel)
        fetch = per_dispatch(os.path.join(out_dir, "pmc_fetch_" + c), "FETCH_SIZE", kname)
        write = per_dispatch(os.path.join(out_dir, "pmc_write_" + c), "WRITE_SIZE", kname)
        if not fetch or not write:
            print("%s: no counter rows for %s" % (c, kname))
            continue
        f_kib, w_kib = statistics.median(fetch), statistics.median(write)
        res = {"config": c, "kernel": kernel, "frames": frames, "round": rnd,
               "fetch_size_kib": f_kib, "write_size_kib": w_kib, "dispatches": [len(fetch), len(write)],
               "hbm_read_bytes_per_launch": int(2 * f_kib * 1024), "hbm_write_bytes_per_launch": int(w_kib * 1024),
               "hbm_bytes_per_launch": int((2 * f_kib + w_kib) * 1024),
               "correction": "read = 2 x FETCH_SIZE (gfx950 half-count), KiB -> bytes x1024"}
        with open(os.path.join(root, "profiles", "pmc_%s.json" % c), "w") as f:
            json.dump(res, f, indent=1)
        print(c, json.dumps(res))


if __name__ == "__main__":
    main()
