"""Is a repeated C2 launch over the SAME batch cheaper than over fresh data?  Per-launch HIP-event
times for: the same 128-frame region repeated; two regions alternating; the same region with a
512 MB scrub (torch fill, untimed) between launches; and 256-frame launches."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import libiqo_amd as L

SW, SH, DW, DH = 3840, 2160, 1920, 1080
FS, FD = SW * SH, DW * DH
cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
r = L.LanczosResizer(3, SW, SH, DW, DH, device=0)
s = torch.cuda.current_stream()
N = 512
src = torch.randint(0, 256, (N * FS,), dtype=torch.uint8, device="cuda")
dst = torch.empty(N * FD, dtype=torch.uint8, device="cuda")
scrub = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")

def launch(k, frames=128):
    r.resize_device(frames, SW, FS, src.data_ptr() + k * 128 * FS, DW, FD, dst.data_ptr() + k * 128 * FD, stream=s)

def run(seq, do_scrub=False, frames=128):
    ev = []
    for k in seq:
        if do_scrub:
            scrub.fill_(k & 255)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s); launch(k, frames); b.record(s)
        ev.append((a, b))
    torch.cuda.synchronize()
    t = [a.elapsed_time(b) for a, b in ev][2:]
    return sum(t) / len(t)

for rep in range(2):
    print("rep", rep, flush=True)
    print("  same region x12            %.4f" % run([0] * 12), flush=True)
    print("  alternating 2 regions      %.4f" % run([0, 1] * 6), flush=True)
    print("  cycling 4 regions          %.4f" % run([0, 1, 2, 3] * 3), flush=True)
    print("  same region, scrub between %.4f" % run([0] * 12, True), flush=True)
    print("  cycling 4, scrub between   %.4f" % run([0, 1, 2, 3] * 3, True), flush=True)
    print("  256-frame launches (per 128) same %.4f  alternating %.4f" % (run([0] * 8, frames=256) / 2, run([0, 2] * 4, frames=256) / 2), flush=True)
