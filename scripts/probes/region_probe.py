"""C2 128-frame launch time at each 128-frame region of one large allocation (torch), and of
separate 128-frame allocations, interleaved, to see whether the cost follows the memory region."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import libiqo_amd as L

SW, SH, DW, DH = 3840, 2160, 1920, 1080
FS, FD = SW * SH, DW * DH
r = L.LanczosResizer(3, SW, SH, DW, DH, device=0)
s = torch.cuda.current_stream()

def t(src, dst, frames, reps=10):
    for _ in range(2):
        r.resize_device(frames, SW, FS, src, DW, FD, dst, stream=s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        r.resize_device(frames, SW, FS, src, DW, FD, dst, stream=s)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
src = torch.randint(0, 256, (N * FS,), dtype=torch.uint8, device="cuda")
dst = torch.empty(N * FD, dtype=torch.uint8, device="cuda")
small = [(torch.randint(0, 256, (128 * FS,), dtype=torch.uint8, device="cuda"),
          torch.empty(128 * FD, dtype=torch.uint8, device="cuda")) for _ in range(2)]
for rep in range(2):
    row = []
    for k in range(N // 128):
        row.append(t(src.data_ptr() + k * 128 * FS, dst.data_ptr() + k * 128 * FD, 128))
    print("rep %d  big-alloc 128-frame regions: %s" % (rep, " ".join("%.4f" % x for x in row)), flush=True)
    print("rep %d  separate 128-frame allocs: %s" % (rep, " ".join("%.4f" % t(a.data_ptr(), b.data_ptr(), 128) for a, b in small)), flush=True)
    for n in (256, 512, N):
        print("rep %d  one launch of %d frames at offset 0: %.4f ms (%.6f /frame)" % (rep, n, t(src.data_ptr(), dst.data_ptr(), n, 5), t(src.data_ptr(), dst.data_ptr(), n, 5) / n), flush=True)
    # second half of the 256 frames alone
    print("rep %d  frames 128..255 alone: %.4f; dst swapped regions (src k=0, dst k=1): %.4f" % (
        rep, t(src.data_ptr() + 128 * FS, dst.data_ptr() + 128 * FD, 128), t(src.data_ptr(), dst.data_ptr() + 128 * FD, 128)), flush=True)
