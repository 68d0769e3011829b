"""Streaming HBM rates on this MI355X for the pipeline's byte counts: a 0.8 GB
write-only fill (the splitter's output), a 0.8 -> 0.8 GB copy (the FFT's
traffic) and a 0.8 GB read-only reduction (the adder's input).  Prints GB/s
of algorithmic bytes per op, median of 10."""
import torch

n = 24500 * 4 * 32 * 32 * 2  # configs[1] subgrids, float32 words (0.80 GB)
a = torch.empty(n, dtype=torch.float32, device="cuda").normal_()
b = torch.empty_like(a)
out = torch.empty(1, dtype=torch.float32, device="cuda")


def rate(fn, nbytes, reps=10):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(
            enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    ms = ts[len(ts) // 2]
    return ms, nbytes / ms / 1e6


for name, fn, nbytes in (
        ("fill (write 0.8 GB)", lambda: b.fill_(0.0), 4 * n),
        ("copy (0.8 + 0.8 GB)", lambda: b.copy_(a), 8 * n),
        ("sum (read 0.8 GB)", lambda: out.copy_(a.sum()), 4 * n)):
    ms, gbs = rate(fn, nbytes)
    print(f"{name:22s} {ms:8.4f} ms {gbs:8.1f} GB/s", flush=True)
