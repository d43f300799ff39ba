"""Write rate of torch's fill_ (a linear store sweep) against the buffer size: is the ~6 TB/s the C2
path launch reaches the rate the chip writes a buffer of its path matrix's size at?
    python tools/probe_fill.py"""
import torch


def rate(nbytes: int, reps: int = 5) -> float:
    buf = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
    buf.fill_(1.0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        buf.fill_(2.0)
    e1.record()
    e1.synchronize()
    del buf
    torch.cuda.empty_cache()
    return nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9


if __name__ == "__main__":
    c2 = 4096 * 16 * 66048 * 4  # the C2 path matrix at its padded pitch (17.3 GB)
    for n in (1 << 30, 4 << 30, 8 << 30, 12 << 30, c2, 2 * c2, 64 << 30):
        print(f"fill_ {n / 1e9:7.2f} GB: {rate(n):7.1f} GB/s", flush=True)
