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




def rate_custom(nbytes: int, x: float, vec: int, reps: int = 5) -> float:
    """tools/micro/fillcmp.hip's linear one-shot store kernel on a torch buffer (value x, vec dwordx4 per lane)."""
    import ctypes
    import os
    lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "micro", "v", "libfillcmp.so"))
    lib.fillcmp_lin.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_float, ctypes.c_int, ctypes.c_void_p]
    buf = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    n = buf.numel() // (1024 * vec) * (1024 * vec)
    lib.fillcmp_lin(buf.data_ptr(), n, x, vec, s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        lib.fillcmp_lin(buf.data_ptr(), n, x, vec, s)
    e1.record()
    e1.synchronize()
    del buf
    torch.cuda.empty_cache()
    return n * 4 * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9


def compare() -> None:
    c2 = 4096 * 16 * 66048 * 4
    for x in (0.0, 2.0, 1.2345678):
        print(f"torch fill_({x}) {c2 / 1e9:.2f} GB: ", end="")
        buf = torch.empty(c2 // 4, dtype=torch.float32, device="cuda")
        buf.fill_(x)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            buf.fill_(x)
        e1.record()
        e1.synchronize()
        print(f"{c2 * 5 / (e0.elapsed_time(e1) * 1e-3) / 1e9:7.1f} GB/s", flush=True)
        del buf
        torch.cuda.empty_cache()
        for vec in (1, 4, 16):
            print(f"  fillcmp lin x={x} vec={vec}: {rate_custom(c2, x, vec):7.1f} GB/s", flush=True)


if __name__ == "__main__":
    import sys
    if "--compare" in sys.argv:
        compare()
    else:
        c2 = 4096 * 16 * 66048 * 4  # the C2 path matrix at its padded pitch (17.3 GB)
        for n in (1 << 30, 4 << 30, 8 << 30, 12 << 30, c2, 2 * c2, 64 << 30):
            print(f"fill_ {n / 1e9:7.2f} GB: {rate(n):7.1f} GB/s", flush=True)
