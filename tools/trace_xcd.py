"""Per-launch, per-XCD contract times and shader clocks from trace-variant stamps (tools/micro/trace_variant.sh,
tools/kprof_step.py --trace-timed OUT.npy): 16 slots of 256 workgroups, one slot per traced launch; per workgroup
[0] s_memrealtime at start, [1] XCC id, [2 .. 35] s_memrealtime at the end of each contract, [36] / [37] s_memtime
at start / end (shader-clock cycles), [38] contracts, [39] s_memrealtime at the end (100 MHz).

    python tools/trace_xcd.py FILE.npy [FILE.npy ...]
"""
import sys

import numpy as np

US = 1 / 100.0  # s_memrealtime ticks at 100 MHz


def main() -> None:
    for fn in sys.argv[1:]:
        b = np.load(fn).astype(np.int64)
        print(f"# {fn}: slot, workgroups, contracts, start / end (us from the first start), mean contract time (us) on "
              "the even / odd XCDs, shader clock (MHz) even / odd")
        rows = [b[k * 256:(k + 1) * 256] for k in range(16)]
        used = [(k, t[(t[:, 39] > 0) & (t[:, 38] > 0)]) for k, t in enumerate(rows)]
        used = [(k, t) for k, t in used if len(t)]
        t0 = min(t[:, 0].min() for _, t in used)
        for k, t in used:
            dur = (t[:, 39] - t[:, 0]) * US
            mhz = (t[:, 37] - t[:, 36]) / dur
            x = t[:, 1]
            d, xs = [], []
            for row in t:
                n = min(int(row[38]), 34)
                st = np.concatenate([[row[0]], row[2:2 + n]])
                d.append(np.diff(st) * US)
                xs += [int(row[1])] * n
            d, xs = np.concatenate(d), np.array(xs)
            print(f"slot {k:2d}: {len(t):3d} WGs {int(t[:, 38].sum()):5d} contracts  start {(t[:, 0].min() - t0) * US:8.0f}.."
                  f"{(t[:, 0].max() - t0) * US:8.0f}  end {(t[:, 39].max() - t0) * US:8.0f}  contract even "
                  f"{d[xs % 2 == 0].mean():6.1f} odd {d[xs % 2 == 1].mean():6.1f}  clock even {mhz[x % 2 == 0].mean():6.0f} "
                  f"odd {mhz[x % 2 == 1].mean():6.0f}")


if __name__ == "__main__":
    main()
