"""Summarise a per-workgroup timestamp trace of resident_kernel (SMC_EXPERIMENT_TRACE builds,
tools/kprof_step.py --trace / tools/kprof.py --trace): per-XCD finish times, the idle tail of the
launch (CU-time between a workgroup's last contract and the launch end), and per-contract phase times.

    python tools/trace_summary.py gpurun_out/trace_c2_step.npy [--grid 256]

Slots (gbm.hip SMC_TRACE): 0 kernel start, 1 XCC id, 2 + 2r simulation of round r done, 3 + 2r its
CF done (rounds < 18), 39 workgroup end; with --cf (SMC_EXPERIMENT_TRACE_CF) 2 + 6 r + k, k = 0 simulation
done, 1 column sums in LDS, 2 M-mean done, 3 FFT done (rounds < 6).  s_memrealtime ticks at 100 MHz.
"""
import argparse

import numpy as np


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--grid", type=int, default=256)
    ap.add_argument("--cf", action="store_true", help="SMC_EXPERIMENT_TRACE_CF build: CF sub-steps of rounds 0..5")
    a = ap.parse_args()
    t = np.load(a.trace)[: a.grid].astype(np.int64)
    us = 0.01  # 100 MHz
    t0 = t[:, 0].min()
    start = (t[:, 0] - t0) * us
    end = (t[:, 39] - t0) * us
    span = end.max()
    xcc = t[:, 1]
    print(f"launch span {span:.1f} us, workgroup starts {start.min():.1f}..{start.max():.1f} us")
    idle = span - end
    print(f"tail: workgroup ends {end.min():.1f}..{end.max():.1f} us, mean idle {idle.mean():.1f} us "
          f"({idle.mean() / span:.2%} of the CU-time)")
    for x in sorted(set(xcc.tolist())):
        m = xcc == x
        print(f"  XCC {x}: {m.sum()} WGs, end {end[m].min():.1f}..{end[m].max():.1f} us")
    if a.cf:
        ghz = (t[:, 37] - t[:, 36]) / ((t[:, 39] - t[:, 0]) * 10.0)  # s_memtime cycles / ns
        for x in sorted(set(xcc.tolist())):
            m = xcc == x
            print(f"  XCC {x}: mean core clock {ghz[m].mean():.3f} GHz (min {ghz[m].min():.3f})")
        prev = t[:, 0]
        for r in range(6):
            k = [t[:, 2 + 6 * r + i] for i in range(4)]
            d = [(k[0] - prev) * us] + [(k[i] - k[i - 1]) * us for i in range(1, 4)]
            print(f"  round {r}: sim {d[0].mean():6.1f} us  payoff+colsum {d[1].mean():5.2f}  "
                  f"M-mean {d[2].mean():5.2f}  FFT+targets {d[3].mean():5.2f} us (max {d[1].max():.2f} "
                  f"{d[2].max():.2f} {d[3].max():.2f})")
            prev = k[3]
        return
    rounds = []
    prev = t[:, 0]
    for r in range(18):
        sim, cf = t[:, 2 + 2 * r], t[:, 3 + 2 * r]
        ok = (sim > 0) & (cf > 0)
        if not ok.any():
            break
        rounds.append(r)
        s = (sim[ok] - prev[ok]) * us
        c = (cf[ok] - sim[ok]) * us
        print(f"  round {r:2d}: {ok.sum():3d} WGs  sim {s.mean():7.1f} us (min {s.min():.1f} max {s.max():.1f})"
              f"  cf {c.mean():5.1f} us (max {c.max():.1f})")
        prev = np.where(ok, cf, prev)
    n = np.array([sum(1 for r in rounds if t[w, 3 + 2 * r] > 0) for w in range(len(t))])
    print(f"contracts per WG: {np.bincount(n)}")


if __name__ == "__main__":
    main()
