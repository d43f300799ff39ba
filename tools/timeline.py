"""Kernel timeline of a rocprofv3 --kernel-trace CSV (…_kernel_trace.csv): every kernel from the
`--skip`-th launch of `--anchor` on, relative to that launch's start, with its queue and stream, plus the
spacing of consecutive anchor launches (their overlap when negative).

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -- python3 bench.py --steps 10 ...
    python tools/timeline.py gpurun_out/tl/.../..._kernel_trace.csv [--anchor resident_kernel] [--rows 40]
"""
import argparse
import csv


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--anchor", default="resident_kernel")
    ap.add_argument("--skip", type=int, default=4, help="anchor launches to skip (warm-up)")
    ap.add_argument("--rows", type=int, default=40)
    a = ap.parse_args()
    with open(a.csv) as f:
        rows = list(csv.DictReader(f))
    key = lambda *names: next(k for k in rows[0] if any(n.lower() == k.lower() for n in names))
    kn, ks, ke = key("Kernel_Name"), key("Start_Timestamp"), key("End_Timestamp")
    kq = next((k for k in rows[0] if k.lower() in ("queue_id",)), None)
    kst = next((k for k in rows[0] if k.lower() in ("stream_id",)), None)
    ev = sorted(((int(r[ks]), int(r[ke]), r[kn], r.get(kq, "") if kq else "", r.get(kst, "") if kst else "")
                 for r in rows), key=lambda e: e[0])
    anchors = [e for e in ev if a.anchor in e[2]]
    if len(anchors) <= a.skip:
        raise SystemExit(f"only {len(anchors)} {a.anchor} launches")
    t0 = anchors[a.skip][0]
    print("# start_ms end_ms dur_ms queue stream kernel (relative to an anchor launch's start)")
    n = 0
    for s, e, name, q, st in ev:
        if s < t0 - 50_000:
            continue
        print(f"{(s - t0) / 1e6:9.3f} {(e - t0) / 1e6:9.3f} {(e - s) / 1e6:7.3f} q{q} s{st} {name[:80]}")
        n += 1
        if n >= a.rows:
            break
    sp = [(anchors[i + 1][0] - anchors[i][0]) / 1e6 for i in range(a.skip, len(anchors) - 1)]
    ov = [(anchors[i + 1][0] - anchors[i][1]) / 1e6 for i in range(a.skip, len(anchors) - 1)]
    du = [(x[1] - x[0]) / 1e6 for x in anchors[a.skip:]]
    if sp:
        print(f"# {a.anchor}: {len(du)} launches, duration avg {sum(du) / len(du):.4f} ms, start-to-start avg "
              f"{sum(sp) / len(sp):.4f} ms, next start - end avg {sum(ov) / len(ov) * 1e3:.1f} us")


if __name__ == "__main__":
    main()
