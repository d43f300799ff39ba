"""Round-5 records: from gpurun_out/final5 (tools/micro/r05_final.sh) write profiles/r05/final/ -- per config the
bench line, the rocprofv3 kernel stats of the same bench command, the stats and per-dispatch durations of the
dominant launch alone (kprof) -- and profiles/r05/records.md, a table that checks each line's kernel_ms against
the isolated launches' rocprof average (dispatches 2 .. 1 + kernel_iters: the bench times kernel_iters launches
after one warm-up launch, and the first dispatch of a fresh process runs cold).

    python tools/r05_records.py [--src gpurun_out/final5]
"""
import argparse
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("resident_kernel", "wave_kernel", "packed_kernel", "basket_resident_kernel", "rows_kernel", "cf_kernel")


def dispatches(trace: str, names: tuple[str, ...]) -> list[tuple[str, float]]:
    with open(trace) as f:
        rows = list(csv.DictReader(f))
    out = []
    for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
        n = r["Kernel_Name"]
        if any(k in n for k in names):
            out.append((n, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out", "final5"))
    ap.add_argument("--dst", default=os.path.join(ROOT, "profiles", "r05"))
    a = ap.parse_args()
    final = os.path.join(a.dst, "final")
    os.makedirs(final, exist_ok=True)
    lines = ["# Round-5 closing records (tools/micro/r05_final.sh on one MI355X; tools/r05_records.py)", "",
             "`kernel_ms` is the bench's own timing of the dominant launch (HIP events around `kernel_iters` = 10",
             "back-to-back launches on one stream after one warm-up launch); `iso rocprof` is the rocprofv3 kernel",
             "trace of the same launch shape alone (`iso_<cfg>_kernel_stats.csv`, `iso_<cfg>_dispatches.txt`),",
             "averaged over dispatches 2 .. 11 as the bench times them.  The path launches change speed with the",
             "chip's clock, which the power limiter moves under the store stream (C2 launch 1.3-2.0 GHz,",
             "`pmc_c2_clock.txt`), so back-to-back launches drift by a few %.", "",
             "| config | ms/step | kernel (line) | kernel_ms | iso rocprof (2..11) | agree | frac | bench-command rocprof avg "
             "(all dispatches, overlapped ones from dispatch to end) |",
             "|---|---|---|---|---|---|---|---|"]
    for cfg in ("c2", "c2h256", "c3", "c5", "lockstep", "e2e", "c2f64"):
        bench = os.path.join(a.src, f"bench_{cfg}.out")
        if not os.path.exists(bench):
            continue
        text = open(bench).read().strip().splitlines()[-1]
        d = json.loads(text)
        with open(os.path.join(final, f"bench_{cfg}.json"), "w") as f:
            f.write(text + "\n")
        r = d["roofline"]
        kern = r["kernel"].split("(")[0].split("+")[0]
        iso_avg, bench_avg = None, None
        for tag in ("iso", "prof"):
            st = glob.glob(os.path.join(a.src, f"{tag}_{cfg}", "**", "*kernel_stats.csv"), recursive=True)
            tr = glob.glob(os.path.join(a.src, f"{tag}_{cfg}", "**", "*kernel_trace.csv"), recursive=True)
            if st:
                shutil.copy(st[0], os.path.join(final, f"{tag}_{cfg}_kernel_stats.csv"))
                with open(st[0]) as f:
                    for row in csv.DictReader(f):
                        if kern in row["Name"] and tag == "prof" and bench_avg is None:
                            bench_avg = float(row["AverageNs"]) / 1e6
            if tr:
                ds = dispatches(tr[0], (kern,))
                if tag == "iso" and ds:
                    with open(os.path.join(final, f"iso_{cfg}_dispatches.txt"), "w") as f:
                        f.write(f"# {kern}: per-dispatch durations (ms) of tools/kprof_* alone\n")
                        for n, ms in ds:
                            f.write(f"{ms:.4f}  {n[:90]}\n")
                    sel = ds[1:11] if len(ds) > 2 else ds
                    iso_avg = sum(ms for _, ms in sel) / len(sel)
        agree = f"{(r['kernel_ms'] / iso_avg - 1) * 100:+.1f} %" if iso_avg else "-"
        lines.append(f"| {cfg} | {d['ms_per_step']:.4f} | `{r['kernel']}` | {r['kernel_ms']:.4f} | "
                     f"{iso_avg:.4f} | {agree} | {r['frac']:.4f} | {bench_avg:.4f} |" if iso_avg and bench_avg else
                     f"| {cfg} | {d['ms_per_step']:.4f} | `{r['kernel']}` | {r['kernel_ms']:.4f} | - | - | {r['frac']:.4f} | - |")
    # PMC: C2 traffic per launch and the clock under the launches
    for name in ("pmc_c2_WRITE_SIZE", "pmc_c2_FETCH_SIZE", "pmc_c2_clock", "pmc_c2f64_clock"):
        cc = glob.glob(os.path.join(a.src, name, "**", "*counter_collection.csv"), recursive=True)
        if cc:
            shutil.copy(cc[0], os.path.join(final, f"{name}_counter_collection.csv"))
    lines += ["", "PMC over the C2 launch (`final/pmc_c2_*_counter_collection.csv`): see `pmc_c2_traffic.txt` and "
              "`pmc_c2_clock.txt` (tools/pmc_summary.py, tools/pmc_clock.py)."]
    with open(os.path.join(a.dst, "records.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
