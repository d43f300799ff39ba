"""Round-6 records: from gpurun_out/final6 (tools/micro/r06_final.sh) write profiles/r06/final/ -- per config the
bench line, the rocprofv3 kernel stats of the same bench command, the stats and per-dispatch durations of the
dominant launch alone (kprof) -- and profiles/r06/records.md, a table that checks each line's kernel_ms

  * against the SAME launches in the bench command's own rocprofv3 trace: bench.py times its last kernel_iters
    calls one at a time on a drained stream (smc_time_launches: the first kernel's start to the last kernel's
    end), so the trace's last kernel_iters calls of the dominant kernel(s) are exactly those launches;
  * against the launch shape alone in tools/kprof_* (dispatches 2 .. 11: the first dispatch of a process runs cold).

    python tools/r06_records.py [--src gpurun_out/final6]
"""
import argparse
import csv
import glob
import json
import math
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIGS = ("c2", "c2h256", "c3", "c5", "lockstep", "e2e", "c2f64", "c2ref", "c2refhw")


def trace_rows(trace: str, names: tuple[str, ...]) -> list[tuple[str, int, int]]:
    with open(trace) as f:
        rows = list(csv.DictReader(f))
    out = []
    for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
        n = r["Kernel_Name"]
        if any(k in n for k in names):
            out.append((n, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return out


def kernel_names(line_kernel: str) -> tuple[str, ...]:
    """'rows_kernel+cf_kernel' -> the kernels of one call; 'resident_kernel(sliced)' -> resident_kernel."""
    return tuple(k.split("(")[0].strip() for k in line_kernel.split("+"))


def last_calls(rows: list[tuple[str, int, int]], calls: int, per_call: int) -> list[float]:
    """ms from the first kernel's start to the last kernel's end of each of the trace's last `calls` calls."""
    sel = rows[-calls * per_call:]
    out = []
    for i in range(0, len(sel), per_call):
        grp = sel[i:i + per_call]
        out.append((max(e for _, _, e in grp) - min(s for _, s, _ in grp)) / 1e6)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out", "final6"))
    ap.add_argument("--dst", default=os.path.join(ROOT, "profiles", "r06"))
    a = ap.parse_args()
    final = os.path.join(a.dst, "final")
    os.makedirs(final, exist_ok=True)
    lines = ["# Round-6 closing records (tools/micro/r06_final.sh on one MI355X; tools/r06_records.py)", "",
             "`kernel_ms` is the bench's own timing of the dominant launch: `kernel_iters` calls after the timed region,",
             "each alone on a drained stream, from the first kernel's start to the last kernel's end by the kernels' own",
             "execution timestamps (`smc_time_launches`), ÷ launches per call. The same bench command run again under",
             "rocprofv3 (`prof_<cfg>`) prints its own line; `trace` is that run's rocprofv3 record of exactly the calls",
             "its line times (the trace's last `kernel_iters` calls of the kernel(s), `prof_<cfg>_kernel_trace_tail.txt`).",
             "`own` compares the prof run's kernel_ms with its trace (one set of launches timed two ways; under the",
             "profiler the launch events of the 43-µs e2e launch read high); `line` compares the bench line's kernel_ms",
             "(an unprofiled run) with that trace (two runs of the same command: run-to-run spread). `frac (trace)`",
             "is the line's algorithmic bytes over the trace time ÷ 8 TB/s. `alone` is the launch shape in `tools/kprof_*`,",
             "dispatches 2 .. 11 (`iso_<cfg>_*`).", "",
             "| config | ms/step | kernel (line) | kernel_ms (line) | frac (line) | trace | line vs trace | kernel_ms (prof run) "
             "| own vs trace | frac (trace) | alone (kprof) |",
             "|---|---|---|---|---|---|---|---|---|---|---|"]
    for cfg in CONFIGS:
        bench = os.path.join(a.src, f"bench_{cfg}.out")
        if not os.path.exists(bench):
            continue
        text = open(bench).read().strip().splitlines()[-1]
        d = json.loads(text)
        with open(os.path.join(final, f"bench_{cfg}.json"), "w") as f:
            f.write(text + "\n")
        r = d["roofline"]
        names = kernel_names(r["kernel"])
        b_rank = d["config"]["contracts_per_gpu"]
        launches = math.ceil(b_rank / r["contracts_per_launch"])
        iters = r.get("kernel_iters") or 10
        same = alone = None
        for tag in ("prof", "iso"):
            st = glob.glob(os.path.join(a.src, f"{tag}_{cfg}", "**", "*kernel_stats.csv"), recursive=True)
            tr = glob.glob(os.path.join(a.src, f"{tag}_{cfg}", "**", "*kernel_trace.csv"), recursive=True)
            if st:
                shutil.copy(st[0], os.path.join(final, f"{tag}_{cfg}_kernel_stats.csv"))
            if not tr:
                continue
            rows = trace_rows(tr[0], names)
            if tag == "prof":
                per_call = launches * len(names)
                calls = last_calls(rows, iters, per_call)
                with open(os.path.join(final, f"prof_{cfg}_kernel_trace_tail.txt"), "w") as f:
                    f.write(f"# bench command's trace: the last {iters} calls of {'+'.join(names)} ({per_call} "
                            "dispatches per call), ms from the first start to the last end\n")
                    for ms in calls:
                        f.write(f"{ms:.4f}\n")
                same = sum(calls) / len(calls) / launches
            else:
                with open(os.path.join(final, f"iso_{cfg}_dispatches.txt"), "w") as f:
                    f.write(f"# {'+'.join(names)}: per-dispatch durations (ms) of tools/kprof_* alone\n")
                    for n, s, e in rows:
                        f.write(f"{(e - s) / 1e6:.4f}  {n[:90]}\n")
                per = [(e - s) / 1e6 for _, s, e in rows]
                k = len(names)
                sums = [sum(per[i:i + k]) for i in range(0, len(per) - k + 1, k)]
                sel = sums[1:11] if len(sums) > 2 else sums
                alone = sum(sel) / len(sel) if sel else None
        kp = None
        pout = os.path.join(a.src, f"prof_{cfg}.out")
        if os.path.exists(pout):
            plines = [ln for ln in open(pout).read().splitlines() if ln.startswith("{")]
            if plines:
                kp = json.loads(plines[-1])["roofline"]["kernel_ms"]
                with open(os.path.join(final, f"prof_{cfg}_line.json"), "w") as f:
                    f.write(plines[-1] + "\n")
        agree = f"{(kp / same - 1) * 100:+.1f} %" if same and kp else "-"
        agree_line = f"{(r['kernel_ms'] / same - 1) * 100:+.1f} %" if same else "-"
        frac_file = r["algorithmic_bytes_per_launch"] / (same * 1e-3) / (r["peak"] * 1e9) if same else None
        fmt = lambda x: f"{x:.4f}" if x is not None else "-"  # noqa: E731
        lines.append(f"| {cfg} | {d['ms_per_step']:.4f} | `{r['kernel']}` | {r['kernel_ms']:.4f} | {r['frac']:.4f} | "
                     f"{fmt(same)} | {agree_line} | {fmt(kp)} | {agree} | {fmt(frac_file)} | {fmt(alone)} |")
    pm = sorted(glob.glob(os.path.join(a.src, "pmc_*")))
    for p in pm:
        cc = glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True)
        if cc:
            shutil.copy(cc[0], os.path.join(final, f"{os.path.basename(p)}_counter_collection.csv"))
    if pm:
        lines += ["", "PMC passes (`final/pmc_*_counter_collection.csv`; summaries `pmc_*.txt` by tools/pmc_summary.py and "
                  "tools/pmc_clock.py)."]
    with open(os.path.join(a.dst, "records.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
