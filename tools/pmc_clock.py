"""Shader clock and VALU issue rate per dispatch from a rocprofv3 --pmc run that collected GRBM_GUI_ACTIVE
(GPU-clock cycles the graphics block was busy, one value per XCD) and optionally SQ_INSTS_VALU / SQ_BUSY_CYCLES.
    clock_MHz  = GRBM_GUI_ACTIVE per XCD / dispatch duration (rocprofv3 on this pool reports one instance, the
                 SUM over the chip's XCDs: it is divided by --xcds; with per-XCD instances, their mean)
    valu_frac  = SQ_INSTS_VALU x 4 cycles / (SIMDs x GRBM cycles): VALU issue slots used at the clock the
                 kernel actually ran at (each wave64 VALU instruction holds its SIMD 4 cycles; 4 SIMDs per CU)
Usage: python tools/pmc_clock.py DIR|CSV [--kernel SUBSTRING] [--cus 256] [--xcds 8] [--min-ms 0.3] [--all]
(round 4 printed the aggregate as if it were one XCD: clocks 8x and issue fractions 1/8 of the true values)
The counter window is longer than a short dispatch's own duration, so GRBM_GUI_ACTIVE / duration reads high
below ~0.3 ms (MI355X_MICROARCH.md, DVFS give-back: round 5 printed 9.7-12.6 GHz for the 0.06-0.3 ms network
kernels): such dispatches get no clock or issue fraction (--min-ms), and a clock above the 2.4 GHz peak is
never printed as a measurement."""
import argparse
import csv
import glob
from collections import defaultdict


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("--xcds", type=int, default=8, help="XCDs summed into one aggregated GRBM_GUI_ACTIVE instance")
    ap.add_argument("--min-ms", type=float, default=0.3,
                    help="dispatches shorter than this get no clock (the counter window outlasts them)")
    ap.add_argument("--peak-mhz", type=float, default=2400.0, help="the shader clock's peak (MI355X_MICROARCH.md)")
    a = ap.parse_args()
    # keyed by (file, dispatch): two runs in one directory reuse dispatch ids (summing them doubled the counters)
    per: dict[tuple, dict] = defaultdict(lambda: {"ctr": defaultdict(float), "inst": defaultdict(int)})
    files = [a.dir] if a.dir.endswith(".csv") else sorted(glob.glob(f"{a.dir}/**/*counter_collection.csv", recursive=True))
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if a.kernel not in row["Kernel_Name"]:
                    continue
                d = per[(f, int(row["Dispatch_Id"]))]
                d["name"] = row["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-40:]
                d["dur"] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
                c = row["Counter_Name"]
                d["ctr"][c] += float(row["Counter_Value"])
                d["inst"][c] += 1
    last_file = None
    for key in sorted(per):
        f, disp = key
        if f != last_file:
            print(f"# {f}")
            last_file = f
        d = per[key]
        g, n = d["ctr"].get("GRBM_GUI_ACTIVE"), d["inst"].get("GRBM_GUI_ACTIVE", 1)
        line = f"{disp:5d} {d['name']:40s} {d['dur'] * 1e3:8.3f} ms"
        if g:
            cyc = g / n if n > 1 else g / a.xcds  # GPU-clock cycles of one XCD
            mhz = cyc / d["dur"] / 1e6
            if d["dur"] * 1e3 < a.min_ms:
                line += f"  (shorter than {a.min_ms} ms: no clock)"
            elif mhz > a.peak_mhz:
                line += f"  (counter window outlasts the dispatch: {mhz:.0f} MHz > peak, not a clock)"
            else:
                line += f"  clock {mhz:6.0f} MHz"
                v = d["ctr"].get("SQ_INSTS_VALU")
                if v:
                    line += f"  VALU {v / d['dur'] / 1e9:6.1f} G wave-inst/s, issue frac {v * 4 / (a.cus * 4 * cyc):.2f}"
        print(line)


if __name__ == "__main__":
    main()
