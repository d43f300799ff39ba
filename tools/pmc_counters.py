"""Per-kernel averages of every counter in rocprofv3 --pmc output directories (counter_collection CSVs),
summed over the agent's instances (XCDs / SEs), the first dispatch of each kernel skipped when there are
more.  Usage: python tools/pmc_counters.py DIR|CSV [DIR|CSV ...] [--kernel SUBSTRING]"""
import argparse
import csv
import glob
from collections import defaultdict


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="")
    a = ap.parse_args()
    for d in a.dirs:
        vals: dict[tuple[str, str], dict[int, float]] = defaultdict(dict)
        # a counter_collection CSV, or a directory (every run under it: give one run per directory, as
        # dispatch ids of different runs collide)
        files = [d] if d.endswith(".csv") else glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
        for f in files:
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if a.kernel not in row["Kernel_Name"]:
                        continue
                    name = row["Kernel_Name"].replace("(anonymous namespace)::", "")
                    k = (name.split("(")[0][-60:], row["Counter_Name"])
                    disp = int(row["Dispatch_Id"])
                    vals[k][disp] = vals[k].get(disp, 0.0) + float(row["Counter_Value"])
        print(d)
        for (kern, ctr), per in sorted(vals.items()):
            xs = [per[i] for i in sorted(per)]
            xs = xs[1:] if len(xs) > 1 else xs
            print(f"  {kern:60s} {ctr:24s} {sum(xs) / len(xs):.4e}  (n={len(xs)})")


if __name__ == "__main__":
    main()
