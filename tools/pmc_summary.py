"""Per-launch HBM bytes from rocprofv3 --pmc counter_collection CSVs (separate WRITE_SIZE and
FETCH_SIZE passes).  Counters are in KiB; FETCH_SIZE is doubled (gfx950 tallies 16-B/lane
streaming reads at half, MI355X_MICROARCH.md HBM section).  The first dispatch (warm-up) is
skipped.

    python tools/pmc_summary.py <write_dir> <fetch_dir> <kernel-substring>
"""
import csv
import glob
import json
import sys


def per_dispatch(d: str, kernel: str, counter: str) -> list[float]:
    vals: dict[int, float] = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                    k = int(row["Dispatch_Id"])
                    vals[k] = vals.get(k, 0.0) + float(row["Counter_Value"])
    return [vals[k] for k in sorted(vals)][1:]


def main() -> None:
    wdir, fdir, kernel = sys.argv[1:4]
    w = per_dispatch(wdir, kernel, "WRITE_SIZE")
    f = per_dispatch(fdir, kernel, "FETCH_SIZE")
    wb = 1024.0 * sum(w) / len(w)
    fb = 1024.0 * sum(f) / len(f)
    print(json.dumps({"write_size_bytes": wb, "fetch_size_bytes_raw": fb, "fetch_size_bytes_corrected": 2 * fb,
                      "hbm_bytes_per_launch": wb + 2 * fb, "samples": [len(w), len(f)]}))


if __name__ == "__main__":
    main()
