"""Per-kernel duration summary of a rocprofv3 SQLite output (run_results.db): name, calls,
average / min / max ms.  python tools/rocpd_stats.py <db> [name-substring ...]"""
import sqlite3
import sys


def stats(db: str, keys: list[str]) -> list[tuple[str, int, float, float, float]]:
    con = sqlite3.connect(db)
    rows = con.execute("select name, count(*), avg(end - start), min(end - start), max(end - start) "
                       "from kernels group by name order by sum(end - start) desc").fetchall()
    out = []
    for name, n, avg, lo, hi in rows:
        if not keys or any(k in name for k in keys):
            out.append((name, n, avg / 1e6, lo / 1e6, hi / 1e6))
    return out


if __name__ == "__main__":
    for name, n, avg, lo, hi in stats(sys.argv[1], sys.argv[2:]):
        print(f"{name[:90]:90s} calls {n:5d} avg {avg:8.4f} ms  min {lo:8.4f}  max {hi:8.4f}")
