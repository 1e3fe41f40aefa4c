"""Per-kernel duration statistics from a rocprofv3 database (the .db that
`rocprofv3 --kernel-trace --stats` writes by default), in the columns of the
kernel_stats.csv of `--output-format csv`: name, calls, total / average /
min / max duration (ns), percentage, plus the dispatch's VGPR / SGPR counts.

usage: python tools/rocpd_stats.py <results.db> [out.csv]
"""
import csv
import sqlite3
import sys


def kernel_stats(db):
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
        "max(vgpr_count), max(accum_vgpr_count), max(sgpr_count) from kernels group by name "
        "order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    return [{"Name": r[0], "Calls": r[1], "TotalDurationNs": int(r[2]), "AverageNs": round(r[3], 1),
             "Percentage": round(100.0 * r[2] / total, 3), "MinNs": int(r[4]), "MaxNs": int(r[5]),
             "VGPR": r[6], "AccumVGPR": r[7], "SGPR": r[8]} for r in rows]


def main():
    stats = kernel_stats(sys.argv[1])
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.DictWriter(out, fieldnames=list(stats[0].keys()) if stats else ["Name"])
    w.writeheader()
    for s in stats:
        w.writerow(s)


if __name__ == "__main__":
    main()
