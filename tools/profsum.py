"""Summarise a rocprofv3 results DB (or kernel_stats CSV) into per-kernel avg durations."""
import sqlite3
import sys


def main(path):
    con = sqlite3.connect(path)
    rows = con.execute("select name, count(*), avg(end-start), min(end-start), max(end-start), "
                       "sum(end-start) from kernels group by name order by sum(end-start) desc").fetchall()
    print(f"{'calls':>6} {'avg_us':>9} {'min_us':>9} {'max_us':>9}  kernel")
    for name, c, avg, mn, mx, tot in rows:
        print(f"{c:6d} {avg/1e3:9.2f} {mn/1e3:9.2f} {mx/1e3:9.2f}  {name[:100]}")


if __name__ == "__main__":
    main(sys.argv[1])
