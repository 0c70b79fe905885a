"""Per-kernel (and per-stream) duration table of a rocprofv3 --kernel-trace database.
usage: python tools/kernel_table.py <results.db> [top]"""
import sqlite3
import sys


def main():
    db, top = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30
    c = sqlite3.connect(db)
    q = ("select name, stream_id, grid_x, count(*), sum(end-start)/1e6, avg(end-start)/1e3 from kernels "
         "group by name, stream_id, grid_x order by sum(end-start) desc limit %d" % top)
    print("%-58s %6s %9s %7s %10s %10s" % ("kernel", "stream", "grid_x", "n", "total_ms", "avg_us"))
    for name, st, gx, n, tot, avg in c.execute(q):
        print("%-58s %6s %9d %7d %10.3f %10.2f" % (name[:58], st, gx, n, tot, avg))


if __name__ == "__main__":
    main()
