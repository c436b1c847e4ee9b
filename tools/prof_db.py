"""Per-kernel summary of a rocprofv3 SQLite trace (rocpd schema): total / count / average
duration per kernel name, over the last ``steps`` equal parts of the trace if asked.

  python tools/prof_db.py results.db [top_n] [per_step_divisor]
"""
import sqlite3
import sys


def summary(db, top=40, div=1.0):
    c = sqlite3.connect(db)
    rows = c.execute("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s "
                     "on d.kernel_id = s.id").fetchall()
    agg = {}
    for name, a, b in rows:
        t = agg.setdefault(name, [0, 0.0])
        t[0] += 1
        t[1] += (b - a) / 1e3
    tot = sum(v[1] for v in agg.values())
    print(f"{len(rows)} dispatches, {tot / 1e3 / div:.3f} ms kernel time (/ {div})")
    for name, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{us / div:10.1f} us {n / div:8.1f} x {us / n:8.1f} us  {100 * us / tot:5.1f}%  {name[:110]}")


if __name__ == "__main__":
    summary(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40, float(sys.argv[3]) if len(sys.argv) > 3 else 1.0)
