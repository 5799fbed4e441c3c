"""Per-kernel summary of a rocprofv3 SQLite result (rocpd ``kernels`` view).

    python tools/rocpd_summary.py gpurun_out/prof/run_results.db [steps] [top]
"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end-start), avg(end-start) from kernels group by name "
                     "order by sum(end-start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    print(f"{'kernel':90s} {'calls':>6s} {'ms/step':>9s} {'avg us':>9s} {'share':>6s}")
    for name, n, s, a in rows[:top]:
        print(f"{name[:90]:90s} {n:6d} {s / 1e6 / steps:9.3f} {a / 1e3:9.1f} {100 * s / tot:5.1f}%")
    print(f"total ms/step {tot / 1e6 / steps:.3f}")


if __name__ == "__main__":
    main()
