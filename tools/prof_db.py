"""Per-kernel summary of a rocprofv3 run database (rocpd sqlite output):
    python tools/prof_db.py <run_results.db> [name filter]"""
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    rows = c.execute("select name, count(*), avg(end-start)/1000.0, min(end-start)/1000.0, sum(end-start)/1e6 "
                     "from kernels where name like ? group by name order by 5 desc", (f"%{flt}%",)).fetchall()
    for r in rows:
        print(f"{r[0][:80]:80s} n={r[1]:5d} avg_us={r[2]:9.2f} min_us={r[3]:9.2f} total_ms={r[4]:8.2f}")


if __name__ == "__main__":
    main()
