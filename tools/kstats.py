"""Summarise a rocprofv3 rocpd database: per-kernel count, mean and total ms."""
import glob
import sqlite3
import sys

db = sys.argv[1] if len(sys.argv) > 1 else sorted(glob.glob("gpurun_out/prof_bc7/**/*.db", recursive=True))[-1]
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), avg(end-start)/1e6, sum(end-start)/1e6 from kernels "
                 "group by name order by 4 desc").fetchall()
for name, n, avg, tot in rows:
    if "gic" in name:
        print(f"{name[:70]:70s} {n:4d} {avg:10.3f} {tot:10.3f}")
