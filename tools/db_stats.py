"""Kernel summary (name, calls, total/avg ms) from a rocprofv3 rocpd sqlite database."""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else cols[0])
rows = db.execute(f"select {name}, count(*), sum(end-start)/1e6, avg(end-start)/1e6 from kernels group by {name} "
                  "order by sum(end-start) desc").fetchall()
tot = sum(r[2] for r in rows)
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{r[2]:10.3f} ms {100 * r[2] / tot:5.1f}%  n={r[1]:5d}  avg={r[3]:9.4f} ms  {r[0][:110]}")
