"""Per-kernel stats (calls, total / average ms) from a rocprofv3 rocpd SQLite database (profiling aid)."""
import collections
import sqlite3
import sys

db = sys.argv[1]
c = sqlite3.connect(db)
tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
suf = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch_"))[len("rocpd_kernel_dispatch_"):]
names = {r[0]: r[1] for r in c.execute(f"select id, display_name from rocpd_info_kernel_symbol_{suf}")}
agg = collections.defaultdict(lambda: [0, 0])
for kid, s, e in c.execute(f"select kernel_id, start, end from rocpd_kernel_dispatch_{suf}"):
    a = agg[names.get(kid, str(kid))]
    a[0] += 1
    a[1] += e - s
top = sorted(agg.items(), key=lambda kv: -kv[1][1])[: int(sys.argv[2]) if len(sys.argv) > 2 else 40]
print("Name,Calls,TotalDurationMs,AverageMs")
for k, (n, t) in top:
    print(f"\"{k[:90]}\",{n},{t / 1e6:.3f},{t / n / 1e6:.4f}")
