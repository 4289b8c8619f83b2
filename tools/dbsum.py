"""Per-kernel summary of a rocprofv3 kernel-trace database (last ``--frac`` of the dispatches)."""
import collections
import glob
import sqlite3
import sys

path = sys.argv[1]
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
db = glob.glob(path + "/**/*.db", recursive=True)[0] if not path.endswith(".db") else path
c = sqlite3.connect(db)
rows = c.execute("select name, start, end from kernels order by start").fetchall()
part = rows[int(len(rows) * (1 - frac)):]
agg = collections.defaultdict(lambda: [0, 0.0])
for n, s, e in part:
    agg[n][0] += 1
    agg[n][1] += (e - s) / 1e3
tot = sum(v[1] for v in agg.values())
span = (part[-1][2] - part[0][1]) / 1e3
print(f"dispatches {len(part)}  busy {tot:.0f} us  span {span:.0f} us")
for n, (k, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{k:6d} {t:10.1f} us {t / k:8.2f} us/launch  {n[:120]}")
