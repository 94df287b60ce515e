"""Summarise a rocprofv3 rocpd database (kernel trace): per-kernel totals, and with --last-step
the timeline of the last build run (kernels after the last k_pass_ids launch)."""
import sqlite3
import sys

db = sys.argv[1]
c = sqlite3.connect(db)
rows = c.execute("select name, start, end, stream_id from kernels order by start").fetchall()
if "--last-step" in sys.argv:
    idx = [i for i, r in enumerate(rows) if r[0].startswith("skm::k_pass_ids")]
    if idx:
        rows = rows[idx[-1]:]
t0 = rows[0][1]
agg = {}
for name, s, e, sid in rows:
    k = name.split("(")[0][:48]
    a = agg.setdefault(k, [0, 0.0, 0.0])
    a[0] += 1
    a[1] += (e - s) / 1e6
    a[2] = max(a[2], (e - s) / 1e6)
print(f"span {(max(r[2] for r in rows) - t0) / 1e6:.1f} ms over {len(rows)} kernels")
for k, (n, tot, mx) in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
    print(f"{k:50s} n={n:5d} tot={tot:9.1f} ms  avg={tot / n:8.3f}  max={mx:8.2f}")
if "--timeline" in sys.argv:
    for name, s, e, sid in rows:
        if (e - s) > 5e6:
            print(f"{(s - t0) / 1e6:9.1f} {(e - t0) / 1e6:9.1f} st{sid} {name.split('(')[0][:40]}")
