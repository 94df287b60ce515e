"""Print the kernel timeline of the last build run in a rocprofv3 kernel trace (ms from the first
kernel of that run), one line per kernel: start, end, duration, queue."""
import csv
import sys

path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# runs start at k_extract<false>; take the last one
starts = [i for i, r in enumerate(rows) if "k_extract<false>" in r["Kernel_Name"]]
seg = rows[starts[-1]:]
t0 = int(seg[0]["Start_Timestamp"])
for r in seg:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    name = r["Kernel_Name"].split("(")[0].replace("skm::", "")[:40]
    if e - s < 20000 and "chain" not in name:
        continue
    print(f"{s / 1e6:8.3f} {e / 1e6:8.3f} {(e - s) / 1e6:7.3f}  q{r.get('Queue_Id', '?'):>3s}  {name}  grid={r.get('Grid_Size', '')}")
