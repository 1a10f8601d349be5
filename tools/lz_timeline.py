"""Kernel timeline of one Lanczos iteration from a rocprofv3 kernel trace:
python3 tools/lz_timeline.py <t_kernel_trace.csv> [iterations]
Prints gap / duration / kernel for a few iterations in the middle of the
last Lanczos call, and the mean iteration time over that call."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
nit = int(sys.argv[2]) if len(sys.argv) > 2 else 2
marks = [i for i, r in enumerate(rows) if "SrcLzStep" in r["Kernel_Name"] or "SrcLzZ" in r["Kernel_Name"]]
# iterations of the last call: consecutive marks with small index spacing
calls, cur = [], [marks[0]]
for a, b in zip(marks, marks[1:]):
    if b - a <= 12:
        cur.append(b)
    else:
        calls.append(cur)
        cur = [b]
calls.append(cur)
last = calls[-1]
mid = len(last) // 2
t0 = int(rows[last[1]]["Start_Timestamp"])
t1 = int(rows[last[-1]]["Start_Timestamp"])
print(f"iterations in the last call: {len(last)}, mean iteration {(t1 - t0) / 1e3 / (len(last) - 2):.2f} us")
prev = None
for i in range(last[mid], last[mid + nit]):
    r = rows[i]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    prev = e
    name = r["Kernel_Name"].replace("krcn::", "").replace("double", "f64").replace("float", "f32")
    print(f"  gap {gap:5.2f}  dur {(e - s) / 1e3:6.2f}  {name[:110]}")
