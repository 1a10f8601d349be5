"""Per-k CGS2 kernel times from a rocprofv3 kernel trace of a rcv1_stress run:
python3 tools/cgs_trace.py gpurun_out/trace_<tag>/t_kernel_trace.csv"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
seq = [(r["Kernel_Name"].split("(")[0].split("::")[-1][:24], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
       for r in rows]
it, per, span = -1, collections.defaultdict(lambda: collections.defaultdict(float)), {}
first = "k_cgs_rowdots" if any(s[0].startswith("k_cgs_rowdots") for s in seq) else "k_cgs_dots"
for name, t0, t1 in seq:
    if name.startswith(first):
        it += 1
        span[it] = [t0, t1]
    if it >= 0:
        per[it][name] += (t1 - t0) / 1e3
        if name.startswith("k_cgs"):
            span[it][1] = t1
last = sorted(per)[-499:]
for j in [0, 1, 5, 10, 50, 100, 200, 300, 400, 497]:
    d = per[last[j]]
    cg = {k: round(v, 1) for k, v in d.items() if "cgs" in k}
    print(j + 1, cg, "sum", round(sum(cg.values()), 1), "span", round((span[last[j]][1] - span[last[j]][0]) / 1e3, 1))
tot = collections.defaultdict(float)
for j in last:
    for k, v in per[j].items():
        if "cgs" in k:
            tot[k] += v
print("per step (ms):", {k: round(v / 1e3, 2) for k, v in tot.items()}, "sum", round(sum(tot.values()) / 1e3, 2))
