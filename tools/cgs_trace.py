"""Per-k CGS2 kernel times from a rocprofv3 kernel trace of a rcv1_stress run:
python3 tools/cgs_trace.py gpurun_out/trace_<tag>/t_kernel_trace.csv

A CGS2 step starts at its first dot sweep (k_cgs_rowdots / k_cgs_rowdots_v)
after the previous step's last sweep (k_cgs_update_norm, or k_cgs_colsweep
with kNorm = true); kernels are keyed by name with the template arguments."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
seq = [(r["Kernel_Name"].split("(")[0].split("::")[-1][:44], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
       for r in rows]


def is_last(name):
    return name.startswith("k_cgs_update_norm") or (name.startswith("k_cgs_colsweep") and ", true" in name)


it, per, span, open_step = -1, collections.defaultdict(lambda: collections.defaultdict(float)), {}, False
for name, t0, t1 in seq:
    if name.startswith("k_cgs_rowdots") and not open_step:
        it += 1
        span[it] = [t0, t1]
        open_step = True
    if it >= 0 and open_step:
        per[it][name] += (t1 - t0) / 1e3
        if name.startswith("k_cgs"):
            span[it][1] = t1
        if is_last(name):
            open_step = False
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
print("per m=500 step, k = 1..499 (ms):", {k: round(v / 1e3, 2) for k, v in tot.items()},
      "sum", round(sum(tot.values()) / 1e3, 2))
