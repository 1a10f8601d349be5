"""Summarise a rocprofv3 run of bench.py into profiles/ (kernel stats + HBM traffic).

usage: python tools/prof_summary.py <prof_dir> <round_tag> [config:world]
  <prof_dir>/trace/*_kernel_stats.csv      (rocprofv3 --kernel-trace --stats)
  <prof_dir>/fetch/*_counter_collection.csv (rocprofv3 --pmc FETCH_SIZE)
  <prof_dir>/write/*_counter_collection.csv (rocprofv3 --pmc WRITE_SIZE)
Traffic per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes): on gfx950
FETCH_SIZE reports half the bytes of 16-byte-per-lane streaming reads
(MI355X_MICROARCH.md, HBM section) — the matrix streams of both passes are
16 B/lane; the random 8-byte gathers mostly hit L2 and barely register.
Infinity-Cache hits are counted too, so this is memory-side traffic.
"""
import collections
import csv
import glob
import json
import os
import sys


def pmc(path):
    d = collections.defaultdict(list)
    for f in glob.glob(os.path.join(path, "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            d[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in d.items()}


def classify(name):
    """Timed Lanczos launches (bench.py's keys): pass1 = X z (the window pass with
    step B fused in, SrcLzZ; or an unfused SrcLzStep row pass; the early step's SrcLzBeta), combine = the
    slice combine (EpiLz1), pass2 = X^T u fused with step A (EpiLz2)."""
    row_pass = any(k in name for k in ("k_window_pass", "k_tiled_pass", "k_sorted_pass", "k_sorted_pipe",
                                       "k_jag_pass", "k_jag_acc"))
    if row_pass and ("SrcLzZ" in name or "SrcLzStep" in name or "SrcLzSmall" in name or "SrcLzBeta" in name):
        return "pass1"
    if "k_cgs_" in name:   # CGS2 reorthogonalisation: one launch of each kernel per Lanczos step
        return "cgs2_per_step"
    if "k_slice_combine" in name and "EpiLz1" in name:   # k_slice_combine / _small
        return "combine"
    if (row_pass or "k_rows_apply" in name) and "EpiLz2" in name:
        return "pass2"
    if "k_xt_combine" in name and "EpiLz2" in name:   # one-piece plans: the X^T u block partials' combine
        return "pass2"
    if "k_slice_combine" in name and "EpiLz2" in name:   # a sliced pass 2's combine (step A in it)
        return "pass2"
    if row_pass and "SrcGuardPack" in name:   # a column-shard rank's pass 1 (X_p z_p, the packed sums)
        return "pass1"
    if row_pass and "SrcGuard" in name:   # a sliced pass 2's main launch (its partials go to the combine)
        return "pass2"
    return None


def main():
    src, tag = sys.argv[1], sys.argv[2]
    key = sys.argv[3] if len(sys.argv) > 3 else "news20:1"
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(repo, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace", "*_kernel_stats.csv"))[0]
    rows = list(csv.DictReader(open(stats)))
    with open(os.path.join(prof, f"{tag}_kernel_stats.csv"), "w") as f:
        f.write(open(stats).read())
    fetch, write = pmc(os.path.join(src, "fetch")), pmc(os.path.join(src, "write"))
    # the tree the box ran: `git describe --always --dirty` stamped into .rev
    # before the gpurun call and copied next to the profile (tools/prof_bench.sh)
    rf = os.path.join(src, "rev.txt")
    rev = open(rf).read().strip() if os.path.exists(rf) else "unknown"
    lines = [f"# rocprofv3 summary ({tag}, {key}, tree {rev})", "", "| kernel | calls | avg us | share | FETCH MB (x2) | WRITE MB |",
             "|---|---|---|---|---|---|"]
    traffic = collections.defaultdict(float)
    seen = collections.defaultdict(float)
    calls = collections.defaultdict(int)
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
        n = r["Name"]
        fb = 2 * fetch.get(n, 0.0) * 1024
        wb = write.get(n, 0.0) * 1024
        lines.append(f"| `{n[:110]}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | {float(r['Percentage']):.1f}% "
                     f"| {fb/1e6:.2f} | {wb/1e6:.2f} |")
        c = classify(n)
        # per class the loop-step kernel (the most calls), not the final quotient's launch of the same class
        if c and int(r["Calls"]) > calls[c]:
            calls[c] = int(r["Calls"])
            traffic[c] = fb + wb
            seen[c] = float(r["AverageNs"]) / 1e3
    lines += ["", "Per-launch traffic of the timed passes (bytes, 2 x FETCH_SIZE + WRITE_SIZE):", ""]
    for k in sorted(traffic):
        lines.append(f"- {k}: {traffic[k]/1e6:.2f} MB over {seen[k]:.2f} us of kernel time")
    open(os.path.join(prof, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    tj_path = os.path.join(prof, "traffic.json")
    tj = json.load(open(tj_path)) if os.path.exists(tj_path) else {}
    tj[key] = {k: v for k, v in traffic.items()}
    tj[key]["source"] = f"profiles/{tag}_summary.md"
    tj[key]["head"] = rev
    json.dump(tj, open(tj_path, "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
