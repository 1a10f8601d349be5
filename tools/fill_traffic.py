"""After a `tools/gpu.sh prof:<tag>:<cfg>` run: summarise its rocprofv3 data
(tools/prof_summary.py -> profiles/<tag>_<cfg>_summary.md and the
profiles/traffic.json entry, stamped with the tree the box ran) and copy the
bench line of the same call into profiles/<tag>_bench_<cfg>.json with
roofline.traffic / traffic_source taken from that entry.

    python tools/fill_traffic.py <tag> <cfg> [<cfg> ...]
    python tools/fill_traffic.py --key synth:rehearse8 <tag> synth   (a rehearsal line: its own traffic key)
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    argv = sys.argv[1:]
    key = None
    if argv[0] == "--key":
        key, argv = argv[1], argv[2:]
    tag, cfgs = argv[0], argv[1:]
    for cfg in cfgs:
        k = key or f"{cfg}:1"
        prof = os.path.join(REPO, "gpurun_out", f"prof_{tag}_{cfg}")
        subprocess.run([sys.executable, os.path.join(REPO, "tools", "prof_summary.py"), prof, f"{tag}_{cfg}", k],
                       check=True, stdout=subprocess.DEVNULL)
        ent = json.load(open(os.path.join(REPO, "profiles", "traffic.json")))[k]
        line = [x for x in open(os.path.join(REPO, "gpurun_out", f"{tag}_bench_{cfg}.json")) if x.startswith("{")][-1]
        d = json.loads(line)
        r = d["roofline"]
        dom = max(r["launches"], key=lambda k: r["launches"][k]["avg_us"])
        r["traffic"] = ent.get(dom)
        r["traffic_source"] = (f"profiles/traffic.json['{k}'] from {ent['source']} (tree {ent.get('head')}): "
                               "rocprofv3 PMC of the same gpurun call, 2 x FETCH_SIZE + WRITE_SIZE per launch of "
                               f"the dominant kernel ({dom})")
        out = os.path.join(REPO, "profiles", f"{tag}_bench_{cfg}.json")
        json.dump(d, open(out, "w"))
        print(f"{cfg}: {d['value']:.0f} {d['unit']}, {dom} {r['launches'][dom]['avg_us']} us, frac {r['frac']:.3f}, "
              f"traffic {r['traffic'] / 1e6 if r['traffic'] else float('nan'):.1f} MB vs algorithmic "
              f"{r['launches'][dom]['algorithmic_bytes'] / 1e6:.1f} MB -> {out}")


if __name__ == "__main__":
    main()
