"""One summary line of a bench.py JSON log (tools/ab.sh, tools/ab_env.sh)."""
import json
import sys

d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
times = "  ".join(f"{k} {v['avg_us']:7.2f}" for k, v in r["launches"].items())
ro = d.get("reorth")
extra = f"  reorth {ro['ms_per_step']:6.2f} ms" if ro else ""
hw = d.get("hvp_warm_us")
if isinstance(hw, dict):
    extra += f"  hvp {hw['median']:6.2f} us ({d['hvp_warm_frac']['of_8.0_TBps']:.3f})"
print(f"{sys.argv[1]:28s} {d['value']:9.0f} HVP/s  plan1 {r['plan']['pass1']}  {times}{extra}")
pl = d.get("placement")
if pl and pl.get("probed"):
    lz = pl.get("lanczos") or {}
    print(f"{'':28s} placement: kept {pl['kept']} of {pl['us']} us (hot {pl['hot_mb']} MB); "
          f"lanczos calls: kept {lz.get('kept')} of {lz.get('ms')} ms")
