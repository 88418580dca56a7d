"""Compare per-kernel average durations of the A/B rocprofv3 runs (tools/gpu_ab_prof.sh)."""
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/abp"
pat = sys.argv[2] if len(sys.argv) > 2 else ""
res = {}
for v in ("old", "new"):
    for f in sorted(glob.glob(f"{root}/{v}_*/**/*kernel_stats.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            if pat in r["Name"]:
                res.setdefault(r["Name"][:60], {}).setdefault(v, []).append(float(r["AverageNs"]) / 1e3)
for k, d in sorted(res.items(), key=lambda kv: -max(max(x) for x in kv[1].values())):
    print(f"{k:60s} old {['%.1f' % x for x in d.get('old', [])]} new {['%.1f' % x for x in d.get('new', [])]} us")
