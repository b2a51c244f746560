"""Summarise a rocprofv3 --kernel-trace --stats CSV directory: per-kernel totals and per-shape GEMM times."""
import collections
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.2f} ms  ({tot/1e6/steps:.2f} ms per step over {steps} steps)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:45]:
    nm = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.2f} ms/step {float(r['Percentage']):5.1f}% calls={int(r['Calls'])/steps:6.1f} avg={float(r['AverageNs'])/1e3:8.1f}us {nm[:90]}")
# the roofline families bench.py prices (vst/kprof.py): every conv fwd / data-gradient launch
# (halo-tiled + per-tap implicit GEMM) and every weight-gradient launch
fams = {"conv (conv_halo_kernel + conv_gemm_kernel)": ("conv_halo_kernel", "conv_gemm_kernel"),
        "wgrad (wgrad2_kernel + wgrad_kernel + wgrad_halo_kernel)": ("wgrad2_kernel", "wgrad_kernel", "wgrad_halo_kernel")}
for fname, keys in fams.items():
    sel = [r for r in rows if any(k in r["Name"] for k in keys)]
    calls = sum(int(r["Calls"]) for r in sel)
    t = sum(float(r["TotalDurationNs"]) for r in sel)
    if calls:
        print(f"family {fname}: {t/1e6/steps:.2f} ms/step, {calls/steps:.1f} launches/step, avg {t/calls/1e3:.1f} us/launch")
if "-shapes" in sys.argv:
    tr = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in tr:
        n = r["Kernel_Name"]
        if "gemm" in n or "wgrad_kernel" in n:
            key = (n.replace("(anonymous namespace)::", "").split("(")[0][-40:], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
            agg[key][0] += 1
            agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
        print(f"{v[1]/1e3/steps:8.2f} ms/step n={v[0]:3d} avg={v[1]/v[0]:8.1f}us {k}")
