"""Per-kernel time difference between two rocprofv3 --kernel-trace --stats CSV directories (A/B of
two builds on one box): ms per step by kernel name, largest differences first.
usage: python tools/prof_diff.py <dirA> <dirB> <steps>"""
import collections
import csv
import sys


def load(d):
    out = collections.defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(f"{d}/run_kernel_stats.csv")):
        nm = r["Name"].replace("(anonymous namespace)::", "").split("(")[0][:80]
        out[nm][0] += float(r["TotalDurationNs"])
        out[nm][1] += int(r["Calls"])
    return out


a, b, steps = load(sys.argv[1]), load(sys.argv[2]), float(sys.argv[3])
ta, tb = sum(v[0] for v in a.values()), sum(v[0] for v in b.values())
print(f"total A {ta / 1e6 / steps:.2f} ms/step, B {tb / 1e6 / steps:.2f} ms/step")
rows = []
for k in set(a) | set(b):
    da, db = a[k][0] / 1e6 / steps, b[k][0] / 1e6 / steps
    rows.append((db - da, da, db, a[k][1] / steps, b[k][1] / steps, k))
rows.sort(key=lambda r: -abs(r[0]))
for r in rows[:30]:
    print(f"{r[0]:+7.3f}  A {r[1]:7.3f} ({r[3]:5.1f})  B {r[2]:7.3f} ({r[4]:5.1f})  {r[5]}")
