"""Print the key fields of bench.py JSON lines found in the given log files."""
import json
import sys

for f in sys.argv[1:]:
    for line in open(f):
        line = line.strip()
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        r = d.get("roofline", {})
        print(f"== {f}: {d['value']:.2f} {d['unit']} ms/step {d['ms_per_step']:.2f} steps {d['steps']} dtype {d['dtype']}")
        print("   roofline", {k: r.get(k) for k in ("achieved", "peak", "frac", "frac_of_fp32_mfma_peak", "share_of_step")})
        if "wgrad_kernel" in r:
            print("   wgrad", r["wgrad_kernel"])
        for k in ("north_star_vgg19", "cpu_baseline", "full_size_parity"):
            if k in d:
                v = dict(d[k])
                v.pop("step_s", None)
                print("  ", k, v)
