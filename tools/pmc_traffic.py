"""HBM traffic per kernel launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

gfx950 correction (MI355X_MICROARCH.md "HBM"; re-measured here with tools/calib/hbm_calib.hip
on a 1 GiB stream: FETCH_SIZE = 0.500 GiB for dword, dwordx4 and buffer_load_dword reads,
WRITE_SIZE = 1.000 GiB for dword and dwordx4 stores):  bytes = 2 * FETCH_SIZE_KB * 1024 + WRITE_SIZE_KB * 1024.
FETCH counts L2 misses to the fabric, so Infinity-Cache (MALL) hits are included: an upper bound on
true HBM bytes.

usage: python tools/pmc_traffic.py <model> [out.json]     (reads gpurun_out/pmc_<model>_{FETCH,WRITE}_SIZE)
"""
import collections
import csv
import json
import sys

FETCH_CORRECTION = 2.0
PASS_ARGS = {"reconet": "bench.py --steps 2 --warmup 2 --prof-steps 0 (headline policy)",
             "adaattn": "bench.py --model adaattn --steps 2 --warmup 2 --prof-steps 0",
             "adaattn_c5": "bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 2 --warmup 2 "
                           "--prof-steps 0 (config 5 shape, its default f16 policy)",
             "reconet_f32": "bench.py --gemm f32 --steps 2 --warmup 2 --prof-steps 0 (strict fp32 MFMA policy)"}


def load(model, counter):
    path = f"gpurun_out/pmc_{model}_{counter}/run_counter_collection.csv"
    return {r["Dispatch_Id"]: r for r in csv.DictReader(open(path))}


def family(name):
    """kernel family: the unqualified template name (namespaces and arguments dropped)"""
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]


def instance(name):
    """unqualified name with its template arguments, e.g. pil_resize_kernel<3, 5, 5>"""
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("::")[-1]


def after_marker(rows):
    """dispatches after the last vst_marker_kernel (bench.py's timed region)"""
    ids = sorted(rows, key=int)
    marks = [d for d in ids if "vst_marker_kernel" in rows[d]["Kernel_Name"]]
    if not marks:
        return rows
    last = int(marks[-1])
    return {d: r for d, r in rows.items() if int(d) > last}


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    model = args[0] if args else "reconet"
    F, W = load(model, "FETCH_SIZE"), load(model, "WRITE_SIZE")
    if "--after-marker" in sys.argv:
        F = after_marker(F)
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for d, r in F.items():
        name = r["Kernel_Name"]
        keys = {family(name), instance(name)}  # the family, and the template instance when there is one
        for key in keys:
            a = agg[key]
            a[0] += 1
            a[1] += float(r["Counter_Value"]) * 1024 * FETCH_CORRECTION
            a[2] += float(W[d]["Counter_Value"]) * 1024 if d in W else 0.0
    fams = {k: {"launches": n, "read_bytes_per_launch": f / n, "write_bytes_per_launch": w / n,
                "bytes_per_launch": (f + w) / n} for k, (n, f, w) in agg.items()}
    for k, v in sorted(fams.items(), key=lambda kv: -kv[1]["bytes_per_launch"] * kv[1]["launches"])[:15]:
        print(f"{k[:36]:36s} n={v['launches']:4d} read={v['read_bytes_per_launch']/1e6:9.1f} MB "
              f"write={v['write_bytes_per_launch']/1e6:8.1f} MB per launch")
    if len(args) > 1:
        sel = ("dispatches of bench.py's timed steps only (after its vst_marker_kernel dispatch)"
               if "--after-marker" in sys.argv else "every dispatch of the run")
        out = {"model": model, "fetch_correction": FETCH_CORRECTION,
               "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (with --kernel-trace), "
                         f"{PASS_ARGS.get(model, 'bench.py')}; {sel}; bytes = 2*FETCH + WRITE (calibrated, tools/calib)",
               "families": fams}
        json.dump(out, open(args[1], "w"), indent=1)


if __name__ == "__main__":
    main()
