"""MFMA-busy / stall summary per kernel family (and per GEMM instantiation) from the SQ / GRBM passes of
tools/pmc_round.sh.

Per family, over the dispatches after bench.py's vst_marker_kernel (the timed steps):
  mfma_busy      = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x dispatch cycles), dispatch cycles =
                   GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs) -- the share of the chip's MFMA
                   issue capacity the family used while it ran
  clock_ghz      = GRBM_GUI_ACTIVE / 8 / kernel duration (DVFS: the clock the chip held)
  wait_any / wait_inst / active = SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
  per-MFMA instruction mix (VALU, LDS, VMEM, SALU) and LDS bank-conflict cycles per LDS instruction

usage: python tools/pmc_busy.py <model> [out.json]
"""
import collections
import csv
import json
import sys

FAMILIES = ("conv_halo_kernel", "conv_gemm_kernel", "wgrad2_kernel", "wgrad_kernel", "wgrad_halo_kernel", "wgrad_reduce_kernel")
SIMDS = 1024


def load(model, i):
    base = f"gpurun_out/pmcb_{model}_{i}"
    rows = collections.defaultdict(dict)
    for r in csv.DictReader(open(base + "/run_counter_collection.csv")):
        rows[r["Dispatch_Id"]][r["Counter_Name"]] = rows[r["Dispatch_Id"]].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        rows[r["Dispatch_Id"]]["_name"] = r["Kernel_Name"]
    dur = {r["Dispatch_Id"]: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
           for r in csv.DictReader(open(base + "/run_kernel_trace.csv"))}
    for d in rows:
        rows[d]["_ns"] = dur.get(d, 0)
    ids = sorted(rows, key=int)
    marks = [d for d in ids if "vst_marker_kernel" in rows[d]["_name"]]
    last = int(marks[-1]) if marks else -1
    return {d: r for d, r in rows.items() if int(d) > last}


def fam(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]
    return n


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").replace("vstk::", "").split("(")[0]


def main():
    args = sys.argv[1:]
    model = args[0] if args else "reconet"
    p1, p2 = load(model, 1), load(model, 2)
    out = {"model": model, "method": "rocprofv3 --pmc (two passes, --kernel-trace only) of bench.py --steps 2 --warmup 2 "
                                     "--prof-steps 0, dispatches after bench.py's vst_marker_kernel", "families": {}}
    def summary(match):
        a = collections.defaultdict(float)
        n = 0
        for d, r in p1.items():
            if not match(r["_name"]):
                continue
            n += 1
            for k, v in r.items():
                if not k.startswith("_"):
                    a[k] += v
            a["_ns"] += r["_ns"]
        for d, r in p2.items():
            if not match(r["_name"]):
                continue
            for k, v in r.items():
                if not k.startswith("_"):
                    a[k] += v
        if not n:
            return None
        cyc = a["GRBM_GUI_ACTIVE"] / 8
        wc = a["SQ_WAVE_CYCLES"]
        mf = max(a["SQ_INSTS_MFMA"], 1.0)  # (the reduce kernels issue no MFMA: their ratios are per instruction)
        return {
            "launches": n, "ms": a["_ns"] / 1e6,
            "mfma_busy": a["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc),
            "clock_ghz": cyc / a["_ns"],
            "wait_any": a["SQ_WAIT_ANY"] / wc, "wait_inst": a["SQ_WAIT_INST_ANY"] / wc, "active": a["SQ_ACTIVE_INST_ANY"] / wc,
            "valu_per_mfma": a["SQ_INSTS_VALU"] / mf, "lds_per_mfma": a["SQ_INSTS_LDS"] / mf,
            "vmem_rd_per_mfma": a["SQ_INSTS_VMEM_RD"] / mf, "salu_per_mfma": a["SQ_INSTS_SALU"] / mf,
            "lds_conflict_cycles_per_lds_inst": a["SQ_LDS_BANK_CONFLICT"] / max(a["SQ_INSTS_LDS"], 1.0),
        }

    for f in FAMILIES:
        res = summary(lambda name, f=f: fam(name) == f)
        if res is None:
            continue
        out["families"][f] = res
        print(f, {k: round(v, 3) for k, v in res.items()})
    # the GEMM instantiations (template arguments) one by one, largest total time first
    names = collections.Counter()
    for r in p1.values():
        if fam(r["_name"]) in FAMILIES:
            names[short(r["_name"])] += r["_ns"]
    out["kernels"] = {}
    for nm, _ in names.most_common(16):
        out["kernels"][nm] = summary(lambda name, nm=nm: short(name) == nm)
        print(" ", nm, {k: round(v, 3) for k, v in out["kernels"][nm].items()})
    if len(args) > 1:
        json.dump(out, open(args[1], "w"), indent=1)


if __name__ == "__main__":
    main()
