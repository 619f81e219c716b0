#!/usr/bin/env python3
"""Per-kernel totals of a rocprofv3 --pmc pass (run_counter_collection.csv),
one JSON line per kernel: counter sums per launch, launch count, and the
SQ wait/issue fractions of SQ_WAVE_CYCLES when those counters are present.

usage: pmc_kernels.py <dir holding run_counter_collection.csv (searched)> [--note TEXT]
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def main():
    root = Path(sys.argv[1])
    note = sys.argv[sys.argv.index("--note") + 1] if "--note" in sys.argv else None
    files = sorted(root.rglob("*counter_collection.csv"))
    if not files:
        print(json.dumps({"error": f"no counter_collection.csv under {root}"}))
        return
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    dur = defaultdict(dict)  # kernel -> dispatch -> ns
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"].split("(")[0]
                tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
                d = (f.name, row.get("Dispatch_Id", row.get("Correlation_Id", "")))
                disp[k].add(d)
                if row.get("Start_Timestamp") and row.get("End_Timestamp"):
                    dur[k][d] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    if note:
        print(json.dumps({"note": note}))
    for k, c in sorted(tot.items(), key=lambda kv: -sum(kv[1].values())):
        n = max(1, len(disp[k]))
        out = {name: round(v / n, 1) for name, v in sorted(c.items())}
        out["kernel"] = k
        out["launches"] = n
        if dur[k]:
            # mean profiled duration; with GRBM_GUI_ACTIVE (summed over the 8
            # XCDs) the effective clock of the pass (MI355X_MICROARCH.md,
            # DVFS give-back: reads high below ~0.3 ms per dispatch)
            ns = sum(dur[k].values()) / len(dur[k])
            out["dur_us"] = round(ns / 1e3, 2)
            ga = c.get("GRBM_GUI_ACTIVE")
            if ga and ns > 0:
                out["eff_clock_GHz"] = round(ga / n / 8 / ns, 3)
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for name in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if name in c:
                    out["frac_" + name] = round(c[name] / wc, 3)
        print(json.dumps(out))


if __name__ == "__main__":
    main()
