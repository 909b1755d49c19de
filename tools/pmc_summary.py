"""Per-kernel summary of rocprofv3 PMC passes (tools/pmc.sh) over the benchmark: HBM traffic
(FETCH_SIZE x2 per the gfx950 correction + WRITE_SIZE, KiB per dispatch), MFMA busy fraction
(SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x kernel cycles, kernel cycles = GRBM_GUI_ACTIVE / 8 XCDs),
and the wave-cycle split (SQ_WAIT_ANY = parked on s_waitcnt / barrier, SQ_WAIT_INST_ANY = issue
stalls, SQ_ACTIVE_INST_ANY = issuing; quad-cycles, fractions of SQ_WAVE_CYCLES).

Usage: python tools/pmc_summary.py gpurun_out/pmc out.json kernel_substring [kernel_substring ...]"""
import collections
import csv
import glob
import json
import os
import sys


def load(root):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))  # kernel -> counter -> [per dispatch]
    for path in glob.glob(os.path.join(root, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(path)):
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return vals


def main():
    root, out, subs = sys.argv[1], sys.argv[2], sys.argv[3:]
    vals = load(root)
    res = {}
    for sub in subs:
        agg = collections.defaultdict(list)
        name = None
        for k, cs in vals.items():
            if sub in k:
                name = k
                for c, v in cs.items():
                    agg[c] += v
        if not agg:
            continue
        avg = {c: sum(v) / len(v) for c, v in agg.items()}
        r = {"kernel": name[:120], "dispatches": {c: len(v) for c, v in agg.items()}, "avg": avg}
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            r["hbm_bytes_per_dispatch"] = round((2.0 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024.0)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
            r["mfma_busy_frac"] = round(avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * avg["GRBM_GUI_ACTIVE"] / 8.0), 4)
        if "SQ_WAVE_CYCLES" in avg:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in avg:
                    r[c.lower() + "_frac"] = round(avg[c] / avg["SQ_WAVE_CYCLES"], 4)
        res[sub] = r
    json.dump(res, open(out, "w"), indent=1)
    for k, r in res.items():
        print(k, {x: y for x, y in r.items() if x not in ("avg", "dispatches", "kernel")})


if __name__ == "__main__":
    main()
