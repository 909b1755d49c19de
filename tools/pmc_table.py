"""Per-kernel PMC table from rocprofv3 --pmc runs: tools/pmc_table.py <dir> [<dir> ...] [--match substr]
Prints, per kernel name (matching), the per-dispatch average of every counter collected, plus derived
fractions when the SQ counters are present (MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x
GRBM_GUI_ACTIVE/XCDs), wait fractions of SQ_WAVE_CYCLES)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(dirs, match):
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                if match and match not in name:
                    continue
                acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
                dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return acc, dur


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    match = None
    if "--match" in sys.argv:
        match = sys.argv[sys.argv.index("--match") + 1]
        args.remove(match)
    acc, dur = load(args, match)
    for name, cs in sorted(acc.items(), key=lambda kv: -sum(dur[kv[0]])):
        print("==", name[:110], " dispatches ~%d, avg %.1f us" % (len(dur[name]) / max(1, len(cs)), sum(dur[name]) / len(dur[name])))
        avg = {k: sum(v) / len(v) for k, v in cs.items()}
        for k in sorted(avg):
            print("   %-36s %16.1f" % (k, avg[k]))
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
            cyc = avg["GRBM_GUI_ACTIVE"] / 8.0
            print("   MFMA busy frac %.3f (1024 SIMDs x %.0f cycles)" % (avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc), cyc))
        if "SQ_WAVE_CYCLES" in avg:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if k in avg:
                    print("   %s / WAVE_CYCLES %.3f" % (k, avg[k] / avg["SQ_WAVE_CYCLES"]))


if __name__ == "__main__":
    main()
