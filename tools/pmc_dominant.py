"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs, --pmc only) for the
bench's dominant kernel into profiles/<round>/pmc_gcn_fwd_fused.json, which bench.py reads for
roofline.traffic.  FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (L2 <-> fabric requests; on
gfx950 FETCH_SIZE reports half the bytes of wide coalesced streaming reads, see
/opt/skills/guides/MI355X_MICROARCH.md, HBM section).

Usage: python tools/pmc_dominant.py gpurun_out/pmc_bench profiles/r01/pmc_gcn_fwd_fused.json"""
import csv
import json
import sys

KERNEL = "gcn_fwd_fused_kernel"


def per_dispatch(path, counter):
    vals = []
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]))
    return vals


def main():
    root, out = sys.argv[1], sys.argv[2]
    fetch = per_dispatch(root + "/fetch/run_counter_collection.csv", "FETCH_SIZE")
    write = per_dispatch(root + "/write/run_counter_collection.csv", "WRITE_SIZE")
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    res = {
        "kernel": KERNEL + "<512, true>",
        "dispatches": [len(fetch), len(write)],
        "fetch_kib_avg": round(f_kib, 1),
        "write_kib_avg": round(w_kib, 1),
        # gfx950: FETCH_SIZE counts wide streaming reads at half their bytes -> x2 (guide's correction)
        "traffic_bytes_per_launch": round((2.0 * f_kib + w_kib) * 1024.0),
        "note": "averaged over every dispatch of the kernel in `bench.py --steps 3 --warmup 2` "
                "(training steps + the roofline replay: the same 8-layer mix); FETCH x2 per the gfx950 "
                "correction, WRITE as reported",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
