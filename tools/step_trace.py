"""One training step of a rocprofv3 kernel trace (bench.py run): the kernels between the last two
adam_clipped_kernel launches of the timed region, in order, with durations and the idle gaps.  The
timed region ends at the adam before the longest pause between adams (the MAE / oracle legs that
follow it, before bench.py's extra clock-read steps).
  python tools/step_trace.py <run_kernel_trace.csv> [--list]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
adam = [i for i, r in enumerate(rows) if "adam_clipped" in r["Kernel_Name"]]
# the timed steps are followed by the MAE legs and then the roofline's extra steps: take the step
# that ends at the last adam before the longest pause between adams
starts = [int(rows[i]["Start_Timestamp"]) for i in adam]
gaps = [starts[k + 1] - starts[k] for k in range(len(starts) - 1)]
kend = max(range(len(gaps)), key=lambda k: gaps[k]) if gaps else len(adam) - 1
if len(gaps) < 3 or gaps[kend] < 3 * sorted(gaps)[len(gaps) // 2]:
    kend = len(adam) - 1  # no pause: the last two adams
a, b = adam[kend - 1], adam[kend]
step = rows[a + 1:b + 1]
t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
print("launches %d  span %.1f us  kernel-busy %.1f us  gaps %.1f us" % (len(step), (t1 - t0) / 1e3, busy / 1e3,
                                                                        (t1 - t0 - busy) / 1e3))
agg = {}
for r in step:
    k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
    k = k.split("((")[0].split("(float")[0].split("(gwn")[0].split("(long")[0].split("(int")[0][:60]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    c, s = agg.get(k, (0, 0.0))
    agg[k] = (c + 1, s + d)
for k, (c, s) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print("%-62s %3d %8.1f" % (k, c, s))
if "--list" in sys.argv:
    prev = None
    for r in step:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (st - prev) / 1e3 if prev else 0.0
        print("%7.1f %7.1f  %s" % (gap, (en - st) / 1e3, r["Kernel_Name"][:90]))
        prev = en
