"""Per-kernel breakdown of decode steps from a rocprofv3 kernel trace (CSV).

    python tools/step_breakdown.py gpurun_out/prof/run_kernel_trace.csv

Finds sampler launches (one per decode step), takes the steps between consecutive samplers,
and reports per kernel class (by name + grid) the mean duration, and the mean idle gap before it.
"""
import collections
import csv
import sys


def main(path, skip=50):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    samp = [i for i, r in enumerate(rows) if "sample_kernel" in r["Kernel_Name"]]
    # decode steps: consecutive samplers separated by a full step of kernels
    steps = [(a, b) for a, b in zip(samp, samp[1:]) if 100 < b - a < 400][skip:]
    dur = collections.defaultdict(list)
    gap = collections.defaultdict(list)
    tot = []
    for a, b in steps:
        t0 = int(rows[a]["End_Timestamp"])
        tot.append((int(rows[b]["End_Timestamp"]) - t0) / 1e3)
        prev_end = t0
        for i in range(a + 1, b + 1):
            r = rows[i]
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")[-60:]
            key = f"{name} grid={r['Grid_Size_X']}x{r['Grid_Size_Y']}"
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            dur[key].append((e - s) / 1e3)
            gap[key].append((s - prev_end) / 1e3)
            prev_end = e
    n = len(steps)
    print(f"{n} decode steps, mean step {sum(tot) / n:.1f} us")
    tk = tg = 0.0
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        d, g = dur[k], gap[k]
        per_step = len(d) / n
        print(f"{k:80s} x{per_step:5.1f}  dur {sum(d) / len(d):7.2f} us  gap {sum(g) / len(g):6.2f} us  "
              f"step-total {sum(d) / n:7.1f} + {sum(g) / n:6.1f}")
        tk += sum(d) / n
        tg += sum(g) / n
    print(f"kernels {tk:.1f} us + gaps {tg:.1f} us per step")


if __name__ == "__main__":
    main(sys.argv[1])
