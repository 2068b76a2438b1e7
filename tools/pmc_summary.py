"""Counter CSV of a rocprofv3 --pmc pass -> one JSON summary per kernel (average per dispatch).

    python tools/pmc_summary.py <counter_collection.csv> <kernel substring> <algorithmic bytes/launch> > out.json
    python tools/pmc_summary.py --mfma <counter_collection.csv> > out.json   (MFMA-busy pass, per kernel)

FETCH_SIZE / WRITE_SIZE are reported in KiB by rocprofv3. On gfx950 FETCH_SIZE tallies wide
(16 B/lane) streaming reads at half their bytes (MI355X_MICROARCH.md, HBM section), so the HBM
read bytes are FETCH_SIZE x 2; WRITE_SIZE is exact for 16 B/lane stores (other widths uncalibrated).
"""
import csv
import json
import sys
from collections import defaultdict


def main(path, kernel_sub, algo_bytes):
    vals = defaultdict(list)
    names = set()
    for row in csv.DictReader(open(path)):
        if kernel_sub not in row["Kernel_Name"]:
            continue
        names.add(row["Kernel_Name"])
        vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {"kernels": sorted(names), "launches": max((len(v) for v in vals.values()), default=0),
           "algorithmic_bytes_per_launch": algo_bytes}
    for c, v in vals.items():
        kib = sum(v) / len(v)
        out[c + "_KiB_avg"] = round(kib, 2)
        corr = 2 if c == "FETCH_SIZE" else 1
        out[c + "_bytes_per_launch"] = int(kib * 1024 * corr)
        out[c + "_correction"] = corr
    if "FETCH_SIZE_bytes_per_launch" in out and algo_bytes:
        out["fetch_ratio_to_algorithmic"] = round(out["FETCH_SIZE_bytes_per_launch"] / algo_bytes, 4)
    print(json.dumps(out, indent=1))


def _short(name: str) -> str:
    """Kernel name without return type, namespaces and argument list (template arguments kept)."""
    name = name.replace("void ", "", 1).replace("(anonymous namespace)::", "")
    depth, cut, ns = 0, len(name), 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            cut = i
            break
        elif ch == ":" and depth == 0 and name[i - 1] == ":":
            ns = i + 1
    return name[ns:cut]


def mfma(path):
    """mfma_busy_frac = sum SQ_VALU_MFMA_BUSY_CYCLES / (sum GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
    (GRBM_GUI_ACTIVE is summed over the 8 XCDs; 256 CUs x 4 SIMDs); cu_busy_frac likewise from
    SQ_BUSY_CU_CYCLES over 256 CUs x 4 (the counter is in quad-cycles per CU)."""
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    dur = defaultdict(dict)
    for row in csv.DictReader(open(path)):
        k = _short(row["Kernel_Name"])
        per[k][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[k].add(row["Dispatch_Id"])
        dur[k][row["Dispatch_Id"]] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
    out = {}
    for k, c in sorted(per.items(), key=lambda kv: -sum(dur[kv[0]].values())):
        gui = c.get("GRBM_GUI_ACTIVE", 0.0) / 8
        out[k] = {"dispatches": len(disp[k]), "total_us": round(sum(dur[k].values()), 1),
                  "mfma_busy_frac": round(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (gui * 1024), 4) if gui else None,
                  "cu_busy_frac": round(c.get("SQ_BUSY_CU_CYCLES", 0.0) * 4 / (gui * 256 * 4), 3) if gui else None}
    print(json.dumps({"kernels": out}, indent=1))


def per_kernel(path):
    """Every counter of the pass, averaged per dispatch, per kernel (kernels ordered by total duration)."""
    per = defaultdict(lambda: defaultdict(float))
    dur = defaultdict(dict)
    for row in csv.DictReader(open(path)):
        k = _short(row["Kernel_Name"])
        per[k][row["Counter_Name"]] += float(row["Counter_Value"])
        dur[k][row["Dispatch_Id"]] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
    out = {}
    for k, c in sorted(per.items(), key=lambda kv: -sum(dur[kv[0]].values())):
        n = len(dur[k])
        out[k] = {"dispatches": n, "avg_us": round(sum(dur[k].values()) / n, 2),
                  **{name: round(v / n, 1) for name, v in sorted(c.items())}}
    print(json.dumps({"kernels": out}, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "--mfma":
        mfma(sys.argv[2])
    elif sys.argv[1] == "--per-kernel":
        per_kernel(sys.argv[2])
    else:
        main(sys.argv[1], sys.argv[2], int(sys.argv[3]))
