"""Per-launch DAC conv durations from a rocprofv3 kernel-trace CSV (tools/dac_decode_only.py runs the decode
3 times): conv launches grouped by (kernel, grid), each group's per-launch durations in launch order."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
agg = collections.OrderedDict()
for r in rows:
    n = r['Kernel_Name']
    if not any(k in n for k in ('conv_kernel', 'conv_stage_kernel', 'conv_ldr_kernel')):
        continue
    i = n.index('conv_')
    key = (n[i:n.index('>', i) + 1], r['Grid_Size_X'], r['Grid_Size_Y'], r['Grid_Size_Z'])
    agg.setdefault(key, []).append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
tot = sum(sum(v) for v in agg.values())
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(k, len(v), f"{sum(v):.1f} us {100 * sum(v) / tot:.1f} %", [round(x, 1) for x in v[-len(v) // 3:]])
