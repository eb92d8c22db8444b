"""Sum rocprofv3 --pmc counters per kernel (substring match on the name).
usage: python tools/pmc_kernels.py <run_counter_collection.csv> substr [substr ...]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
keys = sys.argv[2:]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    name = r["Kernel_Name"]
    for k in keys:
        if k in name:
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
for k in keys:
    v = agg[k]
    print(f"{k}: {len(disp[k])} dispatches")
    for c, x in sorted(v.items()):
        print(f"   {c:24s} {x:16.0f}")
    if v.get("SQ_WAVES"):
        w = v["SQ_WAVES"]
        print(f"   per wave: cycles {v.get('SQ_WAVE_CYCLES', 0) / w:.0f}  valu {v.get('SQ_INSTS_VALU', 0) / w:.0f}  "
              f"salu {v.get('SQ_INSTS_SALU', 0) / w:.0f}  vmem_rd {v.get('SQ_INSTS_VMEM_RD', 0) / w:.0f}  "
              f"wait_inst_any {v.get('SQ_WAIT_INST_ANY', 0) / w:.0f}  wait_any {v.get('SQ_WAIT_ANY', 0) / w:.0f}  "
              f"active_valu {v.get('SQ_ACTIVE_INST_VALU', 0) / w:.0f}")
