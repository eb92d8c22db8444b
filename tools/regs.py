"""Per-kernel VGPR / scratch summary of a hipcc -Rpass-analysis=kernel-resource-usage log.

usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2> log; python tools/regs.py log [substring ...]
"""
import re
import sys

txt = open(sys.argv[1]).read().split("Function Name: ")[1:]
keys = sys.argv[2:]
for blk in txt:
    name = blk.split()[0]
    if keys and not any(k in name for k in keys):
        continue
    v = re.search(r"VGPRs: (\d+)", blk).group(1)
    sc = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", blk).group(1)
    print(f"{v:>4} {sc:>4}  {re.sub(r'_ZN12_GLOBAL__N_1[0-9]+', '', name)[:110]}")
