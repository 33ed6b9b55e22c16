#!/usr/bin/env python3
"""VGPRs / VGPR spills / scratch per k_trace variant from a
`-Rpass-analysis=kernel-resource-usage` remark stream on stdin."""
import re
import sys

cur, rows = None, {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[bytes/lane\])?: (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    if "k_trace" in k and "ILi8E" in k:
        print(f"{k[18:60]:44s} VGPRs {v.get('VGPRs', 0):4d} spill {v.get('VGPRs Spill', 0):3d} "
              f"scratch {v.get('ScratchSize', 0):5d} waves {v.get('Occupancy', 0)}")
