"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks: one line per kernel
(VGPRs, AGPRs, scratch bytes/lane, occupancy). usage: kres.py < remarks.txt [filter]"""
import re
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
cur, rows = None, {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+)", line)
    if cur and m:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    if flt in k:
        print(f"{k[:90]:90s} vgpr {v.get('VGPRs', '?'):>4} agpr {v.get('AGPRs', '?'):>4} "
              f"scratch {v.get('ScratchSize', '?'):>4} occ {v.get('Occupancy', '?')}")
