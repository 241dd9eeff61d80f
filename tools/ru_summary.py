"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks: one line per kernel
(name, VGPRs, AGPRs, scratch bytes/lane, occupancy, LDS bytes).

    hipcc ... -Rpass-analysis=kernel-resource-usage 2> remarks.txt; python tools/ru_summary.py remarks.txt [filter]
"""
import re
import subprocess
import sys

rows, cur = [], None
for line in open(sys.argv[1], errors="replace"):
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split()[0]] = int(m.group(2))
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for r, n in zip(rows, names):
    n = re.sub(r"\(.*", "", n)
    if flt in n:
        print(f"{n:70s} V{r.get('VGPRs', 0):4d} A{r.get('AGPRs', 0):4d} scr{r.get('ScratchSize', 0):6d} occ{r.get('Occupancy', 0)} lds{r.get('LDS', 0)}")
