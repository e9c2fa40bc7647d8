"""Dispatch timeline of tools/gap_trace.sh: per kernel of the last timed
steps its duration, and the gap from the previous dispatch's end."""
import csv
import glob
import os
import sys

rows = []
for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
k = [r for r in rows if any(x in r["Kernel_Name"] for x in ("unfilter", "fixup", "dir_"))]
last = k[-int(sys.argv[2]) if len(sys.argv) > 2 else -15:]
prev = None
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f"{r['Kernel_Name'][:60]:60s} dur {(e - s) / 1e3:9.2f} us  gap {gap:7.2f} us  grid {r.get('Grid_Size', r.get('Grid_Size_X', '?'))}")
    prev = e
