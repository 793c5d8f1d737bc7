"""Print the kernel trace of a rocprofv3 --kernel-trace CSV directory in dispatch order:
name, duration (us), gap to the previous kernel's end (us).  usage: tools/trace_kernels.py <dir> [name-filter]"""
import csv
import glob
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
flt = sys.argv[2] if len(sys.argv) > 2 else ""
prev = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if flt in r["Kernel_Name"]:
        print(f"{r['Kernel_Name'][:40]:40s} {(e - s) / 1000:9.1f} us  gap {((s - prev) / 1000 if prev else 0):8.1f} us")
    prev = e
