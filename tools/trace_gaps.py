"""Per-call timeline of the replay pipeline from a rocprofv3 trace: kernels (and memory copies, when
traced with --memory-copy-trace) in start order, with the gap before each.  Groups operations into
calls at every k_replay dispatch and prints the median duration and gap per position.
  python tools/trace_gaps.py <rocprofv3 output dir> [first kernel name, default k_replay]"""
import csv
import glob
import statistics
import sys

d = sys.argv[1]
first = sys.argv[2] if len(sys.argv) > 2 else "k_replay"
ops = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
for f in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy:" + r.get("Direction", "?")))
ops.sort()
calls, cur = [], None
for op in ops:
    if first in op[2]:
        cur = [op]
        calls.append(cur)
    elif cur is not None:
        cur.append(op)
calls = [c for c in calls if len(c) == len(calls[-1])][1:]   # same shape, the first one dropped
if not calls:
    sys.exit("no complete calls found")
print(f"{len(calls)} calls of {len(calls[0])} operations (medians, microseconds)")
for i in range(len(calls[0])):
    name = calls[0][i][2][-60:]
    dur = statistics.median((c[i][1] - c[i][0]) / 1e3 for c in calls)
    gap = statistics.median((c[i][0] - c[i - 1][1]) / 1e3 for c in calls) if i else 0.0
    print(f"  {name:60s} gap {gap:8.2f}  dur {dur:9.2f}")
span = statistics.median((c[-1][1] - c[0][0]) / 1e3 for c in calls)
print(f"  first start -> last end: {span:.2f} us")
