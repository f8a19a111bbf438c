"""Print a kernel timeline (start offset, duration, stream) from a rocprofv3 kernel_trace.csv:
   python tools/timeline.py gpurun_out/sp5/stage_kernel_trace.csv [first_kernel_substring]"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
if len(sys.argv) > 2:
    i0 = next(i for i, r in enumerate(rows) if sys.argv[2] in r["Kernel_Name"])
    rows = rows[i0:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows[:60]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print("%10.1f %10.1f %9.1f  q%-3s %s" % (s / 1e3, e / 1e3, (e - s) / 1e3, r["Queue_Id"], r["Kernel_Name"][:60]))
