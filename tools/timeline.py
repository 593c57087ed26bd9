"""Print one step of a rocprofv3 kernel trace (steps delimited by the Adam kernel):
python tools/timeline.py gpurun_out/profg/run_kernel_trace.csv [step]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda x: int(x["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 6
idx = [i for i, x in enumerate(rows) if "adam_kernel" in x["Kernel_Name"]]
a, b = idx[k], idx[k + 1]
t0 = int(rows[a]["End_Timestamp"])
for x in rows[a + 1:b + 1]:
    s = int(x["Start_Timestamp"]) - t0
    e = int(x["End_Timestamp"]) - t0
    print(f"{s / 1e3:8.1f} {e / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{x['Queue_Id']} {x['Kernel_Name'][:90]}")
print(f"step {(int(rows[b]['End_Timestamp']) - t0) / 1e3:.1f} us")
