"""Print one graph-replayed step of a rocprofv3 kernel trace (between two Adam launches):
start / end (us from the previous step's Adam), duration, queue, kernel, grid."""
import csv
import sys

path = sys.argv[1]
which = int(sys.argv[2]) if len(sys.argv) > 2 else 6
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
a, b = idx[which], idx[which + 1]
t0 = int(rows[a]["End_Timestamp"])
for r in rows[a + 1:b + 1]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{s:8.1f} {e:8.1f} {e - s:7.1f} q{r['Queue_Id']} {r['Kernel_Name'][:58]} "
          f"grid={r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}")
