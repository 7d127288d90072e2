"""Timeline of the last plan launch in a rocprofv3 kernel trace: the pqg kernels dispatched after the last
gap of more than `gap` us between dispatches (start / end relative to the first, queue, grid), then
the end time of each queue. Usage: python tools/trace_timeline.py <rocprof dir> [gap_us]"""
import csv
import glob
import sys

d = sys.argv[1]
gap = float(sys.argv[2]) if len(sys.argv) > 2 else 200.0
f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "pqg" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last launch: kernels after the last start gap > gap us from the previous kernel's end
start = 0
end_max = int(rows[0]["End_Timestamp"])
for i in range(1, len(rows)):
    s = int(rows[i]["Start_Timestamp"])
    if s - end_max > gap * 1000:
        start = i
    end_max = max(end_max, int(rows[i]["End_Timestamp"]))
last = rows[start:]
t0 = int(last[0]["Start_Timestamp"])
print("start_us   end_us   dur_us queue grid kernel")
qend = {}
for r in last:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    q = r["Queue_Id"]
    qend[q] = max(qend.get(q, 0), e)
    print(f"{s:8.1f} {e:8.1f} {e - s:8.1f} q{q} {r['Grid_Size_X']:>8} {r['Kernel_Name'][:70]}")
print("queue ends:", {f"q{k}": round(v, 1) for k, v in sorted(qend.items())})
