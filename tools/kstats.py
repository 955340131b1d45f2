"""Print a rocprofv3 kernel_stats.csv as a compact table: name, calls, total ms, avg us, share."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:top]:
    n = r["Name"].split("(")[0].replace("void ", "").replace("cdm::", "")
    print(f'{n[:100]:100s} {r["Calls"]:>6} {float(r["TotalDurationNs"]) / 1e6:9.2f} '
          f'{float(r["AverageNs"]) / 1e3:9.1f} {100 * float(r["TotalDurationNs"]) / tot:5.1f}')
print(f"total {tot / 1e6:.1f} ms")
