"""Per-batch kernel table from a rocprofv3 --kernel-trace run: prof_table.py <run dir> <divisor> [rows]."""
import csv
import os
import subprocess
import sys

d, div = sys.argv[1], float(sys.argv[2])
rows_n = int(sys.argv[3]) if len(sys.argv) > 3 else 30
out = os.path.join(d, "stats.csv")
subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "prof_summary.py"), d, out], check=True,
               stdout=subprocess.DEVNULL)
rows = list(csv.DictReader(open(out)))
for r in rows[:rows_n]:
    print(f'{float(r["TotalDurationNs"]) / 1e6 / div:8.3f} ms {int(r["Calls"]):6d} {float(r["AverageNs"]) / 1e3:9.1f} us  '
          f'{r["Name"][:100]}')
print(f'total {sum(float(r["TotalDurationNs"]) for r in rows) / 1e6 / div:.3f} ms')
