"""Print name / calls / average us of a rocprofv3 kernel_stats.csv (names shortened)."""
import csv
import re
import sys

for path in sys.argv[1:]:
    print("==", path)
    for r in csv.DictReader(open(path)):
        name = re.sub(r"\(.*", "", r["Name"]).replace("void ", "")[:60]
        print(f"  {name:60s} {int(r['Calls']):6d} {float(r['AverageNs'])/1000:10.2f} us {float(r['Percentage']):6.1f}%")
