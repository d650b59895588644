"""Print a rocprofv3 --stats kernel summary (run_kernel_stats.csv) compactly: name, calls, avg us."""
import csv
import sys

for path in sys.argv[1:]:
    print("==", path)
    for r in csv.DictReader(open(path)):
        name = r["Name"].replace("kcc::(anonymous namespace)::", "").replace("void ", "")
        print(f"  {name[:64]:64s} {r['Calls']:>5s} {float(r['AverageNs']) / 1000:9.1f} us")
