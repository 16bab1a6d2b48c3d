import csv, sys
rows=list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:n]:
    print(f"{r['Name'][:80]:80s} calls={r['Calls']:>6} avg_us={float(r['AverageNs'])/1e3:8.2f} total_ms={float(r['TotalDurationNs'])/1e6:8.2f} pct={float(r['Percentage']):5.1f}")
