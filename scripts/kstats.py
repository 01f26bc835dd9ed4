"""print a rocprofv3 kernel_stats.csv as a table"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(f"{r['Name'][:64]:64s} calls={r['Calls']:>5} avg_us={float(r['AverageNs'])/1e3:9.2f} "
          f"tot_ms={float(r['TotalDurationNs'])/1e6:8.2f} pct={float(r['Percentage']):5.1f}")
