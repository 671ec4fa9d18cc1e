import csv, sys
r = list(csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/prof/run_kernel_stats.csv')))
for x in r:
    print(f"{x['Name'][:80]:80s} calls={x['Calls']:>6s} avg_us={float(x['AverageNs'])/1e3:9.2f} tot_ms={float(x['TotalDurationNs'])/1e6:9.2f} pct={float(x['Percentage']):6.2f}")
