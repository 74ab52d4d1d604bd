"""Summarise rocprofv3 counter_collection CSVs: per kernel, counter totals over dispatches."""
import csv, sys, glob, collections
tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((f, r["Dispatch_Id"]))
for k in sorted(tot, key=lambda k: -tot[k].get("SQ_WAVE_CYCLES", 0)):
    print(k, "dispatches", len(disp[k]))
    for c, v in sorted(tot[k].items()):
        print("   %-26s %.4g" % (c, v))
