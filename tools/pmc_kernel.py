"""Mean per-dispatch PMC values of one kernel (name substring) from rocprofv3 csv passes."""
import collections, csv, glob, json, sys
pat = sys.argv[1]
out = {}
for d in sys.argv[2:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        for k, v in agg.items():
            out[k] = sum(v.values()) / len(v)
print(json.dumps(out, indent=1))
