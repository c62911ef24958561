import json, sys
d = json.load(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/stamps.json"))
for k, v in d.items():
    if isinstance(v, dict):
        print(k)
        tot = 0
        for ph, vals in v.items():
            m = sum(vals) / len(vals)
            tot += m
            print(f"  {ph:20s} {m:8.0f}  {vals}")
        print("  total", round(tot))
