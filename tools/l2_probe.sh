#!/bin/bash
# Per-workgroup work held fixed (32-root cooperative tiles), roots per XCD varied: does the search
# slow down as the per-XCD tree footprint outgrows the 4 MB L2?  (diagnostic)
set -e
out=${1:-gpurun_out/l2_probe.jsonl}
: > "$out"
for b in 1024 2048 4096 8192; do
  MZH_ROWS=32 timeout -k 10 120 python -u tools/phase_probe.py --roots $b --kernel coop >> "$out"
done
cat "$out"
