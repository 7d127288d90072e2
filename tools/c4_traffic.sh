#!/bin/bash
# HBM traffic of one C4 launch (125 M rows, all 16 columns): separate rocprofv3 --pmc passes for
# FETCH_SIZE and WRITE_SIZE over bench.py --workload c4, summed over the launch's kernels (each runs
# once per launch) -> gpurun_out/<tag>/traffic_c4.json (copy to profiles/traffic_c4_latest.json).
#   bash tools/c4_traffic.sh <tag>
set -euo pipefail
TAG=$1
OUT=gpurun_out/$TAG/c4pmc; mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pass$i" -o run -- \
    python3 bench.py --workload c4 --rows 125000000 --steps 3 --warmup 1 --no-cpu --no-verify > "$OUT/pass$i.log" 2>&1 \
    || { tail -20 "$OUT/pass$i.log"; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_summary.py "$OUT" --json "$OUT/kernels.json" > "$OUT/summary.txt"
python3 - "$OUT/kernels.json" "gpurun_out/$TAG/traffic_c4.json" <<'PY'
import json, sys
k = json.load(open(sys.argv[1]))
tot = sum(v["traffic_bytes"] for v in k.values())
json.dump({"workload": "C4 rows=125000000 columns=0..15", "rows": 125000000, "columns": list(range(16)),
           "traffic_bytes_per_launch": tot,
           "fetch_bytes_per_launch": sum(v["fetch_bytes"] for v in k.values()),
           "write_bytes_per_launch": sum(v["write_bytes"] for v in k.values()),
           "source": "tools/c4_traffic.sh: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py --workload c4 "
                     "--rows 125000000 --steps 3 --warmup 1 --no-verify; per-kernel averages per dispatch summed "
                     "(FETCH_SIZE doubled: MI355X_MICROARCH.md gfx950 correction)",
           "kernels": {n: {"traffic_bytes": v["traffic_bytes"], "fetch_bytes": v["fetch_bytes"],
                           "write_bytes": v["write_bytes"]} for n, v in k.items()}},
          open(sys.argv[2], "w"), indent=1)
print(f"C4 traffic per launch: {tot / 1e9:.2f} GB")
PY
