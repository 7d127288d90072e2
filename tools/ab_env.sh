#!/bin/bash
# A/B of launch settings on the C2 bench: bash tools/ab_env.sh <tag> "<label>:<ENV=V ...>:<lib or default>" ...
# Each run under its own time limit; stops at the first failure. Two rounds.
set -euo pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for rep in 1 2; do
  for spec in "$@"; do
    IFS=: read -r label envs lib <<< "$spec"
    if [ "$lib" = default ]; then unset PQGPU_LIB; else export PQGPU_LIB=$PWD/$lib; fi
    env $envs timeout -k 10 180 python -u bench.py --no-cpu --steps 50 ${AB_ARGS:-} > "$OUT/$label.$rep.json" 2> "$OUT/$label.$rep.err" \
      || { tail -20 "$OUT/$label.$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e9,1), 'G/s', round(d['ms_per_step']*1e3,1), 'us')" "$OUT/$label.$rep.json" "$label"
  done
done
