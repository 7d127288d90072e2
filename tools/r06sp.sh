set -e
# Split-mode (walk kernel, then expansion kernel) per-kernel times for Zipf 1.5 and 2.0
O=gpurun_out/r06sp; mkdir -p $O
export TMPDIR=/tmp
for z in 1.5 2.0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/z$z -o run -- \
    python3 bench.py --no-cpu --no-e2e --dict-split --zipf $z --steps 10 --warmup 2 > $O/z$z.json 2> $O/z$z.err || { tail -20 $O/z$z.err; exit 1; }
  echo "zipf $z"; python3 tools/kstats.py $O/z$z | grep -v fill
done
