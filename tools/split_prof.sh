set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r05j
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05j/dd_split -o run -- python3 bench.py --workload c4 --rows 125000000 --steps 5 --warmup 1 --no-cpu --c4-cols 8,9,13,14 --dict-split > gpurun_out/r05j/dd_split.json 2> gpurun_out/r05j/dd_split.err
echo "== dd split"; python3 tools/kstats.py gpurun_out/r05j/dd_split
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05j/c2_split -o run -- python3 bench.py --no-cpu --steps 10 --dict-split > gpurun_out/r05j/c2_split.json 2> gpurun_out/r05j/c2_split.err
echo "== c2 split"; python3 tools/kstats.py gpurun_out/r05j/c2_split
