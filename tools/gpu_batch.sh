set -e
O=gpurun_out/r05r; mkdir -p $O
bash tools/ab_c4prof.sh r05r_dd 8,9,13,14 abx/libnb.so abx/libno.so abx/libnone.so
export TMPDIR=/tmp
PQGPU_LIB=$PWD/abx/liblw.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lw -o run -- python3 -u tools/bench_suite.py c3_mixed --cpu-budget 0 --steps 5 --warmup 1 --no-verify > $O/lw.jsonl 2> $O/lw.err || { tail -20 $O/lw.err; exit 1; }
python3 tools/kstats.py $O/lw | head -8
