set -e
O=gpurun_out/r05ac; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_binary.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_c4prof.sh r05ac_p 15 abx/libblk.so default
bash tools/ab_suite_prof.sh r05ac_s "c3_strings" abx/libblk.so parquet-mr_amd/pqgpu/libpqgpu.so
for L in abx/libblk.so parquet-mr_amd/pqgpu/libpqgpu.so; do
PQGPU_LIB=$PWD/$L timeout -k 10 600 python3 bench.py --workload c4 --rows 125000000 --steps 10 --warmup 2 --no-cpu > $O/c4.json 2> $O/c4.err || { tail -30 $O/c4.err; exit 1; }
python3 -c "import json; print('C4 $L', json.load(open('$O/c4.json'))['ms_per_step'])"
done
