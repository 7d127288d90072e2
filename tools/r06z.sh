set -e
# (1) 4-byte DELTA at 5 waves per SIMD (occupancy hint): parity + A/B; (2) dictionary chunk size 8 / 16 / 32 tiles on C2;
# (3) C4 shard, HEAD vs this tree
O=gpurun_out/r06z; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_binary.py -k "delta or DELTA or dba or DBA or dlba or DLBA or optional" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for L in abx/libhead.so parquet-mr_amd/pqgpu/libpqgpu.so abx/libhead.so parquet-mr_amd/pqgpu/libpqgpu.so; do
  PQGPU_LIB=$PWD/$L timeout -k 10 600 python3 tools/bench_suite.py delta_i32 c3_delta str_dba --cpu-budget 0 > $O/s.jsonl 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
  python3 -c "
import json
for l in open('$O/s.jsonl'):
    d=json.loads(l); print('$L', d['workload'], round(d['ms_per_launch'],4), round(d.get('hbm_frac', 0) or 0, 3))"
done
for z in 1.5 2.0; do
for L in parquet-mr_amd/pqgpu/libpqgpu.so abx/libch32.so abx/libch8.so parquet-mr_amd/pqgpu/libpqgpu.so abx/libch32.so abx/libch8.so; do
  PQGPU_LIB=$PWD/$L timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-e2e --zipf $z > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$L zipf $z', round(d['ms_per_step'],4), round(d['roofline']['frac'],3))"
done
done
for L in abx/libhead.so parquet-mr_amd/pqgpu/libpqgpu.so; do
  PQGPU_LIB=$PWD/$L timeout -k 10 400 python3 bench.py --workload c4 --steps 10 --warmup 2 --no-cpu --no-e2e > $O/c4.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/c4.json').read().strip().splitlines()[-1]); print('$L c4', round(d['ms_per_step'],4), round(d['roofline']['frac'],3))"
done
