set -e
# C4, two ranks sharing one GPU, default dispatch: every rank's launch times and re-run counters
O=gpurun_out/r06rh4; mkdir -p $O
export TMPDIR=/tmp
L="--nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 400 python3 -m torch.distributed.run $L --master-port 29551 bench.py --gpus 2 \
  --workload c4 --rows 40000000 --c4-templates 8 --steps 3 --warmup 1 --no-cpu --no-gather > $O/c4.json \
  2> $O/c4.err || { tail -30 $O/c4.err; exit 1; }
grep '"rank"' $O/c4.err
