set -e
# Two-rank rehearsal of the multi-GPU bench path on a one-GPU box: two processes share cuda:0 (gloo
# collectives, bench.py's fewer-GPUs-than-ranks branch); the per-rank time is not a scaling number,
# the run checks the shard / gather / verify path of the current tree end to end.
O=gpurun_out/r06rh; mkdir -p $O
export TMPDIR=/tmp
L="--nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 600 python3 -m torch.distributed.run $L --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 \
  > $O/bench_g2.json 2> $O/bench_g2.err || { tail -30 $O/bench_g2.err; exit 1; }
tail -c 400 $O/bench_g2.json
timeout -k 10 900 python3 -m torch.distributed.run $L --master-port 29532 bench.py --gpus 2 --workload c4 \
  --rows 40000000 --c4-templates 8 --steps 5 --warmup 2 --no-cpu > $O/bench_c4_g2.json 2> $O/bench_c4_g2.err \
  || { tail -30 $O/bench_c4_g2.err; exit 1; }
tail -c 400 $O/bench_c4_g2.json
