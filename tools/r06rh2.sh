set -e
# C4 with two ranks sharing one GPU: per-launch times and the plans' re-run counters (diagnosis of the
# 16 s launches seen in tools/r06rh.sh)
O=gpurun_out/r06rh2; mkdir -p $O
export TMPDIR=/tmp
L="--nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 600 python3 -m torch.distributed.run $L --master-port 29533 bench.py --gpus 2 --workload c4 \
  --rows 40000000 --c4-templates 8 --steps 3 --warmup 1 --no-cpu --no-gather > $O/c4_g2.json 2> $O/c4_g2.err \
  || { tail -30 $O/c4_g2.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c4_g2.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['timer'], d['wall_ms_per_step'], d['rank0_launch_ms'], d['rank0_plan_reruns'])"
