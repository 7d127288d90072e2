set -e
# C4, two ranks sharing one GPU: the same with the PLAIN BYTE_ARRAY one-pass path off (1=0), and with
# it and the fused dictionary launch off (1=0,4=0): which in-kernel wait makes the shared launches slow
O=gpurun_out/r06rh3; mkdir -p $O
export TMPDIR=/tmp
L="--nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
i=0
for D in "1=0" "1=0,4=0"; do
  i=$((i+1))
  PQGPU_DISPATCH=$D timeout -k 10 400 python3 -m torch.distributed.run $L --master-port 2954$i bench.py --gpus 2 \
    --workload c4 --rows 40000000 --c4-templates 8 --steps 3 --warmup 1 --no-cpu --no-gather > $O/c4_$i.json \
    2> $O/c4_$i.err || { tail -30 $O/c4_$i.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/c4_$i.json').read().strip().splitlines()[-1])
print('$D', d['ms_per_step'], d['rank0_launch_ms'], d['rank0_plan_reruns'])"
done
