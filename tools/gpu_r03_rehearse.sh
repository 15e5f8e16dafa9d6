#!/bin/bash
# bench.py's N > 1 path on one GPU over gloo (rehearsal; RCCL needs one GPU
# per rank): 2 and 4 ranks, both modes, each line saved.
set -o pipefail
O=gpurun_out/${1:-rehearse}
mkdir -p $O
export DIPS_BENCH_BACKEND=gloo DIPS_BENCH_ONE_DEVICE=1
port=29533
for n in 2 4; do
  for mode in per-frame overall; do
    port=$((port+1))
    timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus $n --steps 3 --warmup 1 --frames-per-gpu 200 --mode $mode \
      --no-cpu-baseline --no-pcie --no-map --no-per-frame-call > $O/bench_${n}ranks_${mode}.json 2> $O/bench_${n}ranks_${mode}.log
    rc=$?; echo "n=$n mode=$mode rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/bench_${n}ranks_${mode}.log; exit $rc; }
  done
done
for f in $O/bench_*ranks_*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', d['n_gpus'], d['config']['parallelism'], d['check'], {k: (d[k].get('check') or {}).get('equal') for k in ('configs3','configs4')})"; done
