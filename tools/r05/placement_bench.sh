#!/bin/bash
# bench.py with the placement-aware allocation, four consecutive processes
# (where plain allocations alternate between a fast and a slow placement),
# then two with --no-placement-probe; after the placement unit test.  Each
# GPU step has its own time limit; the first failure ends the script.
cd "$(dirname "$0")/../.."
O=gpurun_out/${1:-placement_bench}
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_placement.py \
  > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-pcie --no-map --no-per-frame-call --no-legs --no-tau0"
for i in 1 2 3 4; do
  timeout -k 10 240 python3 bench.py $ARGS > $O/probe$i.json 2> $O/probe$i.log || { tail -5 $O/probe$i.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/probe$i.json')); print('probe', d['value'], d['roofline']['frac'], d['placement'])"
done
for i in 1 2; do
  timeout -k 10 240 python3 bench.py $ARGS --no-placement-probe > $O/plain$i.json 2> $O/plain$i.log || { tail -5 $O/plain$i.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/plain$i.json')); print('plain', d['value'], d['roofline']['frac'], d['placement'])"
done
