#!/bin/bash
# A/B/C of the RGB8 series kernel: A = the tree's library (U = 4 vecs per
# lane), B = exp_u5/ (U = 5), C = exp_c/ (U = 5 + the record's H / L split
# through the carry), alternated on one box (the order below cancels a
# linear drift), the default 4K per-frame batch, 10 timed steps each.
cd "$(dirname "$0")/../.."
O=gpurun_out/ab_u5
mkdir -p $O
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-pcie --no-map --no-per-frame-call --no-legs --no-tau0"
i=0
for v in ${ORDER:-A B C C B A A B C C B A}; do
  i=$((i+1))
  case $v in A) d=. ;; B) d=exp_u5 ;; C) d=exp_c ;; esac
  (cd $d && timeout -k 10 240 python3 bench.py $ARGS) > $O/run${i}_$v.json 2> $O/run${i}_$v.log || exit $?
  python3 -c "import json;d=json.load(open('$O/run${i}_$v.json'));print('$v', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], (d.get('power') or {}).get('ppt_throttle_residency'), d['check']['equal'])"
done
