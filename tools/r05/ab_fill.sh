#!/bin/bash
# A/B of the part-count rule: A = the tree's library (the fewest parts whose
# items fill >= 95 % of the resident wave slots), B = exp_fill/ (the best
# fill over the allowed part counts; 4K: 12 parts of 417 frames instead of
# 5 of 1,000, 8K: 3 of 417 instead of 2 of 625; exp_fill/ was a temporary copy
# of the tree with that rule, not kept), alternated on one box, the
# default 4K per-frame batch plus the configs[3] / configs[4] legs, each
# with the placement-aware allocation.
cd "$(dirname "$0")/../.."
O=gpurun_out/ab_fill
mkdir -p $O
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-pcie --no-map --no-per-frame-call --no-tau0"
i=0
for v in ${ORDER:-A B B A A B B A}; do
  i=$((i+1))
  case $v in A) d=. ;; B) d=exp_fill ;; esac
  (cd $d && timeout -k 10 240 python3 bench.py $ARGS) > $O/run${i}_$v.json 2> $O/run${i}_$v.log || exit $?
  python3 -c "import json;d=json.load(open('$O/run${i}_$v.json'));print('$v', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['roofline']['waves'], d['configs3']['frac'], d['configs4']['frac'], d['check']['equal'], d['placement'][0].get('candidate_kernel_ms'))"
done
