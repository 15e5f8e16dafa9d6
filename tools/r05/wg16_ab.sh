#!/bin/bash
# The part-major series schedule in 256- and 1024-thread workgroups
# (build/alloc_policy_ab, L = 1000 vs 1000x), alternated over four
# rounds on two 124 GB buffers of one process; then the address-translation
# counters of both.  Each GPU step has its own time limit.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-wg16}
mkdir -p $O
timeout -k 10 200 build/alloc_policy_ab 5000 2 4 default,default 1000,1000x 4050 > $O/ab.txt 2> $O/ab.err || exit $?
cat $O/ab.txt
timeout -s KILL 150 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_LFIFO_FULL_sum TCP_UTCL1_STALL_LFIFO_NO_RES_sum \
  --output-format csv -d $O/p1 -o run -- build/alloc_policy_ab 5000 0.25 1 default,default 1000,1000x 4050 > $O/p1.txt 2> $O/p1.err \
  || { echo "pmc rc=$?"; tail -5 $O/p1.err; exit 1; }
echo pmc ok
