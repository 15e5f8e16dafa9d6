#!/bin/bash
# Address-translation counters of the series kernel on the first and the
# second 124 GB frame buffer of one process (build/alloc_policy_ab: buffer
# default#0 runs ~3 points faster than default#1).  One --pmc pass per
# counter group, each under its own time limit; the first failure ends it.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-tlb}
mkdir -p $O
ARGS="5000 0.25 1 default,default 1000 4050"
timeout -k 10 120 build/alloc_policy_ab $ARGS > $O/plain.txt 2> $O/plain.err || exit $?
cat $O/plain.txt
i=0
for grp in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum" \
           "TCP_UTCL1_STALL_LFIFO_NO_RES_sum TCP_UTCL1_LFIFO_FULL_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum" \
           "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- build/alloc_policy_ab $ARGS \
    > $O/p$i.txt 2> $O/p$i.err || { echo "pass $i rc=$?"; tail -5 $O/p$i.err; exit 1; }
  echo "pass $i ok"
done
exit 0
