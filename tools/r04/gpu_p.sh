#!/bin/bash
# Round-4 pass p: the copy pool's run ends on its task count (default) vs on
# every worker checking in (DIPS_POOL_WAIT=workers): parity of the per-frame
# call paths, then the per_frame_call leg alternated over 5 rounds.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04p}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_compact_io.py \
  tests/test_gpu_compat.py > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt; [ $rc -ne 0 ] && { tail -60 $O/pytest.txt; exit $rc; }
timeout -k 10 600 python -u tools/pfc_threads_ab.py --rounds 5 --calls 300 \
  --env-variants "DIPS_POOL_WAIT=tasks|DIPS_POOL_WAIT=workers" > $O/pool_wait_ab.jsonl 2> $O/ab.err; rc=$?
cut -c1-200 $O/pool_wait_ab.jsonl; exit $rc
