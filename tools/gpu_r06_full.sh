# round 6: the whole GPU suite + smoke on one box (the driver's round-end tiers)
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r06full
timeout -k 10 1800 python -u -m pytest tests -m gpu -x -q --timeout 1200 --timeout-method thread \
    > gpurun_out/r06full/pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06full/smoke.txt 2>&1
