# round 6: dips_raw --ranks / alt
set -o pipefail
cd /root/repo
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_native_cli.py \
    > $O/pytest.txt 2>&1
rc=$?; tail -5 $O/pytest.txt; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/pytest.txt | head -40; exit $rc; }
exit 0
