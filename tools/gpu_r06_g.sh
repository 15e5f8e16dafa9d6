# round 6: the added sharded-call tests
set -o pipefail
cd /root/repo
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_alt_shard.py \
    "tests/test_gpu_shard.py::test_native_alt_sharded_over_host_transport" \
    "tests/test_gpu_shard.py::test_native_compat_sharded_over_host_transport" > $O/pytest.txt 2>&1
rc=$?; tail -5 $O/pytest.txt; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/pytest.txt | head -40; exit $rc; }
exit 0
