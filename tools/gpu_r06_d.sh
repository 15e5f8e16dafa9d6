# round 6: the native sharded dips-compat call and the tests added since final_b
set -o pipefail
cd /root/repo
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_shard_native.py \
    tests/test_rust_contract.py tests/test_native_cli.py > $O/pytest.txt 2>&1
rc=$?; tail -5 $O/pytest.txt; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/pytest.txt | head -40; exit $rc; }
exit 0
