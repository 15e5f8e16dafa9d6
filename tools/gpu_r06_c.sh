# round 6: the host-pointer sharded path (streamed feed) -- its GPU tests and
# its rate at one rank against the streamed and staged calls
set -o pipefail
cd /root/repo
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 1200 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_shard_native.py \
    tests/test_gpu_shard.py tests/test_native_cli.py tests/test_rust_contract.py tests/test_gpu_series.py \
    tests/test_gpu_edges.py tests/test_gpu_bench_rehearsal.py > $O/pytest.txt 2>&1
rc=$?; tail -3 $O/pytest.txt; [ $rc -ne 0 ] && { tail -60 $O/pytest.txt; exit $rc; }
timeout -k 10 300 python -u tools/r06/sharded_host_rate.py > $O/sharded_host_rate.json 2> $O/sharded_host_rate.log
rc=$?; cat $O/sharded_host_rate.json; exit $rc
