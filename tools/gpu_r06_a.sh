# round 6: the native sharding's multi-process / bench tests, then the wave
# reserve A/B of the headline kernel (3 vs 4 waves per SIMD)
set -o pipefail
cd /root/repo
timeout -k 10 1500 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_shard.py \
    tests/test_native_cli.py tests/test_gpu_placement.py tests/test_gpu_bench_contract.py \
    tests/test_gpu_bench_rehearsal.py > gpurun_out/r06_tests_a.txt 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
B="--steps 10 --warmup 2 --no-legs --no-cpu-baseline --no-per-frame-call --no-map --no-tau0 --no-pcie --no-check --no-placement-probe"
timeout -k 10 300 python bench.py $B > gpurun_out/b_default.json 2> gpurun_out/b_default.log && \
DIPS_SERIES_WAVES_PER_SIMD=3 timeout -k 10 300 python bench.py $B > gpurun_out/b_w3.json 2> gpurun_out/b_w3.log && \
timeout -k 10 300 python bench.py $B > gpurun_out/b_default2.json 2> gpurun_out/b_default2.log && \
DIPS_SERIES_WAVES_PER_SIMD=3 timeout -k 10 300 python bench.py $B > gpurun_out/b_w3_2.json 2> gpurun_out/b_w3_2.log
