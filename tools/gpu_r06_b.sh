# round 6: halo / series contention at world size 1 (tools/r06/halo_contention.py)
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r06
F=2000 timeout -k 10 400 python -u tools/r06/halo_contention.py > gpurun_out/r06/halo_contention.jsonl 2> gpurun_out/r06/halo_contention.log && \
F=5000 REPS=5 timeout -k 10 400 python -u tools/r06/halo_contention.py > gpurun_out/r06/halo_contention_5000.jsonl 2> gpurun_out/r06/halo_contention_5000.log
