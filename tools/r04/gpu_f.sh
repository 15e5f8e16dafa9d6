#!/bin/bash
# Round-4 pass f: the per-frame call's GPU side in isolation (tools/zc_probe.hip).
cd "$(dirname "$0")/../.."
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 120 tools/zc_probe > $O/zc_probe.jsonl 2> $O/zc_probe.err; rc=$?
cat $O/zc_probe.jsonl; exit $rc
