#!/bin/bash
# Final evidence for the committed library: stage a (tests, smoke, PMC,
# bench, rocprof) then stage b (sustained 100 steps, config sweep).
cd "$(dirname "$0")/../.."
bash tools/r04/gpu_final.sh a r04final5 && bash tools/r04/gpu_final.sh b r04final5_b
