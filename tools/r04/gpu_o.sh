#!/bin/bash
# Round-4 pass o: the series cleared by the RGB8 kernel (kzero) against a fill
# launch (fill), alternated in one process: 1080p 'overall' x 1000 frames
# (configs[1]), 640x480 x 300 and 4K 'per-frame' x 5000 (the headline).
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04o}
mkdir -p $O
timeout -k 10 200 python -u tools/isi_ab.py 1000 50 6 overall kzero,fill 1920x1080 > $O/kzero_1080p.jsonl 2> $O/ab.err || exit $?
timeout -k 10 200 python -u tools/isi_ab.py 300 200 6 overall kzero,fill 640x480 > $O/kzero_480p.jsonl 2>> $O/ab.err || exit $?
timeout -k 10 500 python -u tools/isi_ab.py 5000 10 6 per-frame kzero,fill > $O/kzero_4k.jsonl 2>> $O/ab.err || exit $?
tail -qn1 $O/kzero_*.jsonl | cut -c1-400
