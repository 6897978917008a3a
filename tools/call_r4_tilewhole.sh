#!/bin/bash
# Round 4: the tile kernel with a loop of its own for waves whose lanes all have the same chunk count (seal and open, no Poly1305 predicates before the last chunk)
# (c + 1 < the wave's smallest chunk count): the tile / digest / forged parity tests, then an interleaved
# A/B against the committed build on configs 4 and 5.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q -m gpu \
    -k "tile or digest or random or large_payload or reference or openssl or cfg5 or forged or past_2" \
    --timeout 300 --timeout-method thread > gpurun_out/r4_tilewhole_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r4_tilewhole_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab.sh "base head" "cfg4 cfg5" 3 --no-cold --forged 0 2>&1 | tee gpurun_out/r4_tilewhole_ab.txt
