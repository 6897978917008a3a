#!/bin/bash
# Round 4: the default bench line exactly as the driver runs it (no flags; the host path now on by default).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
t0=$(date +%s)
timeout -k 10 400 python bench.py > gpurun_out/r4_default_noflags.jsonl 2> gpurun_out/r4_default_noflags.err
rc=$?
echo "wall $(( $(date +%s) - t0 )) s, rc $rc"
python3 -c "import json; d=json.loads(open('gpurun_out/r4_default_noflags.jsonl').read().strip().splitlines()[-1]); print(d['value'], d.get('e2e'))"
exit $rc
