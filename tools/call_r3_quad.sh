# round 3: quad-transposed block stores (no LDS ring) in the pipelined kernel's uniform waves: parity + forged tests,
# then interleaved A/B against the LDS-ring build (ring = -DRG_PIPE_QUAD=0) and per-wave cycles
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_gpu_forged.py tests/test_gpu_parity.py tests/test_gpu_sessions.py tests/test_gpu_sessions_dev.py -x -q --timeout 120 --timeout-method thread > gpurun_out/quad_tests.log 2>&1
rc=$?; tail -3 gpurun_out/quad_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab.sh "ring base" cfg2 3 --no-cold --forged 0 || exit $?
for v in ring base; do
  if [ $v = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
  timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 > gpurun_out/q_st_$v.json 2>&1 || exit $?
  echo "== $v $(python3 -c "import json; t=open('gpurun_out/q_st_$v.json').read(); d=json.loads(t[t.index('{'):]); print(d['seal']['cycles_per_wave_mean'], d['seal']['end_us_pct_0_50_90_100'], d['open']['cycles_per_wave_mean'], d['open']['end_us_pct_0_50_90_100'])")"
done
