# round 3, config 2: line stores spread over the keystream rounds (compiler-visible buffer stores) and lane-per-frame
# stores without the ring (nolines) against the default build; interleaved A/B + per-wave cycles
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/ab.sh "base spread nolines" cfg2 3 --no-cold --forged 0 || exit $?
for v in base spread nolines; do
  if [ $v = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
  timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 > gpurun_out/sp_st_$v.json 2>&1 || exit $?
  echo "== $v $(python3 -c "import json; t=open('gpurun_out/sp_st_$v.json').read(); d=json.loads(t[t.index('{'):]); print(d['seal']['cycles_per_wave_mean'], d['seal']['end_us_pct_0_50_90_100'], d['open']['cycles_per_wave_mean'])")"
done
