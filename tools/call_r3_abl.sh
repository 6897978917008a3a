# round 3, config 2: seal with the line stores dropped (abl1) / the LDS ring dropped (abl2) against the default build
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/ab.sh "base abl1 abl2" cfg2 2 --no-cold --no-verify || exit $?
for v in base abl1 abl2; do
  if [ $v = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
  timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 > gpurun_out/abl_st_$v.json 2>&1 || exit $?
  echo "== $v stamps"
  grep -A1 cycles_per_wave gpurun_out/abl_st_$v.json | head -2
done
