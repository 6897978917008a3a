set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 bash tools/ab.sh "base nolines nocur" "cfg2" 3 --no-cold || exit $?
for v in base nolines; do
  if [ $v = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcf_$v -o p -- python3 bench.py --workload cfg2 --steps 5 --warmup 2 --cpu-seconds 0 --no-cold > gpurun_out/pmcf_$v.log 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcw_$v -o p -- python3 bench.py --workload cfg2 --steps 5 --warmup 2 --cpu-seconds 0 --no-cold > gpurun_out/pmcw_$v.log 2>&1 || exit $?
done
echo done
