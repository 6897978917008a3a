# round 3: where config 3's extra HBM bytes come from -- FETCH_SIZE / WRITE_SIZE of the flattened kernel
# in the in-tree build and in the no-payload-store / no-payload-load ablations (output invalid there)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/ft; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for v in ${VS:-base nostore noload}; do
  if [ $v = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/ft/${v}_$c -o p -- \
      python3 bench.py --workload ${W:-cfg3} --steps 5 --warmup 2 --cpu-seconds 0 --no-cold --forged 0 --no-graph > gpurun_out/ft/${v}_$c.log 2>&1
    rc=$?; [ $rc -gt 1 ] && exit $rc  # the ablations fail the bench's final open check (rc 1): counters are in
  done
done
python3 tools/pmc_summary.py gpurun_out/ft/* > gpurun_out/ft_summary.txt 2>&1 || true
