# round 6: shard attribution with per-item stamps, NUMA e2e, config 3 phase stamps, stream-mark A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "== shard_attrib"; RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 300 python tools/shard_attrib.py 1 8 > gpurun_out/shard_attrib.jsonl 2> gpurun_out/shard_attrib.err || exit $?
cat gpurun_out/shard_attrib.jsonl
echo "== numa_e2e"; timeout -k 10 300 python tools/numa_e2e.py > gpurun_out/numa_e2e.json 2> gpurun_out/numa_e2e.err || exit $?
cat gpurun_out/numa_e2e.json; ls /sys/devices/system/node/; cat /sys/fs/cgroup/cpuset.mems.effective 2>/dev/null; echo
echo "== flat stamps"; RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 300 python tools/flat_stamps.py --per-wave > gpurun_out/flat_stamps.txt 2>&1 || exit $?
head -c 3000 gpurun_out/flat_stamps.txt
echo "== ab cfg2 mark"; tools/ab.sh "base nomark" "cfg2" 4 || exit $?
