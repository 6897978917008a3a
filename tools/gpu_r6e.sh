# round 6 profile set, part 1: shard attribution with the waves' clock, default bench line + its rocprofv3
# kernel stats, per-config kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== shard_attrib"; RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 300 python tools/shard_attrib.py 1 2 4 8 > gpurun_out/shard_attrib.jsonl 2> gpurun_out/shard_attrib.err || exit $?
cat gpurun_out/shard_attrib.jsonl
G="bash tools/gpu_run.sh"
$G default defprof || exit $?
for W in cfg2 cfg3 cfg4; do RG_WORKLOAD=$W $G prof || exit $?; done
echo "== shard_probe levers (world 8 / 1)"
for v in "" "RG_PROBE_SEGMENTS=2" "RG_PROBE_STAGED=1"; do
    echo "-- ${v:-default}"; env $v timeout -k 10 300 python tools/shard_probe.py 8 1 || exit $?
done
