# round 6: config 2's per-wave stamps on the round-6 build (diag), normal seal (mode 3) and compute only (mode 1)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for m in 3 1; do
    echo "== stamps mode $m"; RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 300 python tools/stamps.py --workload cfg2 --mode $m > gpurun_out/stamps_cfg2_m$m.txt 2>&1 || exit $?
    grep -v amdgpu.ids gpurun_out/stamps_cfg2_m$m.txt | head -c 1500
done
