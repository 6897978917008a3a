# round 3: config-2 step cycles of the pipelined kernel by unrolled position, and the time in an exact vmcnt(16) wait
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
RG_AEAD_LIB=tools/build/librg_wst.so timeout -k 10 120 python tools/wstamps.py > gpurun_out/wst.json 2>gpurun_out/wst.err || exit $?
cat gpurun_out/wst.json
RG_AEAD_LIB=tools/build/librg_wst.so timeout -k 10 120 python tools/wstamps.py --mode 7 > gpurun_out/wst_m7.json 2>&1 || exit $?
echo "== m7"; cat gpurun_out/wst_m7.json
