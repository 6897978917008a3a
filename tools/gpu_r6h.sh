# round 6: config 3 with the workgroup-wide phase A (tools/build/librg_wga.so, built from the working tree):
# parity of every flat/forged/digest test on it, then an interleaved A/B against the in-tree build and its
# per-wave phases (diag build of the same source)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "== parity on wga"; RG_AEAD_LIB=tools/build/librg_wga.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wga_parity.log 2>&1 || { tail -40 gpurun_out/wga_parity.log; exit 1; }
tail -3 gpurun_out/wga_parity.log
echo "== ab cfg3"; tools/ab.sh "base wga" "cfg3" 3 || exit $?
echo "== stamps wga"; RG_AEAD_LIB=tools/build/librg_wgadiag.so timeout -k 10 300 python tools/flat_stamps.py --per-wave > gpurun_out/flat_stamps_wga.txt 2>&1 || exit $?
head -c 2500 gpurun_out/flat_stamps_wga.txt
