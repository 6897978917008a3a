set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
PYTEST_K="failclosed or resources" tools/gpu_run.sh ktest || exit $?
echo "== l2tail"; timeout -k 10 120 tools/build/l2tail > gpurun_out/l2tail.json 2>&1 || exit $?
tail -3 gpurun_out/l2tail.json
echo "== ab cfg2"; tools/ab.sh "base r5 tailsc1 tailnt" "cfg2" 3 || exit $?
echo "== ab cfg4/5"; tools/ab.sh "base r5" "cfg4 cfg5" 2 || exit $?
