set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
tools/gpu_run.sh testall || exit $?
echo "== ab cfg2 mark"; tools/ab.sh "base nomark r5" "cfg2" 3 || exit $?
