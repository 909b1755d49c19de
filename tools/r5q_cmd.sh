set -o pipefail
cd $GRAFT_REPO_ROOT 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5t; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/t_all.log 2>&1
grep -E "passed|failed|FAILED" $O/t_all.log | tail -30
